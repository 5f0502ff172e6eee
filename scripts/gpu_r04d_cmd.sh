# C3 kernel trace (where the 0.133 ms step goes) and the adversarial fallback at full C4 size
set -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
PASSES=trace bash scripts/profile.sh r04d_c3 --config C3 --steps 30 --warmup 5 --no-parity-sample --em-iters 0 --no-shard-sim || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_r04d_c3 $OUT/summary_c3 > $OUT/summary_c3.txt 2>&1; head -14 $OUT/summary_c3.txt
timeout -k 10 300 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err; rc=$?; cat $OUT/fold.json; tail -3 $OUT/fold.err; exit $rc

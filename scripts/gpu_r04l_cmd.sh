# fb_exact_kernel in 8-wave blocks (tree) vs 4-wave (x256): fallback tests, C3 / C4 A/B,
# the adversarial case
set -o pipefail
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "fallback or exact" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/x256.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/x256.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold.json

# the statistics kernel without the folded fallback (the gate-list pass's flags get an
# fb_exact_kernel launch from flag_count[3]), K1 W' / bias' staged in LDS in
# fb_bwd2_kernel: fallback / K1 / gated tests, A/B against the previous commit,
# the adversarial case
set -o pipefail
OUT=gpurun_out/r04k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "k1 or fallback or exact or C3 or c3 or diag or S5 or fused or gated or C4 or c4" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
PARITY=1 timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/head.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold.json

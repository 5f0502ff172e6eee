# the gate-list pass's exact fallback inside fb_split_kernel's list mode (4 <= S <= 6:
# no fb_exact_kernel launch after it): fallback / gated / C3 tests, C3 and C4 A/B
# against the previous commit (head), the adversarial case
set -o pipefail
OUT=gpurun_out/r04m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "k1 or fallback or exact or C3 or c3 or diag or S5 or S4 or fused or gated" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
PARITY=1 timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/head.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold.json

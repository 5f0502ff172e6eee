# tree = list-pass fallback folded into stats_list_m_kernel + short K1 inside
# fb_bwd2_kernel / the list pass (C3); A/B against the previous commit (head), the
# gate-list fallback as an fb_exact_kernel launch (nofl, built before the K1 change),
# emission_u_kernel in 12-wave (em12) / 8-wave (em8) blocks; GPU tests on the tree
set -o pipefail
OUT=gpurun_out/r04j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "k1 or fallback or exact or C3 or c3 or diag or S5 or fused or gated" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 bash scripts/ab_lib.sh build/ab/head.so build/ab/nofl.so build/ab/em12.so build/ab/em8.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
PARITY=1 timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/head.so build/ab/nofl.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
timeout -k 10 600 bash scripts/ab_lib.sh --args "--N 12500 --steps 40 --warmup 5" build/ab/head.so build/ab/em12.so > $OUT/ab_12k.txt 2>&1; cat $OUT/ab_12k.txt
export VBHEM_LIB_PATH=$(realpath build/ab/nofl.so)
timeout -k 10 900 python -u -m pytest tests -v -m gpu -k "fallback or exact" --timeout 300 --timeout-method thread > $OUT/tests_nofl.log 2>&1 || { tail -40 $OUT/tests_nofl.log; exit 1; }
tail -2 $OUT/tests_nofl.log
timeout -k 10 600 python -u scripts/fold_bench.py 100000 > $OUT/fold_nofl.json 2> $OUT/fold.err || { tail -20 $OUT/fold.err; exit 1; }
cat $OUT/fold_nofl.json

# A/B: fb_list4_kernel with the round-4 backward step (C4), the split kernel at 4 lanes
# per column for S = 5 (C3), plus the C3-shape parity tests on that variant
set -o pipefail
OUT=gpurun_out/r04e; mkdir -p $OUT
PARITY=1 timeout -k 10 900 bash scripts/ab_lib.sh build/ab/l4r4.so > $OUT/ab_c4.txt 2>&1; cat $OUT/ab_c4.txt
PARITY=1 timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/lpc5.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt
VBHEM_LIB_PATH=$(realpath build/ab/lpc5.so) timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "C3 or diag or S5 or odd or c3" --timeout 300 --timeout-method thread > $OUT/tests_lpc5.log 2>&1; tail -2 $OUT/tests_lpc5.log
VBHEM_LIB_PATH=$(realpath build/ab/l4r4.so) timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "S8 or C4 or c4 or mfma or list4" --timeout 300 --timeout-method thread > $OUT/tests_l4r4.log 2>&1; tail -2 $OUT/tests_l4r4.log
exit 0

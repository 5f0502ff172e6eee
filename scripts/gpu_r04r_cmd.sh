# fb_bwd2_kernel<5> with 3 base-state columns per lane (cpl3: 32 pairs per wave, C3's
# 80,000 pairs in one round of 3,072 waves instead of 1.24 rounds of 21-pair waves)
set -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
VBHEM_LIB_PATH=$(realpath build/ab/cpl3.so) timeout -k 10 900 python -u -m pytest tests -q -m gpu -k "C3 or c3 or S5 or diag or fused or gated or fallback or pairs" --timeout 300 --timeout-method thread > $OUT/tests_cpl3.log 2>&1 || { tail -40 $OUT/tests_cpl3.log; exit 1; }
tail -2 $OUT/tests_cpl3.log
PARITY=1 timeout -k 10 600 bash scripts/ab_lib.sh --args "--config C3 --steps 60 --warmup 5" build/ab/cpl3.so > $OUT/ab_c3.txt 2>&1; cat $OUT/ab_c3.txt

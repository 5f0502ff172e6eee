# fb_split_kernel list mode at S = 11, 12 with A' read from LDS instead of registers
# (atl: 236 VGPRs, no scratch; tree: 256 VGPRs + 124 B of spills at S = 12): C5 A/B
set -o pipefail
OUT=gpurun_out/r04q; mkdir -p $OUT
timeout -k 10 1000 bash scripts/ab_lib.sh --args "--config C5 --steps 4 --warmup 1" build/ab/atl.so > $OUT/ab_c5.txt 2>&1; cat $OUT/ab_c5.txt
VBHEM_LIB_PATH=$(realpath build/ab/atl.so) timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "S12 or C5 or c5" --timeout 300 --timeout-method thread > $OUT/tests_atl.log 2>&1; tail -2 $OUT/tests_atl.log

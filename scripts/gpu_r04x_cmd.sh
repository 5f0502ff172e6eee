# fb_bwd2_kernel<S <= 5> at 4 waves per SIMD (16-wave blocks: C3's 3,816 tiles in one
# round of 4,096 slots instead of 1.24 rounds of 3,072) with unpadded slab columns (LDS)
set -o pipefail
OUT=gpurun_out/r04x; mkdir -p $OUT
VBHEM_LIB_PATH=$(realpath build/ab/w4p0.so) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "bwd2_in_kernel_prep or k1_in_recursion or fused_match or exact_fallback_gated" > $OUT/targeted.log 2>&1 || { tail -30 $OUT/targeted.log; exit 1; }
tail -1 $OUT/targeted.log
bash scripts/ab_lib.sh --args "--config C3 --steps 20 --warmup 3" build/ab/w4p0.so build/ab/w3p0.so

#!/bin/bash
# round 6: K1 inside fb_bwd4_kernel (VBHEM_K1_BWD4=1, experiment): the S = 8 parity tests
# with it on, then the C4 A/B (bwd kernel time; the emission GEMM still runs for the list
# pass).  scripts/gpu_step10.sh TAG
set -o pipefail
TAG=${1:-r06u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VBHEM_K1_BWD4=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "S8 or s8 or C4 or c4 or bwd4 or exact_fallback or range_check or prepared or golden" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
PARITY=1 bash scripts/ab_env.sh --args "--steps 40 --warmup 5" "VBHEM_K1_BWD4=1" > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt

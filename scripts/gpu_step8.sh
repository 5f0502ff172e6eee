#!/bin/bash
# round 6: bwd2 at 4 waves per SIMD for S <= 5 (C3 in one round of wave tiles):
# the bwd2 / C3 tests, then C3 A/B against the 12-wave build.  scripts/gpu_step8.sh TAG
set -o pipefail
TAG=${1:-r06r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "bwd2 or C3 or c3 or split or fused or exact_fallback or golden or face" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh --args "--config C3 --steps 200 --warmup 5" build/ab/libB12.so > $OUT/ab_c3.txt 2>&1 || { cat $OUT/ab_c3.txt; exit 1; }
cat $OUT/ab_c3.txt

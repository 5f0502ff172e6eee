#!/bin/bash
# round 6: gate_list_kernel with 32 chunk counts in flight per thread -- gated tests, then
# A/B against the previous build at C4 and the 12,500-base shard.  scripts/gpu_step14.sh TAG LIB
set -o pipefail
TAG=${1:-r06y}; LIB=${2:-build/ab/libGL8.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "gated or fused or golden or C4 or c4 or trials" > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh --args "--steps 40 --warmup 5" $LIB > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
bash scripts/ab_lib.sh --args "--N 12500 --steps 200 --warmup 5" $LIB > $OUT/ab_shard.txt 2>&1 || { cat $OUT/ab_shard.txt; exit 1; }
cat $OUT/ab_shard.txt

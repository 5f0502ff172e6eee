#!/bin/bash
# round 6: emission_db_kernel at two waves per SIMD (amdgpu_waves_per_eu(2): 230 VGPRs, no
# AGPRs, against 232 + 32 = one wave per SIMD) -- C5 bit-identity and A/B.
set -o pipefail
TAG=${1:-r06w}; LIB=${2:-build/ab/libW2.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VBHEM_LIB_PATH=$(pwd)/$LIB timeout -k 10 300 python -u -m pytest tests/test_emission_db.py -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" $LIB > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt

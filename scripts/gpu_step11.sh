#!/bin/bash
# round 6: emission_db_kernel<38,2,1,512> (VBHEM_EM_DB1=1: one tile per wave, 8-wave
# blocks, 4 waves per SIMD) -- bit-identity vs the single-buffer path, then C5 A/B.
set -o pipefail
TAG=${1:-r06v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VBHEM_EM_DB1=1 timeout -k 10 300 python -u -m pytest tests/test_emission_db.py -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1
rc=$?; tail -2 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_env.sh --args "--config C5 --steps 3 --warmup 1" "VBHEM_EM_DB1=1" > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt

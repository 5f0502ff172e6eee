#!/bin/bash
# round 6: non-temporal E stores (VBHEM_EM_STORE_AUX=2) A/B on C4 and C5.  scripts/gpu_step9.sh TAG LIB
set -o pipefail
TAG=${1:-r06t}; LIB=${2:-build/ab/libNT.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/ab_lib.sh --args "--steps 40 --warmup 5" $LIB > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" $LIB > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt

#!/bin/bash
# round 6: fb_bwd4_kernel compiled with other LLVM scheduling strategies, C4 A/B.
set -o pipefail
TAG=${1:-r06ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/ab_lib.sh --args "--steps 40 --warmup 5" build/ab/lib_max-ilp.so build/ab/lib_iterative-ilp.so > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt

#!/bin/bash
# round 6: C5 base groups of 12 GB of per-pair buffers (9 groups of 113 k bases, every
# 32-bit-offset kernel version still applies) against 8 GB (14 groups).
set -o pipefail
TAG=${1:-r06x}; LIB=${2:-build/ab/libG12.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" $LIB > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt

#!/bin/bash
# Same-box A/B of library builds with more timed launches than ab_lib.sh's default, plus
# the VALU microbenchmark:  scripts/gpu_ab.sh TAG "bench args" lib1.so lib2.so ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -x build/ubench_valu ]; then timeout -k 10 120 ./build/ubench_valu > $OUT/ubench_valu.txt 2>&1 || exit 1; head -40 $OUT/ubench_valu.txt | grep -v "^ " ; fi
bash scripts/ab_lib.sh --args "$ARGS" "$@" > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc

#!/bin/bash
# Bitwise A/B of the tree's library against build/ab/libold.so, the two-rank test on
# both, the GPU suite (no -x) and the C4 / C5 bench A/B.  scripts/gpu_step2.sh TAG
set -o pipefail
TAG=${1:-r06b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/new.npz > $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
VBHEM_LIB_PATH=$(pwd)/build/ab/libold.so timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/old.npz >> $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
python scripts/cmp_libs.py diff $OUT/new.npz $OUT/old.npz | tee -a $OUT/cmp.txt
VBHEM_LIB_PATH=$(pwd)/build/ab/libold.so timeout -k 10 300 python -u -m pytest tests/test_dist_native.py -q --timeout 200 --timeout-method thread > $OUT/dist_old.log 2>&1; tail -2 $OUT/dist_old.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -8 $OUT/tests.log; [ $rc -gt 1 ] && exit $rc
bash scripts/ab_lib.sh build/ab/libold.so > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
PARITY=1 bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" build/ab/libold.so > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt
exit 0

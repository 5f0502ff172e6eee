#!/bin/bash
# C5 emission A/B (double-buffered chunks vs VBHEM_EM_NODB), bitwise comparison of the
# two, and the GPU suite.   scripts/gpu_step3.sh TAG
set -o pipefail
TAG=${1:-r06f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/db.npz > $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
VBHEM_EM_NODB=1 timeout -k 10 300 python scripts/cmp_libs.py dump $OUT/nodb.npz >> $OUT/cmp.txt 2>&1 || { tail $OUT/cmp.txt; exit 1; }
python scripts/cmp_libs.py diff $OUT/db.npz $OUT/nodb.npz | tee -a $OUT/cmp.txt | grep C5
PARITY=1 bash scripts/ab_env.sh --args "--config C5 --steps 3 --warmup 1" "VBHEM_EM_NODB=1" > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log; exit $rc

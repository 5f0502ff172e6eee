#!/bin/bash
# One GPU call: the co-execution microbenchmark (+ its PMC pass), the GPU suite, and a
# same-box A/B of the tree's library against build/ab/libold.so at C4 and C5.
#   scripts/gpu_step1.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-r06a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ROOT=$(pwd)
timeout -k 10 120 ./build/ubench_coexec > $OUT/coexec.txt 2>&1 || { cat $OUT/coexec.txt; exit 1; }
cat $OUT/coexec.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F64 -d $ROOT/$OUT/coexec_pmc -o pmc --output-format csv -- $ROOT/build/ubench_coexec > $ROOT/$OUT/coexec_pmc.log 2>&1) || { tail -5 $OUT/coexec_pmc.log; exit 1; }
echo coexec pmc ok
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_lib.sh build/ab/libold.so > $OUT/ab_c4.txt 2>&1 || { cat $OUT/ab_c4.txt; exit 1; }
cat $OUT/ab_c4.txt
PARITY=1 bash scripts/ab_lib.sh --args "--config C5 --steps 3 --warmup 1" build/ab/libold.so > $OUT/ab_c5.txt 2>&1 || { cat $OUT/ab_c5.txt; exit 1; }
cat $OUT/ab_c5.txt
exit 0

#!/bin/bash
# EM-loop check: MFMA layout probe, the EM tests, a kernel trace of one C4 shard run.
set -o pipefail
OUT=gpurun_out/em; mkdir -p $OUT
timeout -k 10 60 ./scripts/mfma_layout.bin > $OUT/mfma_layout.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_native_em.py tests/test_dist_native.py tests/test_vbhmm_em.py \
  -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o em -- \
  python3 $GRAFT_REPO_ROOT/scripts/em_probe.py 12500 20 > $GRAFT_REPO_ROOT/$OUT/probe.log 2>&1
rc=$?; tail -3 $GRAFT_REPO_ROOT/$OUT/probe.log; exit $rc

#!/bin/bash
# GPU check: selected -m gpu tests, then a kernel trace of one bench run (profile.sh, trace pass).
# Usage: scripts/gpu_tt.sh TAG "test paths" [bench args...]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $TESTS -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
PASSES=trace bash scripts/profile.sh $TAG "$@"

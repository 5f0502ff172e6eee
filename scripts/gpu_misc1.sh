#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist_native.py -x -v --timeout 240 --timeout-method thread > gpurun_out/dist_native.log 2>&1; rc=$?
tail -5 gpurun_out/dist_native.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/host_overhead.py 12500 && timeout -k 10 120 python scripts/host_overhead.py 100000

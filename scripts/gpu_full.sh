#!/bin/bash
# Round check: every -m gpu test, then the default bench line (C4).
set -o pipefail
TAG=${1:-full}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; tail -c 600 gpurun_out/$TAG/bench.json; exit $rc

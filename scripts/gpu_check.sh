#!/bin/bash
# GPU check used during development: selected -m gpu tests, then one bench line.
# Usage: scripts/gpu_check.sh TAG "pytest -k expression or test paths" [bench args...]
set -o pipefail
TAG=${1:-chk}; TESTS=${2:-tests}; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -5 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -c 3000 $OUT/bench.json; exit $rc

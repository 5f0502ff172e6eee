#!/bin/bash
# Round-end evidence on one box: every -m gpu test, then the bench lines for C4 (default),
# C3 and C5.  Outputs under gpurun_out/TAG/.   scripts/gpu_final.sh TAG [NOTEST=1]
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$NOTEST" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in C4 C3 C5; do
  timeout -k 10 400 python -u bench.py --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err
  rc=$?; tail -c 300 $OUT/bench_$cfg.json; echo; [ $rc -ne 0 ] && exit $rc
done
exit 0

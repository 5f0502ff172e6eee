#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line (C4), then the kernel trace +
# 4 PMC passes of the same bench (scripts/profile.sh).  Outputs under gpurun_out/TAG/
# and gpurun_out/prof_TAG/.   scripts/gpu_round.sh TAG   (NOTEST=1, NOPROF=1, CONFIGS="C4 C3 C5")
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$NOTEST" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in ${CONFIGS:-C4}; do
  timeout -k 10 400 python -u bench.py --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err
  rc=$?; tail -c 400 $OUT/bench_$cfg.json; echo; [ $rc -ne 0 ] && exit $rc
done
[ "$NOPROF" = 1 ] && exit 0
bash scripts/profile.sh $TAG --steps 20 --warmup 5 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_$TAG $OUT/summary_c4 > $OUT/summary.txt 2>&1
cat $OUT/summary.txt | head -30
exit 0

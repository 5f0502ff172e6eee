#!/bin/bash
# Round-end evidence on one box, outputs under gpurun_out/TAG/ (and prof_TAG*):
#   the -m gpu suite and smoke(); bench lines for C4 (default), C3, C5; the C4 kernel
#   trace + 4 PMC passes (scripts/profile.sh) and kernel traces of C3 and C5.
#   scripts/gpu_final.sh TAG        (NOTEST=1: skip the suite; NOBENCH=1: skip the bench
#                                    lines; NOPROF=1: skip profiles; SHARD=1: also the
#                                    12,500-base kernel trace)
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$NOTEST" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; [ $rc -gt 1 ] && exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
  tail -1 $OUT/smoke.log
fi
for cfg in C4 C3 C5; do
  [ "$NOBENCH" = 1 ] && break
  timeout -k 10 600 python -u bench.py --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err
  rc=$?; tail -c 300 $OUT/bench_$cfg.json; echo; [ $rc -ne 0 ] && exit $rc
done
shard() {
  PASSES=trace bash scripts/profile.sh ${TAG}_shard --N 12500 --steps 20 --warmup 5 --no-parity-sample --em-iters 0 || exit $?
  python3 scripts/prof_summary.py gpurun_out/prof_${TAG}_shard $OUT/summary_shard > $OUT/summary_shard.txt 2>&1
  head -12 $OUT/summary_shard.txt
}
if [ "$NOPROF" = 1 ]; then
  [ "$SHARD" = 1 ] && shard
  exit 0
fi
bash scripts/profile.sh $TAG --steps 20 --warmup 5 || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_$TAG $OUT/summary_c4 > $OUT/summary_c4.txt 2>&1
head -12 $OUT/summary_c4.txt
for cfg in C3 C5; do
  PASSES=trace bash scripts/profile.sh ${TAG}_$(echo $cfg | tr A-Z a-z) --config $cfg --steps 10 --warmup 2 --no-parity-sample --em-iters 0 || exit $?
  python3 scripts/prof_summary.py gpurun_out/prof_${TAG}_$(echo $cfg | tr A-Z a-z) $OUT/summary_$(echo $cfg | tr A-Z a-z) > $OUT/summary_$(echo $cfg | tr A-Z a-z).txt 2>&1
  head -12 $OUT/summary_$(echo $cfg | tr A-Z a-z).txt
done
[ "$SHARD" = 1 ] && shard
exit 0

#!/bin/bash
# Copy a scripts/gpu_final.sh TAG run from gpurun_out/ into profiles/ as PREFIX_*:
#   scripts/collect_final.sh TAG PREFIX      (e.g. final r04z)
set -e
TAG=$1; P=$2; IN=gpurun_out/$TAG
cp $IN/tests.log profiles/${P}_gpu_tests.txt
cp $IN/smoke.log profiles/${P}_smoke.txt
for cfg in C4 C3 C5; do
  c=$(echo $cfg | tr A-Z a-z)
  tail -1 $IN/bench_$cfg.json > profiles/${P}_${c}_bench.json
done
cp $IN/summary_c4.json profiles/${P}_c4.json
cp $IN/summary_c4_kernel_stats.csv profiles/${P}_c4_kernel_stats.csv
for c in c3 c5; do
  [ -f $IN/summary_$c.json ] && cp $IN/summary_$c.json profiles/${P}_$c.json
  [ -f $IN/summary_${c}_kernel_stats.csv ] && cp $IN/summary_${c}_kernel_stats.csv profiles/${P}_${c}_kernel_stats.csv
done
ls -la profiles/${P}_*

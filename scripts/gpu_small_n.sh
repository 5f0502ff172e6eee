#!/bin/bash
# fixed per-step cost at strong-scaling shard sizes: bench at several N + a kernel trace at N=12500
set -o pipefail
mkdir -p gpurun_out
bash scripts/strong_sim.sh || exit 1
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_n12500 -o trace --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --N 12500 --steps 30 --warmup 3 > $ROOT/gpurun_out/prof_n12500.log 2>&1 || exit 1
cd $ROOT && python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_n12500/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:8.2f} pct {r["Percentage"]}')
PY

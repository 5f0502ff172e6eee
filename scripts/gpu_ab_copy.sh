#!/bin/bash
# A/B of the statistics hand-over: pinned-host output written by the kernel vs
# device vector + copy (VBHEM_BENCH_COPY=1), at C3, the 12,500-base shard and C4.
set -o pipefail
mkdir -p gpurun_out
for args in "--config C3" "--N 12500" "--config C4"; do
  for copy in "" 1; do
    VBHEM_BENCH_COPY=$copy timeout -k 10 200 python bench.py $args --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$args', 'copy=${copy:-0}', 'ms/step', round(d['ms_per_step'],4), 'value', round(d['value'],1))"
  done
done

#!/bin/bash
# C3 / 12,500-base shard / C4 bench lines (default hand-over), short runs
set -o pipefail
mkdir -p gpurun_out
for args in "--config C3" "--N 12500" "--config C4"; do
  timeout -k 10 200 python bench.py $args --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/s3.json 2> gpurun_out/s3.err || { tail gpurun_out/s3.err; exit 1; }
  tail -1 gpurun_out/s3.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$args', 'ms/step', round(d['ms_per_step'],4), 'value', round(d['value'],1), 'bwd', round(r['kernel_ms'],4), 'list', round(d['gated_forward']['kernel_ms'],4), 'stats', round(d['stats_kernels_ms_per_step'],4), 'em', round(d['emission_kernel_ms'],4))"
done

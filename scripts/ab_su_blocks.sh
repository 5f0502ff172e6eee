#!/bin/bash
# A/B of stats_list_u_kernel's block count (VBHEM_SU_BLOCKS = blocks over all clusters)
set -o pipefail
mkdir -p gpurun_out
run() {  # args, blocks
  if [ -n "$2" ]; then export VBHEM_SU_BLOCKS=$2; else unset VBHEM_SU_BLOCKS; fi
  timeout -k 10 200 python bench.py $1 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/su.json 2> gpurun_out/su.err || { tail gpurun_out/su.err; exit 1; }
  tail -1 gpurun_out/su.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'blocks=${2:-default}', 'ms/step', round(d['ms_per_step'],4), 'stats', round(d['stats_kernels_ms_per_step'],4))"
}
for b in ${NB12:-"" 2048 4096}; do run "--N 12500" "$b"; done
for b in ${NBC4:-"" 3072 4096 6144}; do run "--config C4" "$b"; done

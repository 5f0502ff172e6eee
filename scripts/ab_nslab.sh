#!/bin/bash
# A/B of the chunk (slab) count of the fused E-step (VBHEM_NSLAB; default kMaxSlabs)
set -o pipefail
mkdir -p gpurun_out
run() {  # args, nslab
  if [ -n "$2" ]; then export VBHEM_NSLAB=$2; else unset VBHEM_NSLAB; fi
  timeout -k 10 200 python bench.py $1 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ns.json 2> gpurun_out/ns.err || { tail gpurun_out/ns.err; exit 1; }
  tail -1 gpurun_out/ns.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'nslab=${2:-default}', 'ms/step', round(d['ms_per_step'],4), 'stats', round(d['stats_kernels_ms_per_step'],4))"
}
for b in "" 256 384; do run "--config C4" "$b"; done
for b in "" 128 96; do run "--N 12500" "$b"; done
for b in "" 96 64; do run "--config C3" "$b"; done

#!/bin/bash
# A/B over (library, environment) combinations on one config:
#   scripts/ab_env_lib.sh "<bench args>" lib1.so:VAR=1 lib1.so: lib2.so:VAR=1 ...
set -o pipefail
ARGS=$1; shift
for rep in 1 2; do
  for combo in "$@"; do
    lib=${combo%%:*}; envs=${combo#*:}
    env $envs VBHEM_LIB_PATH=$(realpath $lib) timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$combo', 'value',round(d['value'],2),'ms',round(d['ms_per_step'],3),'bwd',round(d['roofline']['kernel_ms'],3),'fwd',round(d['gated_forward']['kernel_ms'],3),'stats',round(d['stats_kernels_ms_per_step'],3),'em',round(d['emission_kernel_ms'],3))"
  done
done

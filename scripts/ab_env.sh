#!/bin/bash
# Same-box A/B of environment switches on the tree's library: each setting run twice,
# interleaved with the default, one summary line per run.
#   scripts/ab_env.sh [--args "bench args"] "VAR=value [VAR2=value]" ...
set -o pipefail
ARGS="--steps 10 --warmup 2"
if [ "$1" = "--args" ]; then ARGS="$2"; shift 2; fi
EXTRA="--no-cpu-baseline --no-shard-sim --em-iters 0"
[ "$PARITY" = 1 ] || EXTRA="$EXTRA --no-parity-sample"
for rep in 1 2; do
  for setting in default "$@"; do
    envs=(); [ "$setting" != default ] && envs=($setting)
    env "${envs[@]}" timeout -k 10 200 python bench.py $ARGS $EXTRA > gpurun_out/ab_env.json 2>&1 || { tail -5 gpurun_out/ab_env.json; exit 1; }
    tail -1 gpurun_out/ab_env.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); ps=d.get('parity_sample') or {}; g=d.get('gated_forward') or {}; print('$setting', 'ms',round(d['ms_per_step'],4),'bwd',round(d['roofline']['kernel_ms'],4),'fwd/step',round(g.get('ms_per_step',0),4),'stats',round(d['stats_kernels_ms_per_step'],4),'em',round(d['emission_kernel_ms'],4), 'LLerr', ps.get('LL_elbo_max_rel_err'), 'hzerr', ps.get('hat_Z_max_err'))"
  done
done

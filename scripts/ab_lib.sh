# A/B library builds on one box (scripts/build_variant.sh makes them):
#   scripts/ab_lib.sh [--args "bench args"] build/ab/libA.so build/ab/libB.so ...
# each library run twice, interleaved, to see the run-to-run spread ("tree" = the
# tree's own library); PARITY=1 keeps bench's parity sample (L_elbo / hat_Z vs oracle)
set -o pipefail
ARGS="--steps 10 --warmup 2"
if [ "$1" = "--args" ]; then ARGS="$2"; shift 2; fi
EXTRA="--no-cpu-baseline --no-shard-sim --em-iters 0"
[ "$PARITY" = 1 ] || EXTRA="$EXTRA --no-parity-sample"
for rep in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then unset VBHEM_LIB_PATH; else export VBHEM_LIB_PATH=$(realpath $lib); fi
    timeout -k 10 200 python bench.py $ARGS $EXTRA > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); ps=d.get('parity_sample') or {}; print('$lib', 'ms',round(d['ms_per_step'],4),'bwd',round(d['roofline']['kernel_ms'],4),'fwd',round(d['gated_forward']['kernel_ms'],4),'stats',round(d['stats_kernels_ms_per_step'],4),'em',round(d['emission_kernel_ms'],4), 'LLerr', ps.get('LL_elbo_max_rel_err'), 'hzerr', ps.get('hat_Z_max_err'), 'gated_vs_dense', d['dense_schedule']['max_rel_diff_vs_gated'])"
  done
done
unset VBHEM_LIB_PATH

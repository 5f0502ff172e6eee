# A/B library builds on one box (scripts/build_variant.sh makes them):
#   scripts/ab_lib.sh [bench args --] build/ab/libA.so build/ab/libB.so ...
# each library run twice, interleaved, to see the run-to-run spread
set -o pipefail
ARGS="--steps 10 --warmup 2"
if [ "$1" = "--args" ]; then ARGS="$2"; shift 2; fi
for rep in 1 2; do
  for lib in "$@"; do
    VBHEM_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py $ARGS --no-cpu-baseline --no-parity-sample --no-shard-sim --em-iters 0 > gpurun_out/ab.json 2>&1 || exit 1
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'ms',round(d['ms_per_step'],4),'bwd',round(d['roofline']['kernel_ms'],4),'fwd',round(d['gated_forward']['kernel_ms'],4),'stats',round(d['stats_kernels_ms_per_step'],4),'em',round(d['emission_kernel_ms'],4))"
  done
done

# A/B library builds on the C4 bench: scripts/ab_lib.sh build/ab/libA.so build/ab/libB.so ...
# (each run twice, interleaved, to see the run-to-run spread)
set -o pipefail
for rep in 1 2; do
  for lib in "$@"; do
    VBHEM_LIB_PATH=$(realpath $lib) timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>&1 || exit 1
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', 'value',round(d['value'],2),'bwd',round(d['roofline']['kernel_ms'],3),'fwd',round(d['gated_forward']['kernel_ms'],3),'stats',round(d['stats_kernels_ms_per_step'],3),'em',round(d['emission_kernel_ms'],3))"
  done
done

# A/B of the backward-pass lanes per column (VBHEM_BWD_LPC) on C4 and a C5 slice
set -o pipefail
for cfg in "--config C4" "--config C5 --N 100000"; do
  for l in 0 alt; do
    if [ $l = alt ]; then export VBHEM_BWD_LPC=$( [[ $cfg == *C5* ]] && echo 2 || echo 1 ); else unset VBHEM_BWD_LPC; fi
    timeout -k 10 200 python bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>&1 || exit 1
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'lpc=${VBHEM_BWD_LPC:-def}', 'value',round(d['value'],2),'bwd',round(d['roofline']['kernel_ms'],3),'fwd',round(d['gated_forward']['kernel_ms'],3),'stats',round(d['stats_kernels_ms_per_step'],3),'em',round(d['emission_kernel_ms'],3), 'gated', round(d['gated_pairs_frac'],4))"
  done
done

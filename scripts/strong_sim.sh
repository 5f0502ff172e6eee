# single-GPU runs at the shard sizes of an N-GPU strong-scaling run of C4
set -o pipefail
for n in 100000 50000 25000 12500; do
  timeout -k 10 200 python bench.py --N $n --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ss.json 2>&1 || exit 1
  tail -1 gpurun_out/ss.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$n', 'ms/step',round(d['ms_per_step'],3),'bwd',round(d['roofline']['kernel_ms'],3),'fwd',round(d['gated_forward']['kernel_ms'],3),'stats',round(d['stats_kernels_ms_per_step'],3),'em',round(d['emission_kernel_ms'],3))"
done

# GPU tests, then the C5 slice (N = 100,000 of the 10^6 bases: S = 12, d = 16)
set -o pipefail
bash scripts/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py --config C5 --N 100000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c5.json 2>&1 || { tail -5 gpurun_out/c5.json; exit 1; }
tail -1 gpurun_out/c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5 value',d['value'],'bwd',d['roofline']['kernel_ms'],'fwd',d['gated_forward']['kernel_ms'],'em',d['emission_kernel_ms'],'stats',d['stats_kernels_ms_per_step'])"

set -o pipefail
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_gated.json 2>&1 || exit 1
tail -1 gpurun_out/bench_gated.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'bwd',d['roofline']['kernel_ms'],'fwd',d['gated_forward']['kernel_ms'],'stats',d['stats_kernels_ms_per_step'],'em',d['emission_kernel_ms'],'dense',d['dense_schedule'])"

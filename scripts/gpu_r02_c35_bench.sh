#!/bin/bash
# C3 and C5 (N = 10^6) bench lines + rocprofv3 trace and PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
tail -1 gpurun_out/bench_c3.json | cut -c1-300
timeout -k 10 600 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail gpurun_out/bench_c5.err; exit 1; }
tail -1 gpurun_out/bench_c5.json | cut -c1-300
bash scripts/gpu_r02_prof_c35.sh ${1:-r02}

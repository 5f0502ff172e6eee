#!/bin/bash
# Round-2 GPU batch: full GPU suite, drop-in costs, C3 and C5 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/dropin_bench.py > gpurun_out/dropin.jsonl 2> gpurun_out/dropin.err || { tail gpurun_out/dropin.err; exit 1; }
cat gpurun_out/dropin.jsonl
timeout -k 10 300 python bench.py --config C3 --steps 50 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 1; }
tail -1 gpurun_out/bench_c3.json | cut -c1-300
timeout -k 10 600 python bench.py --config C5 --steps 5 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail gpurun_out/bench_c5.err; exit 1; }
tail -1 gpurun_out/bench_c5.json | cut -c1-300

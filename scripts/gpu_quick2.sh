#!/bin/bash
# GPU parity suite (fail fast) then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "kernel", r["kernel"], r["kernel_ms"], "frac", r["frac"])
print("list", d["gated_forward"] and d["gated_forward"]["kernel_ms"], "stats", d["stats_kernels_ms_per_step"], "dense", d["dense_schedule"])
PY

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("value", round(d["value"], 2), "ms", round(d["ms_per_step"], 4), "kernel", r["kernel"], round(r["kernel_ms"], 4), "frac", round(r["frac"], 4))
print("list", d["gated_forward"] and round(d["gated_forward"]["kernel_ms"], 4), "stats", round(d["stats_kernels_ms_per_step"], 4), "em", d["emission_kernel_ms"], "dense", round(d["dense_schedule"]["value"], 2))
PY

#!/bin/bash
# Kernel trace (with timestamps) of a short small-shard bench run: gaps between
# the kernels of one E-step at N = 12,500 (the 8-GPU shard of C4).
set -o pipefail
TAG=${1:-small}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 $ROOT/bench.py --N ${N:-12500} --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log | cut -c1-300

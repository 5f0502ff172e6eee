#!/bin/bash
# Kernel trace of a short bench run (default C5 slice; BENCH_ARGS overrides):
#   scripts/gpu_trace.sh TAG [env assignments...]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
    python3 $ROOT/bench.py ${BENCH_ARGS:---config C5 --N 100000 --steps 2 --warmup 1} --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
f=$(ls $OUT/*/*kernel_stats.csv $OUT/*kernel_stats.csv 2>/dev/null | head -1)
head -14 "$f" | cut -c1-160

#!/bin/bash
# fb_bwd2_kernel check: the GPU tests, then C4 bench A/B over library builds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_lib.sh "$@"

#!/bin/bash
# fused-E-step tests (several base groups, trials, stats variants), then the statistics sweeps
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_emission_u.py tests/test_gpu_scale.py tests/test_trials.py tests/test_robustness.py tests/test_gateway_fused.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/m7_tests.log 2>&1
rc=$?; tail -3 gpurun_out/m7_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_sweep5.sh

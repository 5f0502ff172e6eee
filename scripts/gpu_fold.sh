#!/bin/bash
# folded exact fallback: parity/robustness tests, then the 12.5k shard and C3 timing
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_robustness.py tests/test_emission_u.py tests/test_gpu_scale.py tests/test_trials.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fold_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fold_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/stats_sweep.py --config C4 --N 12500 --reps 40 - VBHEM_NO_FOLD_EXACT=1 > gpurun_out/fold_sweep.log 2>&1 &&
timeout -k 10 200 python -u scripts/stats_sweep.py --config C3 --reps 40 - VBHEM_NO_FOLD_EXACT=1 >> gpurun_out/fold_sweep.log 2>&1
rc=$?; grep setting gpurun_out/fold_sweep.log; exit $rc

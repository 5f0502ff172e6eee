#!/bin/bash
# statistics kernels: tests, then A/B sweeps at C4 and C5 (200 k bases)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_emission_u.py tests/test_gpu_scale.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/m6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/m6_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/stats_sweep.py - VBHEM_NO_STATS_M=1 VBHEM_SU_BLOCKS=512 VBHEM_SU_BLOCKS=768 > gpurun_out/sweep4.log 2>&1 &&
timeout -k 10 300 python -u scripts/stats_sweep.py --config C5 --N 200000 --reps 4 - VBHEM_NO_STATS_M=1 VBHEM_SM_PD=4 VBHEM_SU_BLOCKS=1536 >> gpurun_out/sweep4.log 2>&1
rc=$?; grep setting gpurun_out/sweep4.log; exit $rc

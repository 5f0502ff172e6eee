#!/bin/bash
# statistics kernel choice at C3 and at the 12,500-base C4 shard
set -o pipefail
timeout -k 10 200 python -u scripts/stats_sweep.py --config C3 - VBHEM_STATS_M=1 VBHEM_STATS_M=1,VBHEM_SU_BLOCKS=512 > gpurun_out/sweep5.log 2>&1 &&
timeout -k 10 200 python -u scripts/stats_sweep.py --config C4 --N 12500 - VBHEM_NO_STATS_M=1 VBHEM_SU_BLOCKS=512 VBHEM_SU_BLOCKS=256 >> gpurun_out/sweep5.log 2>&1
rc=$?; grep setting gpurun_out/sweep5.log; exit $rc

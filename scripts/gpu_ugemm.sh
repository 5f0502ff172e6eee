#!/bin/bash
# emission GEMM on the prepared operand: GPU tests, then C4 and a C5 slice with/without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in "--config C4 --steps 10 --warmup 2" "--config C5 --N 100000 --steps 3 --warmup 1"; do
  for v in 0 1; do
    if [ $v = 1 ]; then export VBHEM_NO_UGEMM=1; else unset VBHEM_NO_UGEMM; fi
    timeout -k 10 300 python bench.py $cfg --no-cpu-baseline > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
    tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'no_ugemm=$v', 'value',round(d['value'],3),'ms',round(d['ms_per_step'],3),'bwd',round(d['roofline']['kernel_ms'],3),'fwd',round(d['gated_forward']['kernel_ms'],3),'stats',round(d['stats_kernels_ms_per_step'],3),'em',round(d['emission_kernel_ms'],3))"
  done
done

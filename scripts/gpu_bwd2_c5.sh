#!/bin/bash
# fb_bwd2_kernel for S > 8: GPU tests, then the C5 slice with the bwd2 builds and without bwd2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 300 python bench.py --config C5 --N 100000 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.json 2>&1 || { tail -5 gpurun_out/ab.json; exit 1; }
  tail -1 gpurun_out/ab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', 'value',round(d['value'],3),'ms',round(d['ms_per_step'],3),'bwd',d['roofline']['kernel'],round(d['roofline']['kernel_ms'],3),'em',round(d['emission_kernel_ms'],3))"
}
for lib in "$@"; do VBHEM_LIB_PATH=$(realpath $lib) run $lib || exit 1; done
VBHEM_NO_BWD2=1 run no_bwd2 || exit 1

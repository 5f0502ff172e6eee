# GPU tests, then per-step overhead at shard sizes and a short bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/overhead_probe.py 12500 100000 || exit 1
bash scripts/strong_sim.sh

# resp_kernel's gate lists (StatsArgs::gflag, a look-back over its chunks): the targeted
# parity tests, the whole -m gpu suite, then C3 with and without it (interleaved)
set -o pipefail
OUT=gpurun_out/r04y; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "bwd2_in_kernel_prep or k1_in_recursion or exact_fallback_gated" \
  tests/test_robustness.py > $OUT/targeted.log 2>&1 || { tail -30 $OUT/targeted.log; exit 1; }
tail -2 $OUT/targeted.log
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in resp gate; do
    if [ $v = gate ]; then export VBHEM_NO_RESP_LIST=1; else unset VBHEM_NO_RESP_LIST; fi
    timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline --no-parity-sample --no-shard-sim --em-iters 0 > $OUT/c3_$v$rep.json 2> $OUT/c3_$v$rep.err || { tail -5 $OUT/c3_$v$rep.err; exit 1; }
    tail -1 $OUT/c3_$v$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],1), 'ms', round(d['ms_per_step'],5), 'sync', round(d['synchronous']['ms_per_step'],5), 'bwd', round(d['roofline']['kernel_ms'],5), 'stats', round(d['stats_kernels_ms_per_step'],5))"
  done
done
unset VBHEM_NO_RESP_LIST

# bench.py's pacing with the native RCCL communicator on one rank (VBHEM_BENCH_RCCL_ONE)
# against the default one-rank path, default step counts (C4 and a 12,500-base shard);
# first the RCCL tests (allreduce_to into the pinned statistics buffer)
set -o pipefail
OUT=gpurun_out/r04v2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_em.py -k rccl > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do
  for v in rccl plain; do
    if [ $v = rccl ]; then export VBHEM_BENCH_RCCL_ONE=1; else unset VBHEM_BENCH_RCCL_ONE; fi
    for n in 100000 12500; do
      timeout -k 10 300 python -u bench.py --N $n --no-cpu-baseline --no-parity-sample --no-shard-sim --em-iters 0 > $OUT/${v}_${n}_$rep.json 2> $OUT/${v}_${n}_$rep.err || { tail -5 $OUT/${v}_${n}_$rep.err; exit 1; }
      tail -1 $OUT/${v}_${n}_$rep.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $n, round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'sync', round(d['synchronous']['ms_per_step'],4), 'bwd', round(d['roofline']['kernel_ms'],4), d['collective'])"
    done
  done
done

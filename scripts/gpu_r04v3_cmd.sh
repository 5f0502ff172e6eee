# the C++ EM loop's per-iteration time with the native RCCL communicator on one rank
# (bench.py's em_iteration, VBHEM_BENCH_RCCL_ONE) at a 12,500-base shard and at C4
set -o pipefail
OUT=gpurun_out/r04v3; mkdir -p $OUT
for n in 12500 100000; do
  for v in rccl plain; do
    if [ $v = rccl ]; then export VBHEM_BENCH_RCCL_ONE=1; else unset VBHEM_BENCH_RCCL_ONE; fi
    timeout -k 10 300 python -u bench.py --N $n --no-cpu-baseline --no-parity-sample --no-shard-sim > $OUT/${v}_$n.json 2> $OUT/${v}_$n.err || { tail -5 $OUT/${v}_$n.err; exit 1; }
    tail -1 $OUT/${v}_$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['em_iteration']; print('$v', $n, round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'em', round(e['ms'],4), 'paired', round(e['paired_diff_ms'],4), e['collective'])"
  done
done

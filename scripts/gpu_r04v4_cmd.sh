# (final tree, default-size step counts)
# rehearsal of bench.py's multi-rank path on one GPU: 2 ranks sharing it over gloo, and
# one rank through the native RCCL communicator (VBHEM_BENCH_RCCL_ONE)
set -o pipefail
OUT=gpurun_out/r04v4; mkdir -p $OUT
VBHEM_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --no-parity-sample > $OUT/gloo2.log 2>&1 || { tail -30 $OUT/gloo2.log; exit 1; }
grep '^{' $OUT/gloo2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gloo2', d['n_gpus'], round(d['value'],2), d['collective'], (d.get('em_iteration') or {}).get('ms'))"
VBHEM_BENCH_RCCL_ONE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity-sample --no-shard-sim > $OUT/rccl1.log 2>&1 || { tail -30 $OUT/rccl1.log; exit 1; }
tail -1 $OUT/rccl1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rccl1', d['n_gpus'], round(d['value'],2), d['collective'], (d.get('em_iteration') or {}).get('ms'), (d.get('em_iteration') or {}).get('collective'))"

# the backward kernels timed by events the dispatch records (hipExtLaunchKernelGGL):
# timing tests, C4 / C3 / C5 bench lines, and a C4 kernel trace to compare against
set -o pipefail
OUT=gpurun_out/r04t; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "timing or capi or fused_matches or bench" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for c in C4 C3 C5; do
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline --no-parity-sample --em-iters 0 > $OUT/b_$c.json 2>$OUT/b_$c.err || { tail -5 $OUT/b_$c.err; exit 1; }
  tail -1 $OUT/b_$c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', 'value', round(d['value'],2), 'ms', round(d['ms_per_step'],4), 'kernel_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'shard', (d.get('shard_sim') or {}).get('estep_ceiling_8gpu'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/tr -o tr --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-parity-sample --em-iters 0 --no-shard-sim --steps 20 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/$OUT/tr -name "*kernel_stats.csv" | head -1); grep -E "fb_bwd4|emission_u" $f | cut -c1-160
tail -1 $GRAFT_REPO_ROOT/$OUT/tr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('under trace: kernel_ms', round(d['roofline']['kernel_ms'],4))"

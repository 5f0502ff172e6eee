# completion word instead of per-step events: the new test + fused/gated subset, C3 /
# 12,500-base / C4 bench lines with the word (tree) and with events (VBHEM_BENCH_EVENTS=1)
set -o pipefail
OUT=gpurun_out/r04p; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -v -m gpu -k "completion or fused or gated or fallback" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2; do
for ev in 0 1; do
  for a in "--config C3 --steps 60 --warmup 5" "--N 12500 --steps 40 --warmup 5" "--steps 20 --warmup 3"; do
    if [ $ev = 1 ]; then export VBHEM_BENCH_EVENTS=1; else unset VBHEM_BENCH_EVENTS; fi
    timeout -k 10 300 python bench.py $a --no-cpu-baseline --no-shard-sim --em-iters 0 --no-parity-sample > $OUT/b.json 2>&1 || { tail -5 $OUT/b.json; exit 1; }
    tail -1 $OUT/b.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('events=$ev', '$a'.split('--steps')[0], 'ms', round(d['ms_per_step'],4), 'sync', round(d['synchronous']['ms_per_step'],4), d['handover'][:20])"
  done
done
done
unset VBHEM_BENCH_EVENTS

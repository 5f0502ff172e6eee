#!/bin/bash
# round 6: completion-word pacing.  Tests, then C3 / C4 bench lines with the word and
# with events (VBHEM_BENCH_EVENT=1).  scripts/gpu_step6.sh TAG
set -o pipefail
TAG=${1:-r06n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_done_word.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "done_word or exact_fallback" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
summ() {
python3 - $1 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
s = d.get("shard_sim") or {}
print(sys.argv[1].split("/")[-1], round(d["value"], 2), round(d["ms_per_step"], 5), "frac", round(d["roofline"]["frac"], 4),
      "shard", s.get("estep_ms"), s.get("estep_ceiling_8gpu"))
PY
}
for cfg in C3 C4; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-parity-sample --em-iters 0 > $OUT/$cfg.json 2> $OUT/$cfg.err || exit $?
  summ $OUT/$cfg.json
  VBHEM_BENCH_EVENT=1 timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --no-parity-sample --em-iters 0 > $OUT/${cfg}_ev.json 2> $OUT/${cfg}_ev.err || exit $?
  summ $OUT/${cfg}_ev.json
done

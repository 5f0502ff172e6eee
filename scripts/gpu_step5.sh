#!/bin/bash
# round 6: list4 inline fallback + settle: targeted tests, then the C4 bench line and
# the shard trace.  scripts/gpu_step5.sh TAG
set -o pipefail
TAG=${1:-r06k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "exact_fallback or list4 or range_check or C4 or c4 or gated" > $OUT/t.log 2>&1
rc=$?; tail -3 $OUT/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || exit $?
python3 - $OUT/c4.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
s = d["shard_sim"]
print("C4", round(d["value"], 2), round(d["ms_per_step"], 4), "settle", d["settle"]["steps"], "frac", round(d["roofline"]["frac"], 4),
      "shard", round(s["estep_ms"], 4), "sync", round(s["estep_sync_ms"], 4), "ceil", round(s["estep_ceiling_8gpu"], 3))
PY

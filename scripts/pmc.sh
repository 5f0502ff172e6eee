#!/bin/bash
# Extra PMC passes over bench.py (one rocprofv3 --pmc pass per quoted counter group).
# Usage: scripts/pmc.sh TAG "CTR1 CTR2 ..." ["CTR3 ..."] -- [bench args...]
set -o pipefail
TAG=$1; shift
GROUPS_=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
[ "$1" == "--" ] && shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
k=0
for g in "${GROUPS_[@]}"; do
  k=$((k+1))
  timeout -k 10 300 rocprofv3 --pmc $g -d $OUT/p$k -o p$k --output-format csv -- \
      python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/p$k.log 2>&1
  rc=$?; echo "pass $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - "$OUT" <<'EOF'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(sys.argv[1] + "/p*/*_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "vbhem" in n:
            acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in acc.items():
    print(n)
    for k, v in sorted(c.items()):
        print(f"   {k:32s} {sum(v) / len(v):16.4e}")
EOF

# the idle gap between paced E-steps: torch events vs events without the system-scope
# release vs no per-step event (scripts/gap_probe.py)
set -o pipefail
OUT=gpurun_out/r04o; mkdir -p $OUT
for a in "C3" "C4 12500" "C4"; do
  timeout -k 10 300 python -u scripts/gap_probe.py $a >> $OUT/gap.txt 2>&1 || { tail -20 $OUT/gap.txt; exit 1; }
done
cat $OUT/gap.txt

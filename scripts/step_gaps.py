#!/usr/bin/env python3
"""Per-E-step GPU time and the gap before it, from a rocprofv3 kernel trace
(scripts/step_gaps.py TRACE_CSV [first_kernel_substring]): median over the steps of
each pacing kind (gap < 20 us: run-ahead; else: synchronous)."""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "emission_prep"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, cur = [], None
for r in rows:
    if first in r["Kernel_Name"]:
        cur = [r]
        steps.append(cur)
    elif cur is not None:
        cur.append(r)
kinds = {}
prev = None
for s in steps:
    t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
    if prev is not None:
        gap = (t0 - prev) / 1e3
        k = "run-ahead" if gap < 20 else "sync"
        kinds.setdefault(k, []).append(((t1 - t0) / 1e3, gap, len(s)))
    prev = t1
for k, v in kinds.items():
    nk = st.mode(x[2] for x in v)
    v = [x for x in v if x[2] == nk]
    print(f"{k:10s} steps {len(v):5d}  kernels {nk}  gpu {st.median(x[0] for x in v):8.1f} us  "
          f"gap {st.median(x[1] for x in v):6.1f} us  cadence {st.median(x[0] + x[1] for x in v):8.1f} us")

#!/usr/bin/env python3
"""Median duration (and the median gap before it) per kernel in rocprofv3 kernel
traces, side by side: scripts/kernel_medians.py A.csv B.csv ... (kernels with >= 100
launches; first 200 records skipped)."""
import csv
import statistics as st
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d, g, prev = {}, {}, None
    for r in rows[200:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = r["Kernel_Name"].replace("void ", "").replace("vbhem::", "").split("(")[0][:30]
        d.setdefault(k, []).append((e - s) / 1e3)
        if prev is not None:
            g.setdefault(k, []).append((s - prev) / 1e3)
        prev = e
    return d, g


tabs = [load(p) for p in sys.argv[1:]]
names = [k for k, v in tabs[0][0].items() if len(v) >= 100]
for k in names:
    cells = []
    for d, g in tabs:
        if k in d:
            cells.append(f"{st.median(d[k]):8.2f} (+{st.median(g.get(k, [0])):5.2f})")
        else:
            cells.append(" " * 17)
    print(f"{k:32s}" + "  ".join(cells))

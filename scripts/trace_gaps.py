"""Per-kernel start offsets, gaps and durations of a few gated E-steps from a
rocprofv3 kernel trace (run_kernel_trace.csv): python scripts/trace_gaps.py DIR"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "emission_prep" in r["Kernel_Name"]]
shown = 0
for k in range(len(idx) - 1):
    s, e = idx[k], idx[k + 1]
    if not any("fb_bwd" in r["Kernel_Name"] for r in rows[s:e]) or k < 6:
        continue
    t0 = int(rows[s]["Start_Timestamp"])
    prev = t0
    for r in rows[s:e + 1]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(st - t0) / 1e3:8.1f} gap {(st - prev) / 1e3:6.1f} dur {(en - st) / 1e3:7.1f}  "
              f"{r['Kernel_Name'][:60]}")
        prev = en
    print()
    shown += 1
    if shown == 2:
        break

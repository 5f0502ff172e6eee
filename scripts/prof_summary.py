#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into profiles/.

Reads <dir>/trace/*_kernel_stats.csv (rocprofv3 --kernel-trace --stats) and
<dir>/pmc*/ *_counter_collection.csv (one --pmc pass each) and writes
<out>.json with, per kernel: calls, average duration, and the per-dispatch
averages of every collected counter.  HBM traffic per launch follows
MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so
    traffic_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.

    python scripts/prof_summary.py gpurun_out/prof_TAG profiles/r01_c4
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main(src, out):
    res = {"source": os.path.basename(os.path.normpath(src)), "kernels": {}}
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):  # the bench JSON line of the traced run names the workload
        for line in open(log):
            if line.startswith('{"metric"'):
                b = json.loads(line)
                res.update(N=b["config"]["N"], n_gpus=b["n_gpus"], workload=b["config"]["workload"],
                           bench_under_trace=b)
    pa = os.path.join(src, "pmc_args.txt")
    if os.path.exists(pa):  # scripts/profile.sh: PMC passes without shard-size launches
        res["pmc_args"] = open(pa).read().strip()
        res["pmc_full_size_only"] = "--no-shard-sim" in res["pmc_args"]
    stats = glob.glob(os.path.join(src, "trace", "*_kernel_stats.csv"))
    if stats:
        with open(stats[0]) as f:
            for row in csv.DictReader(f):
                k = res["kernels"].setdefault(short(row["Name"]), {})
                k.update(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]),
                         min_ns=float(row["MinNs"]), max_ns=float(row["MaxNs"]),
                         pct_time=float(row["Percentage"]))
        shutil.copy(stats[0], out + "_kernel_stats.csv")
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for path in sorted(glob.glob(os.path.join(src, "pmc*", "*_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                kn = short(row["Kernel_Name"])
                acc[kn][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[kn] = dict(grid=int(row["Grid_Size"]), wg=int(row["Workgroup_Size"]),
                                lds=int(row["LDS_Block_Size"]), vgpr=int(row["VGPR_Count"]),
                                agpr=int(row["Accum_VGPR_Count"]), sgpr=int(row["SGPR_Count"]),
                                scratch=int(row["Scratch_Size"]))
    for kn, ctrs in acc.items():
        k = res["kernels"].setdefault(kn, {})
        k["launch"] = meta[kn]
        k["counters_per_dispatch"] = {c: sum(v) / len(v) for c, v in ctrs.items()}
        c = k["counters_per_dispatch"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd = 2.0 * c["FETCH_SIZE"] * 1024.0
            wr = c["WRITE_SIZE"] * 1024.0
            k["hbm_bytes_per_launch"] = {"read_corrected": rd, "write": wr, "traffic": rd + wr}
    with open(out + ".json", "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for kn, k in sorted(res["kernels"].items(), key=lambda x: -x[1].get("pct_time", 0)):
        line = f"{kn:45s} calls={k.get('calls', '-'):>4} avg={k.get('avg_ns', 0) / 1e6:8.3f} ms"
        if "hbm_bytes_per_launch" in k:
            line += f"  traffic={k['hbm_bytes_per_launch']['traffic'] / 1e9:7.3f} GB"
        print(line)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

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
    ta = os.path.join(src, "trace_args.txt")
    if os.path.exists(ta):  # scripts/profile.sh: the traced command's bench arguments
        res["trace_args"] = open(ta).read().strip()
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
    # per-dispatch durations from the kernel trace: mean / median / spread per kernel
    # (the summary's own evidence for the roofline kernel's launch time)
    traces = glob.glob(os.path.join(src, "trace", "*_kernel_trace.csv"))
    if traces:
        durs = defaultdict(list)
        with open(traces[0]) as f:
            for row in csv.DictReader(f):
                durs[short(row["Kernel_Name"])].append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
        for kn, v in durs.items():
            v = sorted(v)
            n = len(v)
            res["kernels"].setdefault(kn, {})["trace_launches_ms"] = dict(
                n=n, mean=sum(v) / n, median=(v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])),
                p10=v[int(0.1 * (n - 1))], p90=v[int(0.9 * (n - 1))], min=v[0], max=v[-1])
    res["launch_sizes"] = ("homogeneous: every launch of a kernel in these passes processes the same "
                           "base count (the traced bench runs with --no-shard-sim)"
                           if "--no-shard-sim" in res.get("trace_args", "") else "mixed or unknown")
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
    roofline_check(res)
    with open(out + ".json", "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for kn, k in sorted(res["kernels"].items(), key=lambda x: -x[1].get("pct_time", 0)):
        line = f"{kn:45s} calls={k.get('calls', '-'):>4} avg={k.get('avg_ns', 0) / 1e6:8.3f} ms"
        if "hbm_bytes_per_launch" in k:
            line += f"  traffic={k['hbm_bytes_per_launch']['traffic'] / 1e9:7.3f} GB"
        print(line)


def roofline_check(res):
    """The bench line's roofline fraction recomputed from this summary alone: the
    traced bench's flops per pair x pairs per launch (its `roofline` block) over the
    kernel trace's mean and median launch time of the same kernel, against the fp64
    peak; beside it the bench's live-event value and, when the PMC passes ran, the
    kernel's matrix-core counters."""
    b = res.get("bench_under_trace")
    if not b or "roofline" not in b:
        return
    r = b["roofline"]
    k = res["kernels"].get(r["kernel"], {})
    t = k.get("trace_launches_ms")
    if not t:
        return
    work = r["flops_per_pair"] * r["pairs_per_launch"]   # flops per launch
    chk = dict(kernel=r["kernel"], flops_per_launch=work, peak_TFLOPs=r["peak"],
               trace_mean_ms=t["mean"], trace_median_ms=t["median"], trace_launches=t["n"],
               frac_trace_mean=work / (t["mean"] * 1e-3) / 1e12 / r["peak"],
               frac_trace_median=work / (t["median"] * 1e-3) / 1e12 / r["peak"],
               bench_kernel_ms=r["kernel_ms"], bench_frac=r["frac"])
    c = k.get("counters_per_dispatch", {})
    if "SQ_INSTS_VALU_MFMA_MOPS_F64" in c:
        # MOPS counts 512 flops each (counter_defs.yaml): matrix-core flops per launch
        chk["mfma_f64_flops_per_launch"] = c["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
    for n in ("SQ_INSTS_VALU_MFMA_F64", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_VALU_MFMA_COEXEC_CYCLES"):
        if n in c:
            chk[n] = c[n]
    res["roofline_check"] = chk


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

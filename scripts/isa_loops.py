#!/usr/bin/env python3
"""ISA account of a kernel's innermost loops (the per-quad-step counts).

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S -o k.s file.hip
    python3 scripts/isa_loops.py k.s [kernel-name-substring]

For every backward branch (a loop latch) inside the kernel it prints the loop body's
instruction mix: fp64 VALU, other VALU (int32, moves, permlanes), MFMA, LDS, VMEM,
SALU/SMEM, waits and NOPs, with the fp64 VALU split by opcode.  Loops are the ranges
[label, latch]; nested loops are reported separately (the inner one first).
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "_f64" in op or op in ("v_cvt_f64_i32", "v_cvt_f64_u32", "v_frexp_mant_f64",
                                  "v_frexp_exp_i32_f64", "v_ldexp_f64", "v_rcp_f64"):
            return "valu_f64"
        return "valu_other"
    return "other"


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    lines = open(path).read().split("\n")
    # kernel bodies: from "<name>:" (a function label) to ".Lfunc_end"
    kernels = []
    cur = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", ln)
        if m:
            cur = [m.group(1), i, None]
            kernels.append(cur)
        elif cur and ln.startswith(".Lfunc_end") and cur[2] is None:
            cur[2] = i
    for name, a, b in kernels:
        if want and want not in name:
            continue
        body = lines[a:b]
        labels = {}
        for k, ln in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", ln)
            if m:
                labels[m.group(1)] = k
        print(f"== {name} ({b - a} lines)")
        for k, ln in enumerate(body):
            m = re.match(r"^\s+(s_cbranch_\w+|s_branch)\s+(\.LBB\S+)", ln)
            if not m or m.group(2) not in labels or labels[m.group(2)] >= k:
                continue
            start = labels[m.group(2)]
            cnt, f64 = Counter(), Counter()
            for ln2 in body[start:k + 1]:
                t = ln2.strip()
                if not t or t.startswith((";", ".")) or t.endswith(":"):
                    continue
                op = t.split()[0]
                c = classify(op)
                cnt[c] += 1
                if c == "valu_f64":
                    f64[op] += 1
            if sum(cnt.values()) < 8:
                continue
            print(f"  loop {m.group(2)} (lines {start}-{k}): " +
                  ", ".join(f"{c} {n}" for c, n in sorted(cnt.items())))
            print("     f64: " + ", ".join(f"{o} {n}" for o, n in f64.most_common()))


if __name__ == "__main__":
    main()

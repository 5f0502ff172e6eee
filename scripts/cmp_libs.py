#!/usr/bin/env python3
"""Bit-for-bit comparison of two builds of the library on the same inputs (A/B of a
kernel change that is meant to keep every result identical).

    python scripts/cmp_libs.py dump OUT.npz          # with VBHEM_LIB_PATH=... for the build
    python scripts/cmp_libs.py diff A.npz B.npz

dump: for C4 (N = 1000, the two 500-base shards too, and N = 20000), C5 (N = 1500) and
C3 (N = 2000) one fused E-step from the synthetic posterior: L_elbo, hat_Z and the
packed statistics.  diff: the number of differing entries and the largest relative
difference per array."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(out):
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import host
    from vbhem_amd.em import tilde_n
    from vbhem_amd.estep import EStepEngine
    res = {}
    for name, N, shards in (("C4", 1000, [(0, 1000), (0, 500), (500, 1000)]), ("C4", 20000, [(0, 20000)]),
                            ("C5", 1500, [(0, 1500)]), ("C3", 2000, [(0, 2000)])):
        base, P, opt = vb.synth_workload(name, N=N)
        for lo, hi in shards:
            eng = EStepEngine(base.shard(lo, hi), P.K, P.S, opt["tau"], device="cuda:0")
            eng.set_clusters(host.cluster_constants(P, base.covmode))
            eng.set_log_omega(host.log_omega_tilde(P.alpha))
            tN = tilde_n(eng, opt["Nv"], N)
            st = eng.fused(tN).cpu().numpy()
            torch.cuda.synchronize()
            key = f"{name}_{N}_{lo}_{hi}"
            res[key + "_stats"] = st
            res[key + "_LL"] = eng.LL.cpu().numpy()
            res[key + "_fallback"] = np.array([eng.fallback_count()])
    np.savez(out, **res)
    print("dumped", out, os.environ.get("VBHEM_LIB_PATH", "tree"))


def diff(a, b):
    A, B = np.load(a), np.load(b)
    for k in sorted(A.files):
        x, y = A[k], B[k]
        nd = int((x != y).sum())
        rel = float(np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-300))) if nd else 0.0
        print(f"{k:28s} differing {nd:8d} / {x.size:8d}  max rel {rel:.3e}")


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        diff(sys.argv[2], sys.argv[3])

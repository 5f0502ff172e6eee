"""Backward-pass A/B check on the GPU: L_elbo of fb_bwd4_kernel (MFMA) against
fb_bwd2_kernel (VBHEM_NO_BWD4=1, read when each call plans its kernels) on a C4
workload; prints the largest relative difference and where the mismatches sit
(base index mod 16, cluster).  Development tool.
  python scripts/bwd4_check.py [N]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import pkgload  # noqa: E402

vb = pkgload.load()
from vbhem_amd.estep import EStepEngine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
dev = torch.device("cuda", 0)
base, post, opt = vb.synth_workload("C4", device=dev, N=N)
consts = vb.host.cluster_constants(post, base.covmode)
eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
eng.set_clusters(consts)
eng.set_log_omega(vb.host.log_omega_tilde(post.alpha))
tN = (float(opt["Nv"]) * N) * eng.base.omega
out = {}
for mode in ("bwd4", "bwd2"):
    if mode == "bwd2":
        os.environ["VBHEM_NO_BWD4"] = "1"
    eng.fused(tN)
    torch.cuda.synchronize()
    out[mode] = eng.LL.cpu().numpy().copy()
os.environ.pop("VBHEM_NO_BWD4", None)
a, b = out["bwd4"], out["bwd2"]
rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
print("N", N, "max rel", float(rel.max()), "mean rel", float(rel.mean()))
bad = np.argwhere(rel > 1e-10)
print("mismatched pairs", len(bad), "of", rel.size)
if len(bad):
    i, j = bad[:, 0], bad[:, 1]
    print("base mod 16 histogram", np.bincount(i % 16, minlength=16).tolist())
    print("cluster histogram", np.bincount(j, minlength=post.K).tolist())
    print("first", bad[:10].tolist(), a[tuple(bad[0])], b[tuple(bad[0])])

"""MFMA-kernel A/B check on the GPU: L_elbo of fb_bwd4_kernel against
fb_bwd2_kernel (VBHEM_NO_BWD4=1, read when each call plans its kernels) and the
statistics of fb_list4_kernel against fb_split_kernel's list mode (VBHEM_NO_LIST4=1)
on a C4 workload; prints the largest relative difference and where the mismatches sit
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
out, st = {}, {}
for mode, env in (("mfma", {}), ("split", {"VBHEM_NO_LIST4": "1"}),
                  ("bwd2", {"VBHEM_NO_BWD4": "1", "VBHEM_NO_LIST4": "1"})):
    for k in ("VBHEM_NO_BWD4", "VBHEM_NO_LIST4"):
        os.environ.pop(k, None)
    os.environ.update(env)
    s = eng.fused(tN).cpu().numpy().copy()
    torch.cuda.synchronize()
    out[mode] = eng.LL.cpu().numpy().copy()
    st[mode] = s
for k in ("VBHEM_NO_BWD4", "VBHEM_NO_LIST4"):
    os.environ.pop(k, None)
for m in ("mfma", "split"):
    d = np.abs(st[m] - st["bwd2"]) / np.maximum(np.abs(st["bwd2"]), 1e-300)
    big = np.abs(st["bwd2"]) > 1e-12 * np.abs(st["bwd2"]).max()
    print(m, "stats max rel (entries > 1e-12 max)", float(d[big].max()), "worst index", int(np.argmax(np.where(big, d, 0))))
a, b = out["mfma"], out["bwd2"]
rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
print("N", N, "max rel", float(rel.max()), "mean rel", float(rel.mean()))
bad = np.argwhere(rel > 1e-10)
print("mismatched pairs", len(bad), "of", rel.size)
if len(bad):
    i, j = bad[:, 0], bad[:, 1]
    print("base mod 16 histogram", np.bincount(i % 16, minlength=16).tolist())
    print("cluster histogram", np.bincount(j, minlength=post.K).tolist())
    print("first", bad[:10].tolist(), a[tuple(bad[0])], b[tuple(bad[0])])

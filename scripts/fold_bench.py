"""The exact fallback at full size: a C4 workload whose cluster 0
underflows in the factorised recursion for EVERY base (its transitions put all mass
on sigma + 1 while its emissions favour state 0, SURVEY-style adversarial case), so
the backward pass flags N pairs and the gate-list pass flags them again.  Times the
fused E-step with the fallback folded into resp / statistics kernels (default) and
as separate fb_exact_kernel launches (VBHEM_NO_FOLD_EXACT=1), and checks the two
agree.  Development tool:  python scripts/fold_bench.py [N]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import pkgload  # noqa: E402

vb = pkgload.load()
from vbhem_amd.estep import EStepEngine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
dev = torch.device("cuda", 0)
base, post, opt = vb.synth_workload("C4", device=dev, N=N)
consts = vb.host.cluster_constants(post, base.covmode)
S = post.S
lA = np.full((S, S), -600.0)
for r in range(S):
    lA[r, (r + 1) % S] = 0.0
consts["logA"] = np.array(consts["logA"], copy=True)
consts["logA"][0] = lA
consts["c"] = np.array(consts["c"], copy=True)
consts["c"][0] = 1200.0
consts["c"][0, 0] = -2000.0   # cluster 0 wins every base: gated too
eng = EStepEngine(base, post.K, S, opt["tau"], device=dev)
eng.set_clusters(consts)
eng.set_log_omega(vb.host.log_omega_tilde(post.alpha))
tN = (float(opt["Nv"]) * N) * eng.base.omega
out = {"N": N}
res = {}
for label, env in (("folded", {}), ("separate", {"VBHEM_NO_FOLD_EXACT": "1"})):
    os.environ.pop("VBHEM_NO_FOLD_EXACT", None)
    os.environ.update(env)
    st = eng.fused(tN).clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        st = eng.fused(tN)
    torch.cuda.synchronize()
    out[label + "_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    res[label] = st.cpu().numpy().copy()
    out[label + "_flagged"] = int(eng.fallback_count())
os.environ.pop("VBHEM_NO_FOLD_EXACT", None)
a, b = res["folded"], res["separate"]
out["max_rel_diff"] = float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
print(json.dumps(out))

"""Batched-trials throughput (vbhem_estep_fused_trials): trial-E-steps/s for R
trials in one launch vs one trial per launch, on the C2 / C3 configs (small K,
where one trial leaves the GPU mostly idle).  Synthetic inputs, resident in HBM."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import pkgload

vb = pkgload.load()
from vbhem_amd import host  # noqa: E402
from vbhem_amd.em import _stack_constants  # noqa: E402
from vbhem_amd.estep import EStepEngine  # noqa: E402

dev = torch.device("cuda", 0)
out = []
for cfg, Rs in (("C2", (1, 8, 64)), ("C3", (1, 4, 16, 32))):
    base, post, opt = vb.synth_workload(cfg, device=dev)
    K, S, cov = post.K, post.S, base.covmode
    consts = host.cluster_constants(post, cov)
    logOm = host.log_omega_tilde(post.alpha)
    for R in Rs:
        eng = EStepEngine(base, R * K, S, opt["tau"], device=dev, trials=R)
        eng.set_clusters(_stack_constants([consts] * R))
        eng.set_log_omega(np.concatenate([logOm] * R))
        tN = (float(opt["Nv"]) * base.N) * eng.base.omega
        pin = torch.empty(eng.stats_len, dtype=torch.float64, pin_memory=True)

        def step():
            pin.copy_(eng.fused(tN), non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()

        for _ in range(3):
            step()
        n = 30
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        dt = (time.perf_counter() - t0) / n
        out.append(dict(config=cfg, N=base.N, K=K, S=S, R=R, ms_per_launch=dt * 1e3,
                        trial_estep_per_s=R / dt))
        print(json.dumps(out[-1]), flush=True)

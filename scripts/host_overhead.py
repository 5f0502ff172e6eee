#!/usr/bin/env python3
"""Host-side cost of one fused E-step call (enqueue only) vs its GPU time, at a
small shard (the per-rank size of an 8-GPU strong-scaling run)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 12500
    dev = torch.device("cuda", 0)
    base, post, opt = vb.synth_workload("C4", device=dev, N=N)
    eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
    eng.set_clusters(host.cluster_constants(post, 1))
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    tN = (float(opt["Nv"]) * N) * eng.base.omega
    for _ in range(3):
        eng.fused(tN).cpu()
    torch.cuda.synchronize()
    enq, tot = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        st = eng.fused(tN)
        t1 = time.perf_counter()
        st.cpu()
        t2 = time.perf_counter()
        enq.append(t1 - t0)
        tot.append(t2 - t0)
    print(f"N={N} enqueue {1e3 * sorted(enq)[10]:.3f} ms  step {1e3 * sorted(tot)[10]:.3f} ms (medians)")


if __name__ == "__main__":
    main()

"""Per-step fixed overhead of the fused E-step at shard sizes (experiment)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pkgload
vb = pkgload.load()
from vbhem_amd import _capi, host
from vbhem_amd.estep import EStepEngine

dev = torch.device("cuda", 0)
for N in [int(x) for x in sys.argv[1:]] or [12500, 100000]:
    base, post, opt = vb.synth_workload("C4", device=dev, N=N)
    eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
    eng.set_clusters(host.cluster_constants(post, base.covmode))
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    tN = (float(opt["Nv"]) * N) * eng.base.omega
    pin = torch.empty(eng.stats_len, dtype=torch.float64, pin_memory=True)
    def t_loop(fn, n=50, sync_each=True):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
            if sync_each: torch.cuda.synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3
    r = {}
    r["eager_cpu"] = t_loop(lambda: eng.fused(tN).cpu())
    r["eager_pinned"] = t_loop(lambda: pin.copy_(eng.fused(tN), non_blocking=True))
    r["eager_nosync"] = t_loop(lambda: eng.fused(tN), sync_each=False)
    t0 = time.perf_counter(); [eng.fused(tN) for _ in range(50)]; r["host_enqueue"] = (time.perf_counter() - t0) / 50 * 1e3
    print("N=%d" % N, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}, flush=True)

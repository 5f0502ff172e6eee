#!/usr/bin/env python3
"""Where the idle gap between paced E-steps comes from: ms per E-step over 60 steps
(a) paced as bench.py does (a torch event recorded after each step, the host waiting
on step k-1's event after enqueueing step k), (b) the same with events created
without the system-scope release (hipEventDisableSystemFence; the host still waits on
them), (c) no per-step event, one sync at the end.  Development tool:
python scripts/gap_probe.py [C3|C4] [N]"""
import ctypes
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0)
    base, post, opt = vb.synth_workload(cfg, device=dev, N=N) if N else vb.synth_workload(cfg, device=dev)
    eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
    eng.set_clusters(host.cluster_constants(post, base.covmode))
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    tN = (float(opt["Nv"]) * base.N) * eng.base.omega
    bufs = [eng.host_stats_buffer(), eng.host_stats_buffer()]
    s = torch.cuda.current_stream(dev)
    hip = ctypes.CDLL("libamdhip64.so")
    stream = ctypes.c_void_p(s.cuda_stream)
    nofence = []
    for _ in range(2):
        ev = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(ev), 0x2 | 0x20000000) == 0  # DisableTiming | DisableSystemFence
        nofence.append(ev)
    tev = [torch.cuda.Event(), torch.cuda.Event()]
    for _ in range(10):
        eng.fused(tN, out=bufs[0])
    s.synchronize()
    n = 60
    res = {}
    for mode in ("torch_event", "nofence_event", "no_event", "torch_event", "nofence_event", "no_event"):
        s.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            eng.fused(tN, out=bufs[k % 2])
            if mode == "torch_event":
                tev[k % 2].record(s)
                if k > 0:
                    tev[(k - 1) % 2].synchronize()
            elif mode == "nofence_event":
                hip.hipEventRecord(nofence[k % 2], stream)
                if k > 0:
                    hip.hipEventSynchronize(nofence[(k - 1) % 2])
        s.synchronize()
        res.setdefault(mode, []).append(round((time.perf_counter() - t0) / n * 1e3, 4))
    print(cfg, N, res)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where the host time of one fused E-step goes (medians over 50 calls): the
Python wrapper, the C-ABI call alone (arguments prebuilt), a stream sync on an
idle stream, and the whole step (fused into pinned memory + sync)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(f, n=50):
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e6 * sorted(ts)[n // 2]


def main():
    if os.environ.get("VBHEM_SPIN"):  # spin-wait synchronisation (before the device is set up)
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(int(os.environ["VBHEM_SPIN"])))
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import host, _capi
    from vbhem_amd.estep import EStepEngine
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    dev = torch.device("cuda", 0)
    base, post, opt = vb.synth_workload(cfg, device=dev)
    eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
    eng.set_clusters(host.cluster_constants(post, base.covmode))
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    tN = (float(opt["Nv"]) * base.N) * eng.base.omega
    buf = eng.host_stats_buffer()
    s = torch.cuda.current_stream(dev)
    for _ in range(5):
        eng.fused(tN, out=buf)
    s.synchronize()
    lib = eng.lib
    args = (ctypes.byref(eng._bt), ctypes.byref(eng._ct), eng.T, _capi.ptr(tN), _capi.ptr(eng.logOmega),
            eng._mapped[1], _capi.ptr(eng.hatZ), _capi.ptr(eng.LL), _capi.ptr(eng._ws_fused),
            eng._ws_fused.numel(), eng._stream())

    def py_enq():
        eng.fused(tN, out=buf)
        s.synchronize()

    def c_enq():
        lib.vbhem_estep_fused(*args)
        s.synchronize()

    def full():
        eng.fused(tN, out=buf)
        s.synchronize()

    t_enq_py = []
    t_enq_c = []
    for _ in range(50):
        t0 = time.perf_counter(); eng.fused(tN, out=buf); t_enq_py.append(time.perf_counter() - t0); s.synchronize()
        t0 = time.perf_counter(); lib.vbhem_estep_fused(*args); t_enq_c.append(time.perf_counter() - t0); s.synchronize()
    print(cfg, "enqueue python %.1f us, C call %.1f us" % (1e6 * sorted(t_enq_py)[25], 1e6 * sorted(t_enq_c)[25]))
    print(cfg, "idle sync %.1f us" % med(lambda: s.synchronize()))
    print(cfg, "step via python %.1f us, via prebuilt C args %.1f us" % (med(full), med(c_enq)))
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(s)
    with torch.cuda.stream(side):
        eng.fused(tN, out=buf)
    s.wait_stream(side)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        eng.fused(tN, out=buf)
    torch.cuda.synchronize()

    def gstep():
        g.replay()
        s.synchronize()
    print(cfg, "step via graph replay %.1f us" % med(gstep))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Cost of the MATLAB-facing (host-array) entry points, beside the
device-resident fused E-step that bench.py's `value` measures.

Per config (C2, C3, C4 by default):
  pairs_host  vbhem_estep_pairs_host: what the per-pair MEX drop-in
              (integration/vbhem_hmm_bwd_fwd_mex.c) calls every EM iteration --
              allocate, upload every input, compute, download the six per-pair
              outputs (emit_Mu alone is N*K*S*d*d doubles), free;
  fused_host  vbhem_estep_fused_host: one-shot fused call (base upload + E-step
              + statistics download);
  ctx_fused   vbhem_ctx_fused on a resident context: what the fused MEX gateway
              (integration/vbhem_estep_fused_mex.c) costs per EM iteration after
              the first (cluster constants up, statistics + hat_Z + L_elbo down);
  device      vbhem_estep_fused with everything resident (bench.py's step).
Prints one JSON line per config.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import _capi, host
    from vbhem_amd.estep import EStepEngine
    lib = _capi.lib()
    configs = sys.argv[1:] or ["C2", "C3", "C4"]
    dev = torch.device("cuda", 0)
    for name in configs:
        base, post, opt = vb.synth_workload(name)
        cov, K, S, T = base.covmode, post.K, post.S, opt["tau"]
        consts = host.cluster_constants(post, cov)
        logOm = host.log_omega_tilde(post.alpha)
        bn = {k: np.ascontiguousarray(v) for k, v in base.numpy().items() if isinstance(v, np.ndarray)}
        N, SB, d = base.N, base.SB, base.d
        cn = {k: np.ascontiguousarray(consts[k], dtype=np.float64) for k in ("logA", "logPi", "m", "P", "c")}
        bt = _capi.BaseT(N, SB, d, cov, bn["nstates"].astype(np.int32).ctypes.data, bn["prior"].ctypes.data,
                         bn["A"].ctypes.data, bn["centres"].ctypes.data, bn["covars"].ctypes.data)
        ns = bn["nstates"].astype(np.int32)
        bt.nstates = ns.ctypes.data
        ct = _capi.ClusterT(K, S, *[cn[k].ctypes.data for k in ("logA", "logPi", "m", "P", "c")])
        tN = np.ascontiguousarray((opt["Nv"] * N) * bn["omega"])
        dC = d * d if cov == 1 else d
        res = {"config": name, "N": N, "K": K, "S": S, "d": d}

        def timeit(fn, reps):
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return (time.perf_counter() - t0) / reps * 1e3

        # per-pair drop-in (MEX-equivalent outputs to host memory)
        outs = [np.empty(n) for n in (N * K, N * K * S, N * K * S, N * K * S * d, N * K * S * dC,
                                      N * K * S * S)]

        def pairs_host():
            rc = lib.vbhem_estep_pairs_host(0, ctypes.byref(bt), ctypes.byref(ct), T,
                                            *[o.ctypes.data for o in outs])
            _capi.check(rc, "vbhem_estep_pairs_host")
        res["pairs_host_ms"] = timeit(pairs_host, 2 if name == "C4" else 5)
        res["pairs_host_output_GB"] = sum(o.nbytes for o in outs) / 1e9
        del outs
        L = int(lib.vbhem_stats_len(K, S, d, cov))
        stats = np.empty(L)
        hz = np.empty(N * K)
        ll = np.empty(N * K)

        def fused_host():
            rc = lib.vbhem_estep_fused_host(0, ctypes.byref(bt), ctypes.byref(ct), T, tN.ctypes.data,
                                            logOm.ctypes.data, stats.ctypes.data, hz.ctypes.data,
                                            ll.ctypes.data)
            _capi.check(rc, "vbhem_estep_fused_host")
        res["fused_host_ms"] = timeit(fused_host, 3)
        ctx = ctypes.c_void_p()
        _capi.check(lib.vbhem_ctx_create(0, ctypes.byref(bt), K, S, 1, T, ctypes.byref(ctx)),
                    "vbhem_ctx_create")

        def ctx_fused():
            rc = lib.vbhem_ctx_fused(ctx, ctypes.byref(ct), tN.ctypes.data, logOm.ctypes.data,
                                     stats.ctypes.data, hz.ctypes.data, ll.ctypes.data)
            _capi.check(rc, "vbhem_ctx_fused")
        res["ctx_fused_ms"] = timeit(ctx_fused, 10)

        def ctx_stats_only():
            rc = lib.vbhem_ctx_fused(ctx, ctypes.byref(ct), tN.ctypes.data, logOm.ctypes.data,
                                     stats.ctypes.data, None, None)
            _capi.check(rc, "vbhem_ctx_fused")
        res["ctx_fused_stats_only_ms"] = timeit(ctx_stats_only, 10)
        lib.vbhem_ctx_destroy(ctx)
        eng = EStepEngine(base, K, S, T, device=dev)
        eng.set_clusters(consts)
        eng.set_log_omega(logOm)
        tNd = torch.as_tensor(tN, device=dev)
        pin = torch.empty(eng.stats_len, dtype=torch.float64, pin_memory=True)

        def device_step():
            pin.copy_(eng.fused(tNd), non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
        res["device_fused_ms"] = timeit(device_step, 20)
        print(json.dumps(res), flush=True)
        del eng


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Time the E-step kernels on a config while varying tau (T), to split the
per-step cost of the recursions from the per-pair fixed cost (K1, epilogue).

    python scripts/sweep_T.py [--config C4] [--N 100000] [--T 2 4 6 10 18]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--T", type=int, nargs="+", default=[2, 4, 6, 10, 18])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cov", type=int, default=None, help="override covmode (0 diag, 1 full)")
    args = ap.parse_args()
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import _capi, host
    from vbhem_amd.estep import EStepEngine
    dev = torch.device("cuda", 0)
    name = args.config
    if args.cov is not None:
        vb.CONFIGS[name + "x"] = dict(vb.CONFIGS[name], covmode=args.cov)
        name = name + "x"
    base, post, opt = vb.synth_workload(name, device=dev, N=args.N)
    cov = base.covmode
    consts = host.cluster_constants(post, cov)
    tN = (float(opt["Nv"]) * base.N) * base.omega.to(dev)
    out = []
    for T in args.T:
        eng = EStepEngine(base, post.K, post.S, T, device=dev)
        eng.set_clusters(consts)
        eng.set_log_omega(host.log_omega_tilde(post.alpha))
        eng.fused(tN)
        torch.cuda.synchronize()
        _capi.timing_read()
        _capi.timing_enable(True)
        for _ in range(args.reps):
            eng.fused(tN)
        torch.cuda.synchronize()
        _capi.timing_enable(False)
        t = _capi.timing_read()
        rec = dict(T=T, fb_ms=t["fb_ms"] / max(1, t["fb_launches"]),
                   stats_ms=t["stats_ms"] / max(1, t["stats_launches"]),
                   fallbacks=eng.fallback_count())
        out.append(rec)
        print(json.dumps(rec), flush=True)
        del eng
        torch.cuda.empty_cache()
    if len(out) >= 2:
        a, b = out[0], out[-1]
        per = (b["fb_ms"] - a["fb_ms"]) / (b["T"] - a["T"])
        print(json.dumps({"per_step_ms": per, "fixed_ms": a["fb_ms"] - per * (a["T"] - 1)}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""A/B of the gated-statistics kernels in one process: the fused E-step on a config
under several environment settings (read per launch by vbhem_stats.hip), statistics
time per step from the library's event timing.

    python scripts/stats_sweep.py [--config C4] [--N n] ENV=VAL,ENV=VAL ...   ('-' = defaults)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import _capi, host
    from vbhem_amd.estep import EStepEngine
    dev = torch.device("cuda", 0)
    base, post, opt = vb.synth_workload(args.config, device=dev, N=args.N)
    consts = host.cluster_constants(post, base.covmode)
    tN = (float(opt["Nv"]) * base.N) * base.omega.to(dev)
    eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
    eng.set_clusters(consts)
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    ref = None
    keys = set()
    for rnd in range(2):  # two rounds: the second shows the spread
        for st in args.settings:
            env = {} if st == "-" else dict(kv.split("=") for kv in st.split(","))
            keys |= set(env)
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            out = eng.fused(tN).clone()
            torch.cuda.synchronize()
            if ref is None:
                ref = out
            err = float(((out - ref).abs() / ref.abs().clamp_min(1e-30)).max())
            t0 = time.perf_counter()
            for _ in range(args.reps):
                eng.fused(tN)
            torch.cuda.synchronize()
            step_ms = (time.perf_counter() - t0) * 1e3 / args.reps
            _capi.timing_read()
            _capi.timing_enable(True)
            for _ in range(args.reps):
                eng.fused(tN)
            torch.cuda.synchronize()
            _capi.timing_enable(False)
            t = _capi.timing_read()
            print(json.dumps(dict(round=rnd, setting=st, step_ms=step_ms, stats_ms=t["stats_ms"] / args.reps,
                                  fb_ms=t["fb_ms"] / args.reps, max_rel_vs_first=err)), flush=True)


if __name__ == "__main__":
    main()

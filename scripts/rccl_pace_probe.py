"""Which part of bench.py's multi-rank E-step tail breaks the one-step run-ahead?

One rank, a 12,500-base shard of C4 (rank 0 of 8), 60 E-steps per variant, each paced
two ways: pipelined (step k + 1 enqueued before the host waits for step k's event, as
bench.py / the C++ EM loop) and synchronous (the host waits for every step).
Variants of the step's tail after eng.fused:
  plain     statistics written straight into pinned host memory (out=hs)
  copy      device statistics, then hs.copy_(st, non_blocking=True)
  rccl      device statistics, one-rank RCCL all-reduce, no copy
  rccl+copy device statistics, RCCL all-reduce, then the copy (bench.py's multi-rank path)
  rccl+out  RCCL all-reduce of a side vector, statistics straight into pinned memory
  +timing   the same with bench.py's kernel timing on every 4th step (fb_only events)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import pkgload
    vb = pkgload.load()
    from vbhem_amd import _capi, host
    from vbhem_amd.dist import RcclComm
    from vbhem_amd.estep import EStepEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = vb.CONFIGS["C4"]
    N = int(os.environ.get("PROBE_N", "100000"))
    lo, hi = 0, N // 8
    base, post, opt = vb.synth_workload("C4", device=dev, N=N, shard=(lo, hi))
    eng = EStepEngine(base, cfg["K"], cfg["S"], cfg["tau"], device=dev)
    eng.set_clusters(host.cluster_constants(post, cfg["covmode"]))
    eng.set_log_omega(host.log_omega_tilde(post.alpha))
    tN = (float(opt["Nv"]) * N) * eng.base.omega
    rccl = RcclComm(dev)
    hbufs = [eng.host_stats_buffer(), eng.host_stats_buffer()]
    side = torch.zeros_like(eng.stats)
    done = [torch.cuda.Event(), torch.cuda.Event()]
    stream = torch.cuda.current_stream(dev)

    def launch(k, v):
        timed = v.endswith("+timing") and k % 4 == 0
        v = v.replace("+timing", "")
        if timed:
            _capi.timing_enable(True, fb_only=True)
        hs = hbufs[k % 2]
        if v == "plain":
            eng.fused(tN, out=hs)
        elif v == "rccl+out":
            rccl.allreduce(side)
            eng.fused(tN, out=hs)
        else:
            st = eng.fused(tN)
            if "rccl" in v:
                rccl.allreduce(st)
            if "copy" in v:
                hs.copy_(st, non_blocking=True)
        if timed:
            _capi.timing_enable(False)
        done[k % 2].record(stream)

    steps = 60
    for v in ("plain", "rccl+copy", "plain+timing", "copy+timing", "rccl+timing", "rccl+copy+timing"):
        for _ in range(5):
            launch(0, v)
            stream.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(steps):
            launch(s, v)
            if s > 0:
                done[(s - 1) % 2].synchronize()
        torch.cuda.synchronize()
        tp = (time.perf_counter() - t0) / steps * 1e3
        t0 = time.perf_counter()
        for s in range(steps):
            launch(s, v)
            stream.synchronize()
        ts = (time.perf_counter() - t0) / steps * 1e3
        _capi.timing_read()
        print("%-17s pipelined %.4f ms  synchronous %.4f ms" % (v, tp, ts), flush=True)
    rccl.close()


if __name__ == "__main__":
    main()

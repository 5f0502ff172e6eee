#!/usr/bin/env python3
"""bench.py -- VBHEM-H3M E-steps/sec on MI355X (whole node).

One step = one E-step of the hot path on this rank's shard of base HMMs:
the fused HIP E-step (all N_shard x K pair recursions, responsibilities,
gated Z-weighted statistic reduction, ELBO partials), the RCCL all-reduce of
the packed statistics across ranks, and the statistics' copy to the host
(what the M-step consumes).  Inputs are synthetic and
resident in HBM before the timed region.

Single GPU:   python bench.py [--steps K --warmup W --config C4]
Multi GPU:    python bench.py --gpus N   (starts N rank processes itself), or
              python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 dense (vector and matrix), AMD spec
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)
# sustained v_fma_f64 throughput measured on MI355X by scripts/ubench_valu.hip (4 waves
# per SIMD, 8 independent chains, 40,000 iterations): 2.40 ns per wave-instruction per
# SIMD = 54.6 TF/s (profiles/r02_ubench_valu.txt)
ACHIEVABLE_FP64_VALU_TFLOPS = 54.6
METRIC = ("VBHEM E-steps/sec (whole node), N baseHMMs × K clusters × S states; "
          "ELBO match")


def flops_per_pair(S, Sb, d, T, covmode):
    """Algorithmic flops of one (base, cluster) pair, counted on the reference
    recurrences (exp/log excluded): K1 + K2 + K4 + K3/K5."""
    if covmode == 1:
        k1 = 2 * Sb * S * (2 * d * d + d)
        k5 = 2 * S * Sb * (1 + d + d * d)
    else:
        k1 = 2 * Sb * S * (3 * d)
        k5 = 2 * S * Sb * (1 + 2 * d)
    return k1 + fb_flops_per_pair(S, Sb, T) + k5


def fb_flops_per_pair(S, Sb, T):
    """The part fb_split_kernel executes: K2 backward + K3 termination + K4
    forward (K1 runs in emission_kernel, K5 in stats_kernel)."""
    return bwd_flops_per_pair(S, Sb, T) + fwd_flops_per_pair(S, Sb, T)


def bwd_flops_per_pair(S, Sb, T):
    """K2 backward + K3 termination (the gated schedule's first pass, every pair)."""
    return (T - 1) * S * (2 * S * Sb + 2 * Sb * Sb + S * Sb) + 2 * S * Sb


def fwd_flops_per_pair(S, Sb, T):
    """K4 forward (the gated schedule's second pass, gated pairs only)."""
    return (T - 1) * (2 * S * Sb * Sb + 3 * S * S * Sb)


def emission_flops_per_pair(S, Sb, d, covmode):
    """K1 as executed by emission_kernel: a GEMM with inner dimension KD."""
    kd = d * (d + 1) // 2 + d if covmode == 1 else 2 * d
    return 2 * S * Sb * kd


def transcendentals_per_pair(S, Sb, T):
    """exp/log count of the reference algorithm per pair (T*S^2*Sb exp, T*S*Sb log)."""
    return T * S * S * Sb, T * S * Sb


def fb_bytes_per_pair(S, Sb, d, covmode, K, split=True, backward_only=False, k1_fused=False):
    """Algorithmic HBM bytes of one fb-kernel pair.  Split path: its 1/K share
    of the base transitions/prior + its E tile (emission_kernel output) + its
    outputs (LL, nu_1, sum_xi, sum_t_nu; LL alone for the backward pass).
    With K1 inside the kernel (k1_fused) the 1/K share of the base's prepared
    operand U (Sb x kdp doubles) replaces the E tile.  Generic path: base
    emissions instead of E."""
    out = 8 if backward_only else (1 + S + S * S + S * Sb) * 8
    if split and k1_fused:
        kd = d * (d + 1) // 2 + d if covmode == 1 else 2 * d
        kdp = (kd + 3) // 4 * 4
        return (Sb + Sb * Sb + Sb * kdp) * 8 / K + out
    if split:
        return (Sb + Sb * Sb) * 8 / K + S * Sb * 8 + out
    dC = d * d if covmode == 1 else d
    return (Sb + Sb * Sb + Sb * d + Sb * dC) * 8 / K + out


def committed_traffic(config, N, world, want):
    """HBM bytes per launch of the roofline kernel from the newest committed PMC
    summary for this config (profiles/rNN_<config>.json, made by
    scripts/profile.sh + scripts/prof_summary.py; FETCH_SIZE x2 + WRITE_SIZE per
    MI355X_MICROARCH.md).  The counters cannot be collected inside the timed
    run, so the value is read back here; None when no summary matches.  The
    full-size launches are taken alone when the summary separates them (a bench
    run under the profiler also launches the kernel at the shard size)."""
    import glob
    import re

    def tag_order(path):  # r04z < r04z3 < r04z4 (a plain sort puts r04z_ last)
        m = re.match(r"r(\d+)([a-z]*)(\d*)_", os.path.basename(path))
        return (int(m.group(1)), m.group(2), int(m.group(3) or 0)) if m else (-1, "", 0)

    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{config.lower()}.json")), key=tag_order)
    short = want.split("::")[-1].split("<")[0]
    for path in reversed(cands):
        try:
            with open(path) as f:
                summ = json.load(f)
        except (OSError, ValueError):
            continue
        if summ.get("N") not in (None, N) or summ.get("n_gpus", 1) != world:
            continue
        full = summ.get("full_size_launches", {}).get(short, {})
        if "hbm_bytes" in full:
            return full["hbm_bytes"]["traffic"], os.path.relpath(path, ROOT) + " (full-size launches)"
        if not summ.get("pmc_full_size_only"):
            continue    # PMC passes that mixed launch sizes: not this kernel's traffic
        kern = summ.get("kernels", {})
        # the exact name, else the same kernel under another template argument (the
        # fb_bwd4_kernel<O32> versions, or a summary from before the template)
        for name in [want] + [n for n in kern if n.split("<")[0] == want.split("<")[0] and n != want]:
            k = kern.get(name, {})
            if "hbm_bytes_per_launch" in k:
                return k["hbm_bytes_per_launch"]["traffic"], os.path.relpath(path, ROOT)
    return None, None


def host_cpu():
    """(nproc, CPU model) of the host this process runs on (the GPU box's cores)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 1, model


def cpu_baseline(vo, base_np, consts, T, N_total, K, target_s):
    """Time the oracle's C port of mex.c (1 thread) + responsibilities + stats
    on a bounded sample of bases and scale linearly to N_total."""
    import numpy as np

    def sub(n):
        return {k: (v[:n] if isinstance(v, np.ndarray) else v) for k, v in base_np.items()}

    def run(n):
        b = sub(n)
        t0 = time.perf_counter()
        pr = vo.c_estep_pairs(b, consts, T, nthreads=1)
        tn = np.full(n, 100.0)
        hz, Z = vo.c_responsibilities(pr["LL_elbo"], tn, np.log(np.full(K, 1.0 / K)))
        vo.c_statistics(Z, pr, b["covmode"])
        return time.perf_counter() - t0, pr

    n0 = min(4, base_np["prior"].shape[0])
    t0, _ = run(n0)
    n = int(min(base_np["prior"].shape[0], max(n0, target_s / max(t0 / n0, 1e-9))))
    t, pr = run(n)
    # the same sample with the pairs spread over the host cores this process may use
    # (the MEX itself is single-threaded; reported beside the baseline, not as it)
    threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
    b = sub(n)
    tm0 = time.perf_counter()
    prm = vo.c_estep_pairs(b, consts, T, nthreads=threads)
    tnm = np.full(n, 100.0)
    hzm, Zm = vo.c_responsibilities(prm["LL_elbo"], tnm, np.log(np.full(K, 1.0 / K)))
    vo.c_statistics(Zm, prm, b["covmode"])
    tm = time.perf_counter() - tm0
    nproc, model = host_cpu()
    multi = dict(value=1.0 / (tm * N_total / n), unit="E-steps/s", cores=threads, kind="port",
                 sample=f"the same {n}-base sample, pairs over {threads} OpenMP threads ({tm:.2f} s)",
                 host_nproc=nproc, host_cpu=model,
                 note=("threads = OMP_NUM_THREADS, which the GPU box sets to the one-GPU job's "
                       "CPU share (16 of its logical CPUs; the others belong to the other GPUs' "
                       "jobs); the reference MEX itself is single-threaded"))
    return dict(value=1.0 / (t * N_total / n), unit="E-steps/s", cores=1, kind="port",
                sample=(f"oracle/vbhem_oracle.c (C port of the reference mex.c E-step, 1 thread) + "
                        f"responsibilities + statistics on {n} of {N_total} base HMMs x {K} clusters "
                        f"({t:.1f} s), scaled linearly to N={N_total}; host: {nproc} logical CPUs, "
                        f"{model}"),
                host_nproc=nproc, host_cpu=model,
                seconds=t, n_sample=n, multi=multi), pr, n


def rank_launch_command(n, argv, port):
    """The torch.distributed.run command that starts n rank processes of this script
    with the same arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def resolve_world(gpus, env):
    """How this process runs, from --gpus and the launcher's environment:
    ("launch", n) -- no WORLD_SIZE and n > 1 ranks asked for: start them;
    ("rank", world) -- one rank of a world of `world` processes.
    A --gpus that disagrees with WORLD_SIZE is refused (ValueError)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else int(gpus)
        if n < 1:
            raise ValueError(f"--gpus {n}: at least one GPU")
        return ("launch", n) if n > 1 else ("rank", 1)
    world = int(ws)
    if gpus is not None and int(gpus) != world:
        raise ValueError(f"--gpus {gpus} disagrees with WORLD_SIZE={world} set by the launcher")
    return ("rank", world)


def launch_ranks(n, argv):
    """Start n rank processes as children (torch.distributed.run) and return their
    exit status.  Runs before anything in this process touches the GPU; the
    parent only waits (never exec: see the box rules on processes that have
    initialised the GPU)."""
    backend = os.environ.get("VBHEM_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        import torch  # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible; RCCL needs one GPU per "
                  f"rank (VBHEM_BENCH_BACKEND=gloo rehearses several ranks on fewer GPUs)",
                  file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(rank_launch_command(n, argv, port), env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE set, N > 1 starts them")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--N", type=int, default=None, help="override the number of base HMMs")
    ap.add_argument("--tau", type=int, default=None, help="override tau (experiments only)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity-sample", action="store_true")
    ap.add_argument("--parity-seconds", type=float, default=4.0)
    ap.add_argument("--em-iters", type=int, default=10,
                    help="EM iterations timed for the em_iteration block (0: skip)")
    ap.add_argument("--no-shard-sim", action="store_true",
                    help="skip the single-GPU run at the 8-GPU shard size (N/8 bases)")
    ap.add_argument("--settle-ms", type=float, default=600.0,
                    help="untimed E-steps, run-ahead as in the timed region, for at least this "
                         "long before the warmup steps: the GPU's clocks settle (0: none)")
    args = ap.parse_args()
    try:
        mode, world = resolve_world(args.gpus, os.environ)
    except ValueError as ex:
        print(f"bench.py: {ex}", file=sys.stderr)
        return 2
    if mode == "launch":
        return launch_ranks(world, sys.argv[1:])

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    # one rank per GPU over RCCL ("nccl"); VBHEM_BENCH_BACKEND=gloo rehearses the
    # multi-rank path with several ranks sharing the GPUs there are (host-staged)
    backend = os.environ.get("VBHEM_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import pkgload
    vb = pkgload.load()
    from vbhem_amd import _capi, host
    from vbhem_amd.dist import make_allreduce, shard_range
    from vbhem_amd.estep import EStepEngine

    cfg = vb.CONFIGS[args.config]
    N = args.N or cfg["N"]
    K, S, Sb, d, T, cov = cfg["K"], cfg["S"], cfg["Sb"], cfg["d"], cfg["tau"], cfg["covmode"]
    if args.tau is not None:
        T = args.tau
    lo, hi = shard_range(N, rank, world)
    base, post, opt = vb.synth_workload(args.config, device=dev, N=N, shard=(lo, hi))
    eng = EStepEngine(base, K, S, T, device=dev)
    consts = host.cluster_constants(post, cov)
    logOm = host.log_omega_tilde(post.alpha)
    eng.set_clusters(consts)
    eng.set_log_omega(logOm)
    tN = (float(opt["Nv"]) * N) * eng.base.omega
    allreduce = make_allreduce()
    # the native collective: an RCCL communicator of our own (include/vbhem_dist.h),
    # all-reduced in-stream by the C++ EM loop and by the E-steps below; torch's
    # process group then only carries the barriers and the timing maxima
    rccl, rccl_err = None, None
    # (VBHEM_BENCH_RCCL_ONE: a one-rank communicator on a one-GPU run, to rehearse the path)
    if ((world > 1 and backend == "nccl") or os.environ.get("VBHEM_BENCH_RCCL_ONE")) \
            and not os.environ.get("VBHEM_BENCH_NO_RCCL"):
        from vbhem_amd.dist import RcclComm
        try:
            rccl = RcclComm(dev)
        except Exception as ex:  # noqa: BLE001 -- reported, then torch's RCCL path
            rccl_err = repr(ex)
        ok = torch.tensor([0.0 if rccl is None else 1.0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() < 1.0 and rccl is not None:
            rccl.close()
            rccl = None
    # the statistics land in pinned host memory (what the host M-step reads): one
    # rank writes them there straight from the statistics kernel; several ranks
    # all-reduce the device vector, then copy it
    # two of them: with one E-step of run-ahead the next step writes the other one
    hbufs = [eng.host_stats_buffer(), eng.host_stats_buffer()]
    try:  # the buffers' device addresses (the kernel copy after the all-reduce)
        hs_dev = [eng.stats_address(h) for h in hbufs]
    except Exception:  # noqa: BLE001 -- not mappable here: the stream copy instead
        hs_dev = None
    host_stats = hbufs[0]
    done = [torch.cuda.Event(), torch.cuda.Event()]
    stream = torch.cuda.current_stream(dev)

    # the collective's own time, taken only in the instrumented breakdown pass (never
    # in the timed region): HIP events around the in-stream RCCL call, or the host
    # clock around a host-staged (gloo) all-reduce
    ar_timing = {"on": False, "ms": []}

    def collective(st, k, hs):
        if ar_timing["on"]:
            if rccl is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            else:
                torch.cuda.synchronize()
                h0 = time.perf_counter()
        if rccl is not None and hs_dev is not None:
            # reduced, then written into the pinned buffer by a kernel on the same
            # stream (a hipMemcpy here broke the run-ahead: 0.34 -> 0.63 ms per
            # 12,500-base step, profiles/r04v2_rccl_pacing.txt)
            rccl.allreduce_to(st, hs_dev[k % 2])
        elif rccl is not None:
            rccl.allreduce(st)
        else:
            allreduce(st)
        if ar_timing["on"]:
            if rccl is not None:
                e1.record(stream)
                e1.synchronize()
                ar_timing["ms"].append(e0.elapsed_time(e1))
            else:
                torch.cuda.synchronize()
                ar_timing["ms"].append((time.perf_counter() - h0) * 1e3)
        if not (rccl is not None and hs_dev is not None):
            hs.copy_(st, non_blocking=True)

    # one rank: the E-step's last kernel stores a ticket into a coherent pinned word
    # once the statistics are in host memory (vbhem_arm_done_word), and the host polls
    # it -- no event after each step: an event is a queue marker that idles the GPU
    # ~5.7 us per E-step (12,500-base trace, gpurun_out/prof_r06l_shard).  With a
    # collective the statistics are final only after it: an event there.
    word = (eng.done_word() if world == 1 and rccl is None and not os.environ.get("VBHEM_BENCH_COPY")
            and not os.environ.get("VBHEM_BENCH_EVENT") else None)
    tickets = [0, 0]
    seq = [0]

    def launch(k):
        """Enqueue E-step k: statistics into pinned host buffer k % 2, then its ticket
        (or an event)."""
        hs = hbufs[k % 2]
        if world == 1 and rccl is None and not os.environ.get("VBHEM_BENCH_COPY"):
            if word is not None:
                seq[0] += 1
                tickets[k % 2] = seq[0]
                eng.fused(tN, out=hs, done=(word, seq[0]))
                return hs
            eng.fused(tN, out=hs)
        else:
            collective(eng.fused(tN), k, hs)
        done[k % 2].record(stream)
        return hs

    def wait(k):
        """The host waits for E-step k's statistics."""
        if word is not None:
            word.wait(tickets[k % 2])
        else:
            done[k % 2].synchronize()

    def step():
        """One E-step, the host waiting for its statistics before anything else."""
        hs = launch(0)
        stream.synchronize()
        return hs

    # clock settling: the card reaches its steady clocks only after ~0.5 s of
    # sustained work (C4, same box: 1.84 ms per timed step after 5 warmup steps,
    # 1.795 ms after 300 -- gpurun_out/r06j); the untimed steps below run the timed
    # region's own protocol for --settle-ms, then the W warmup steps follow as before
    # (several ranks: every E-step has a collective, so all ranks run the same step
    # count -- from one timed step, the largest over the ranks -- not a time limit)
    settle = {"ms": 0.0, "steps": 0}
    if args.settle_ms > 0:
        ts = time.perf_counter()
        n = 0
        if world > 1:
            step()  # (the first one pays the communicator's lazy setup)
            t1s = time.perf_counter()
            step()
            nset = torch.tensor([min(20000, int(args.settle_ms / max(1e-3, (time.perf_counter() - t1s) * 1e3)) + 1)],
                                dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(nset, op=dist.ReduceOp.MAX)
            nset = int(nset.item())
            for n in range(nset):
                launch(n)
                if n > 0:
                    wait(n - 1)
            n = nset + 1
        else:
            while (time.perf_counter() - ts) * 1e3 < args.settle_ms:
                launch(n)
                if n > 0:
                    wait(n - 1)
                n += 1
        torch.cuda.synchronize()
        settle = {"ms": (time.perf_counter() - ts) * 1e3, "steps": n}
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    _capi.timing_read()  # drop warmup records
    # inside the timed region only the fb launches are timed (two HIP events on the
    # launch stream around the roofline's kernel) and only in every TIME_EVERY-th
    # E-step: an event record is a queue marker that costs ~5 us of idle GPU on
    # each side of the kernel (10 us of a 160 us C3 step).  The per-kernel
    # breakdown comes from a separate instrumented pass below.
    time_every = 1 if args.steps < 8 else 4
    # E-steps as the C++ EM loop issues them (vbhem_em_run): step k + 1 is enqueued
    # before the host waits for step k's statistics (one step of run-ahead), so the
    # GPU does not idle while the host takes a step's statistics and launches the
    # next; every step's statistics still reach pinned host memory and are waited for
    t0 = time.perf_counter()
    for s in range(args.steps):
        if s % time_every == 0:
            _capi.timing_enable(True, fb_only=True)
        stats = launch(s)
        if s % time_every == 0:
            _capi.timing_enable(False)
        if s > 0:
            wait(s - 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    stats = stats.clone()
    _capi.timing_enable(False)
    if world > 1:
        dist.barrier()
    dt = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    per_rank_s = [float(dt.item())]
    if world > 1:
        gath = [torch.zeros_like(dt) for _ in range(world)]
        dist.all_gather(gath, dt)
        per_rank_s = [float(g.item()) for g in gath]
    dt = max(per_rank_s)
    tk = _capi.timing_read()
    # the same steps with the host waiting on each before launching the next (the
    # rate of an E-step whose statistics must be on the host before anything else)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ts0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dts = torch.tensor([time.perf_counter() - ts0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dts, op=dist.ReduceOp.MAX)
    dts = float(dts.item())
    # per-kernel breakdown (emission, gated forward, statistics): a few more E-steps
    # with every launch timed (not part of `value`)
    bd_steps = max(1, min(args.steps, 5))
    _capi.timing_enable(True)
    ar_timing["on"] = True
    for _ in range(bd_steps):
        step()
    torch.cuda.synchronize()
    ar_timing["on"] = False
    tkb = _capi.timing_read()
    _capi.timing_enable(False)
    # the kernels the library launched for the two recursion passes (named by the launch)
    bwd_kernel_launched, list_kernel_launched = _capi.last_kernel(0), _capi.last_kernel(1)
    # the all-reduce's time per E-step on every rank (breakdown pass), max over ranks
    ar_ms = float(np.mean(ar_timing["ms"])) if ar_timing["ms"] else None
    per_rank_ar = [ar_ms]
    if world > 1:
        t_ = torch.tensor([ar_ms if ar_ms is not None else -1.0], dtype=torch.float64, device=dev)
        gath = [torch.zeros_like(t_) for _ in range(world)]
        dist.all_gather(gath, t_)
        per_rank_ar = [float(g.item()) if g.item() >= 0 else None for g in gath]
    # fraction of pairs the gate Z > 1e-8 keeps (the gated schedule's second pass)
    zk = (eng.hatZ * tN.view(-1, 1)) > 1e-8
    n_gated = int(zk.sum().item())
    if world > 1:
        ng = torch.tensor([n_gated], dtype=torch.float64, device=dev)
        dist.all_reduce(ng)
        n_gated = int(ng.item())

    # the dense schedule (both sweeps for every pair, same outputs) on the same
    # inputs, for reference: a few steps, reported beside `value`, then its fb
    # kernel (K2-K4 for every pair) timed alone for its roofline fraction
    dense_steps = max(1, min(args.steps, 5))
    prev_mode = _capi.set_fused_mode(_capi.FUSED_DENSE)
    step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    td0 = time.perf_counter()
    for _ in range(dense_steps):
        dstats = step()
    torch.cuda.synchronize()
    dstats = dstats.clone()
    dtd = torch.tensor([time.perf_counter() - td0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dtd, op=dist.ReduceOp.MAX)
    _capi.timing_read()
    _capi.timing_enable(True, fb_only=True)
    for _ in range(dense_steps):
        step()
    torch.cuda.synchronize()
    tkd = _capi.timing_read()
    _capi.timing_enable(False)
    dense_kernel_launched = _capi.last_kernel(0)
    _capi.set_fused_mode(prev_mode)
    dense_rel = float((dstats - stats).abs().max() / stats.abs().max().clamp_min(1e-300))

    # one whole EM iteration as an EM loop pays it (the C++ loop, vbhem_em_run): the
    # E-step, the all-reduce, the statistics' copy to the host, the bound, the M-step
    # and the next iteration's psi prelude + constant upload
    def em_iteration(engine, n_total):
        """Per-iteration cost of the C++ EM loop (vbhem_em_run_ext).  Primary: the
        loop's own host clock -- the time at which each iteration's bound reaches
        the host -- over one long run, the median of the per-iteration differences
        after the first two.  Beside it the median of 5 paired differences
        (t(run of 1 + n iterations) - t(run of 1)) / n, where the per-run set-up
        (posterior upload, result copies) cancels."""
        if args.em_iters <= 0:
            return None
        from vbhem_amd import native_em
        o = dict(opt, minDiff=0.0)          # no early stop: exactly max_iter + 1 iterations
        kw = dict(total_N=n_total, allreduce=None if rccl else allreduce, comm=rccl)

        def timed(n, stamps=False):
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            r = native_em.run(post, engine, o, max_iter=n, timestamps=stamps, **kw)
            torch.cuda.synchronize()
            dt_ = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(dt_, op=dist.ReduceOp.MAX)
            return float(dt_.item()), r

        timed(1)
        n_long = max(20, 4 * args.em_iters)
        _, rl = timed(n_long, stamps=True)
        steps = np.diff(rl.iter_seconds)[2:] * 1e3
        ms_loc = float(np.median(steps))
        if world > 1:   # the slowest rank's clock
            t_ = torch.tensor([ms_loc], dtype=torch.float64, device=dev)
            dist.all_reduce(t_, op=dist.ReduceOp.MAX)
            ms_loc = float(t_.item())
        pairs = []
        for _ in range(5):
            t_a, ra = timed(1)
            t_b, rb = timed(1 + args.em_iters)
            pairs.append((t_b - t_a) / max(1, rb.iters - ra.iters) * 1e3)
        # the loop's per-iteration math kernel (bound + M-step + next prelude on the
        # device), timed with events in one more run
        _capi.timing_read()
        _capi.timing_enable(True)
        timed(1 + args.em_iters)
        _capi.timing_enable(False)
        tm = _capi.timing_read()
        math_ms = tm["em_math_ms"] / tm["em_math_launches"] if tm["em_math_launches"] else None
        return dict(ms=ms_loc, per_s=1e3 / ms_loc, iterations=int(steps.size),
                    iteration_ms_p10_p90=[float(np.percentile(steps, 10)),
                                          float(np.percentile(steps, 90))],
                    paired_diff_ms=float(np.median(pairs)), paired_diff_all_ms=pairs,
                    math_kernel_ms=math_ms,
                    collective=("RCCL in the loop (vbhem_rccl_allreduce_sum, %d ranks)" % world
                                if rccl else ("torch.distributed callback" if world > 1 else "none")),
                    method=("median of the per-iteration differences of the loop's own host clock "
                            "(vbhem_em_run_ext iter_seconds) over a %d-iteration run, iterations 3.. ; "
                            "paired_diff_ms: median of 5 x (t(run of %d) - t(run of 1)) / %d"
                            % (n_long + 1, 1 + args.em_iters + 1, args.em_iters)))

    em_it = em_iteration(eng, N)
    step()   # hat_Z / L_elbo of the bench's own constants again (the EM run moved them)

    # host math of one EM iteration in C++ (vbhem_em_host_iteration: bound, M-step,
    # next prelude; replicated on every rank), and the Python host path for reference
    from vbhem_amd import native_em
    hst = stats.numpy().copy()
    hi = native_em.HostIteration(post, opt, cov)
    hi(hst)
    nrep = 200
    th0 = time.perf_counter()
    for _ in range(nrep):
        hi(hst)
    host_ms = (time.perf_counter() - th0) / nrep * 1e3
    th0 = time.perf_counter()
    st = host.unpack_stats(hst, K, S, d, cov)
    Nj = st["Nj"] + 1e-50
    L = host.lower_bound(st["Lt1"], st["Lt7"], Nj, logOm, post, consts, opt, cov)
    host.mstep(host.finish_statistics(st, cov), Nj, opt, cov, post.W0mode)
    host.cluster_constants(post, cov)
    host_py_ms = (time.perf_counter() - th0) * 1e3

    # strong-scaling simulation on this GPU: rank 0's shard of an 8-GPU run (the
    # first N/8 bases of the same N-base set), E-step and EM iteration
    shard_sim = None
    if world == 1 and not args.no_shard_sim and N >= 8 * 64:
        ns = N // 8
        base_s, _, _ = vb.synth_workload(args.config, device=dev, N=N, shard=(0, ns))
        eng_s = EStepEngine(base_s, K, S, T, device=dev)
        eng_s.set_clusters(consts)
        eng_s.set_log_omega(logOm)
        tN_s = (float(opt["Nv"]) * N) * eng_s.base.omega
        hs = [eng_s.host_stats_buffer(), eng_s.host_stats_buffer()]
        ev_s = [torch.cuda.Event(), torch.cuda.Event()]
        for _ in range(3):
            eng_s.fused(tN_s, out=hs[0])
            stream.synchronize()
        # the timed region's pacing: one step of run-ahead, the host waiting for each
        # step's statistics by the completion word (or an event, as above)
        word_s = eng_s.done_word() if word is not None else None
        seq_s = [0]

        def run_ahead(n=None, ms=None):
            t0 = time.perf_counter()
            k = 0
            tick = [0, 0]
            while (k < n) if n is not None else ((time.perf_counter() - t0) * 1e3 < ms):
                if word_s is not None:
                    seq_s[0] += 1
                    tick[k % 2] = seq_s[0]
                    eng_s.fused(tN_s, out=hs[k % 2], done=(word_s, seq_s[0]))
                else:
                    eng_s.fused(tN_s, out=hs[k % 2])
                    ev_s[k % 2].record(stream)
                if k > 0:
                    if word_s is not None:
                        word_s.wait(tick[(k - 1) % 2])
                    else:
                        ev_s[(k - 1) % 2].synchronize()
                k += 1
            stream.synchronize()
            return time.perf_counter() - t0

        # the clocks settle again (the host-side math above left the GPU idle)
        if args.settle_ms > 0:
            run_ahead(ms=args.settle_ms)
        nss = max(20, args.steps)
        es_ms = run_ahead(n=nss) / nss * 1e3
        ts0 = time.perf_counter()
        for _ in range(nss):
            eng_s.fused(tN_s, out=hs[0])
            stream.synchronize()
        es_sync_ms = (time.perf_counter() - ts0) / nss * 1e3
        em_s = em_iteration(eng_s, N)
        shard_sim = {"bases": ns, "estep_ms": es_ms,
                     "estep_ceiling_8gpu": (dt / args.steps * 1e3) / es_ms,
                     "estep_sync_ms": es_sync_ms,
                     "estep_sync_ceiling_8gpu": (dts / args.steps * 1e3) / es_sync_ms,
                     "em_iteration": em_s,
                     "em_ceiling_8gpu_excl_allreduce": (em_it["ms"] / em_s["ms"]
                                                        if em_it and em_s else None),
                     "note": ("one GPU running rank 0's shard of an 8-GPU strong-scaling run; "
                              "the ceilings divide the full-N time by the shard time and leave "
                              "out the RCCL all-reduce of the packed statistics")}
        del eng_s

    if rank != 0:
        if rccl is not None:
            rccl.close()
        if world > 1:
            dist.destroy_process_group()
        return

    fb_launch_ms = tk["fb_ms"] / max(1, tk["fb_launches"])
    pairs_per_launch = tk["fb_pairs"] / max(1, tk["fb_launches"])
    split = S <= 16 and Sb <= S and d <= 64
    gated = split and tkb["gated_fwd_launches"] > 0
    # K1 inside the recursion kernels (fb_bwd2_kernel and fb_split_kernel's list mode, short
    # K1 inner dimension): no emission GEMM launch was timed
    k1_fused = gated and tkb["em_launches"] == 0
    if gated:
        fpp = bwd_flops_per_pair(S, Sb, T)
        if k1_fused:
            fpp += emission_flops_per_pair(S, Sb, d, cov)
    else:
        fpp = fb_flops_per_pair(S, Sb, T) if split else flops_per_pair(S, Sb, d, T, cov)
    achieved = fpp * pairs_per_launch / (fb_launch_ms * 1e-3) / 1e12
    bpp = fb_bytes_per_pair(S, Sb, d, cov, K, split, backward_only=gated, k1_fused=k1_fused)
    n_exp, n_log = transcendentals_per_pair(S, Sb, T)
    kname = bwd_kernel_launched
    traffic, traffic_src = committed_traffic(args.config, N, world, kname)
    # the gate-list pass: one launch per base group (14 at C5's N = 10^6); its rate is the
    # step's gated pairs over the step's summed list-pass time
    gf_launches_per_step = tkb["gated_fwd_launches"] / bd_steps
    gf_ms = tkb["gated_fwd_ms"] / max(1, tkb["gated_fwd_launches"])
    gf_step_ms = tkb["gated_fwd_ms"] / bd_steps
    dense_ms = tkd["fb_ms"] / max(1, tkd["fb_launches"])
    dense_fpp = fb_flops_per_pair(S, Sb, T) if split else flops_per_pair(S, Sb, d, T, cov)
    dense_ach = dense_fpp * tkd["fb_pairs"] / max(1, tkd["fb_launches"]) / (dense_ms * 1e-3) / 1e12
    res = {
        "metric": METRIC,
        "value": args.steps / dt,
        "unit": "E-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": dict(settle, note="untimed run-ahead E-steps before the warmup steps, "
                                    "until the clocks settle (--settle-ms)"),
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (BASELINE.md generator, seeded), resident in HBM",
        "config": {"workload": (f"{args.config}: N={N} base HMMs, K={K} clusters, S={S} states, "
                                f"Sb={Sb}, d={d}, {'full' if cov == 1 else 'diag'} cov, tau={T}, "
                                f"Nv={opt['Nv']}"),
                   "N": N, "K": K, "S": S, "Sb": Sb, "d": d, "tau": T,
                   "parallelism": f"bases sharded over {world} GPU(s), 1 RCCL all-reduce/E-step"},
        "collective": dict(
            ({"kind": ("native RCCL communicator (vbhem_rccl_allreduce_to: all-reduce, then "
                       "an in-stream kernel copy into the pinned statistics buffer)"
                       if hs_dev is not None else
                       "native RCCL communicator (vbhem_rccl_allreduce_sum, then a stream copy)"),
              "ranks": world}
             if rccl is not None else
             {"kind": ("torch.distributed all_reduce (%s backend)" % backend
                       if world > 1 else "none (one rank)"),
              "ranks": world, "rccl_error": rccl_err}),
            allreduce_ms=(max(a for a in per_rank_ar if a is not None)
                          if any(a is not None for a in per_rank_ar) else None),
            allreduce_ms_per_rank=per_rank_ar,
            allreduce_timing=("HIP events around the in-stream all-reduce call (+ its copy to "
                              "the pinned buffer), mean over the %d-step breakdown pass; max over "
                              "ranks" % bd_steps if rccl is not None else
                              "host clock around the host-staged all-reduce with device syncs, "
                              "mean over the %d-step breakdown pass; max over ranks" % bd_steps
                              if world > 1 else None),
            statistics_doubles=int(stats.numel()),
            shard_bases_per_rank=[shard_range(N, r, world)[1] - shard_range(N, r, world)[0]
                                  for r in range(world)],
            ms_per_step_per_rank=[s / args.steps * 1e3 for s in per_rank_s]),
        "pacing": ("one E-step of run-ahead (the C++ EM loop's): step k+1 is enqueued before "
                   "the host waits for step k's statistics in pinned memory"
                   + (" -- by polling the completion word the step's last kernel writes "
                      "(vbhem_arm_done_word)" if word is not None else " -- by an event")),
        "synchronous": {"value": args.steps / dts, "ms_per_step": dts / args.steps * 1e3,
                        "note": "the host waits for each step's statistics before launching "
                                "the next (no overlap of the host hand-over)"},
        "pairs_per_s": N * K * args.steps / dt,
        "roofline": {
            # the compute roof (the contract's "mfma"): fp64 dense, 78.6 TF/s, the same for
            # v_mfma_f64 and the vector ALU; see the note for which unit runs what
            "bound": "mfma",
            "achieved": achieved,
            "peak": PEAK_FP64_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP64_TFLOPS,
            "achievable_peak": ACHIEVABLE_FP64_VALU_TFLOPS,
            "frac_of_achievable": achieved / ACHIEVABLE_FP64_VALU_TFLOPS,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": kname,
            "kernel_ms": fb_launch_ms,
            "timed_launches": tk["fb_launches"],
            "timed_every_nth_step": time_every,
            "flops_per_pair": fpp,
            "pairs_per_launch": pairs_per_launch,
            "note": (("fp64 issue-bound: the recursion's contractions on v_mfma_f64_4x4x4f64, the "
                      "software exp/log on the VALU (the two do not co-issue)"
                      if ("bwd4" in kname or "bwd12" in kname) else
                      "fp64 VALU-bound (software exp/log + contractions on the vector ALU)") +
                     "; peak = MI355X FP64 dense "
                     "78.6 TF/s (vector = matrix rate); achievable_peak = the sustained "
                     "v_fma_f64 rate measured on this chip by scripts/ubench_valu.hip "
                     "(4 waves/SIMD, independent chains); flops counted on the reference "
                     "recurrences this kernel runs (" + ("K1 emission GEMM + " if k1_fused else "")
                     + ("K2 backward + K3 termination, every "
                     "pair" if gated else "K2-K4") + "), excluding exp/log"),
            "hbm": {"algorithmic_bytes_per_launch": bpp * pairs_per_launch,
                    "achieved_GBs": bpp * pairs_per_launch / (fb_launch_ms * 1e-3) / 1e9,
                    "peak_GBs": PEAK_HBM_GBS,
                    "frac": bpp * pairs_per_launch / (fb_launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS},
            "exp_log_per_pair_reference": [n_exp, n_log],
        },
        "schedule": "gated" if gated else "dense",
        "metric_definition": ("one E-step = every (base, cluster) pair's backward recursion and "
                              "L_elbo, hat_Z, the gated statistics (vbhem_compute_Statistics.m:35 "
                              "keeps pairs with Z > 1e-8; the forward sweep runs for those pairs "
                              "only, the reference computes it for all and discards the rest), the "
                              "ELBO partials, the all-reduce and the copy to the host; outputs "
                              "equal the dense schedule's (dense_schedule.max_rel_diff_vs_gated)"),
        "gated_pairs_frac": n_gated / float(N * K),
        "gated_forward": ({"kernel": list_kernel_launched,
                           "kernel_ms": gf_ms,
                           "launches_per_step": gf_launches_per_step,
                           "ms_per_step": gf_step_ms,
                           "pairs_per_step": n_gated / world,
                           "flops_per_pair": fb_flops_per_pair(S, Sb, T),
                           "achieved_TFLOPs": fb_flops_per_pair(S, Sb, T) * n_gated / world
                           / max(gf_step_ms * 1e-3, 1e-12) / 1e12,
                           "note": "achieved = the step's gated pairs (this rank) x K2-K4 flops "
                                   "over the step's summed list-pass launch time"}
                          if gated else None),
        "dense_schedule": {"value": dense_steps / float(dtd.item()), "unit": "E-steps/s",
                           "steps": dense_steps, "max_rel_diff_vs_gated": dense_rel,
                           "fb_kernel": dense_kernel_launched,
                           "fb_kernel_ms": dense_ms,
                           "roofline_frac": dense_ach / PEAK_FP64_TFLOPS,
                           "achieved_TFLOPs": dense_ach,
                           "flops_per_pair": dense_fpp},
        "emission_kernel_ms": tkb["em_ms"] / max(1, tkb["em_launches"]),
        "k1_in_backward": k1_fused,
        "k1_note": ("K1 (the emission GEMM, mex.c:715-865) runs inside the recursion kernels "
                    "(fb_bwd2_kernel, fb_split_kernel list mode; kdp <= 8 fmas per entry): no emission "
                    "kernel, no E buffer; emission_kernel_ms is 0" if k1_fused else
                    "K1 in emission_u_kernel (E written to HBM, read by the recursion)"),
        "stats_kernels_ms_per_step": tkb["stats_ms"] / bd_steps,
        "breakdown_steps": bd_steps,
        "em_math_kernel_ms": em_it["math_kernel_ms"] if em_it else None,
        "em_math_note": ("the per-iteration math of the EM loop (vbhem_em_run: bound, M-step, "
                         "next psi prelude) as the loop runs it: one device kernel on the "
                         "E-step stream, replicated on every rank, HIP-event timed; "
                         "host_math_cpp_ms: the same math in C++ on the host "
                         "(vbhem_em_host_iteration, the loop's path for d > 16 or S > 32), "
                         "host_math_python_ms: the Python host path"),
        "host_math_cpp_ms": host_ms,
        "host_math_python_ms": host_py_ms,
        "em_iteration": em_it,
        "shard_sim": shard_sim,
        "elbo": L,
    }
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import vbhem_oracle as vo  # cpu_baseline leg only
        base_np = eng.base.numpy() if hasattr(eng.base, "numpy") else base.numpy()
        cb, pr, n = cpu_baseline(vo, base_np, consts, T, N, K, args.cpu_seconds)
        res["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample",
                                                  "host_nproc", "host_cpu")}
        res["cpu_baseline_multithread"] = cb["multi"]
        res["speedup_vs_cpu"] = res["value"] / cb["value"]
    if world == 1 and not args.no_parity_sample:
        # the checker on bases spread evenly over all N (every base group of a large
        # run), 16 host threads, ~ --parity-seconds of CPU: L_elbo and hat_Z of the
        # bench's own E-step (hat_Z of a base depends on its own L_elbo row only)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import vbhem_oracle as vo  # checker only
        base_np = eng.base.numpy() if hasattr(eng.base, "numpy") else base.numpy()
        thr = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
        t0p = time.perf_counter()
        vo.c_estep_pairs(vo.base_subset(base_np, slice(0, 8)), consts, T, nthreads=1)
        per_base = (time.perf_counter() - t0p) / 8 / max(1, thr)
        nps = int(min(N, max(16, args.parity_seconds / max(per_base, 1e-9))))
        idx = np.unique(np.linspace(0, N - 1, nps).astype(np.int64))
        ref = vo.c_estep_pairs(vo.base_subset(base_np, idx), consts, T, nthreads=thr)
        hz_ref, _ = vo.c_responsibilities(ref["LL_elbo"], tN.cpu().numpy()[idx], logOm)
        g = eng.LL.cpu().numpy()[idx]
        hz = eng.hatZ.cpu().numpy()[idx]
        ll_err = float(np.max(np.abs(g - ref["LL_elbo"]) /
                              np.maximum(np.abs(ref["LL_elbo"]), 1e-300)))
        hz_big = hz_ref > 1e-8
        hz_err = float(max(np.max(np.abs(hz - hz_ref)[hz_big] / hz_ref[hz_big], initial=0.0),
                           np.max(np.abs(hz - hz_ref)[~hz_big], initial=0.0)))
        res["parity_sample"] = {"LL_elbo_max_rel_err": ll_err, "hat_Z_max_err": hz_err,
                                "pairs": int(idx.size * K), "bases": int(idx.size),
                                "sample": ("bases evenly spaced over all N (every base group), "
                                           "oracle/vbhem_oracle.c on %d host threads" % thr),
                                "tolerance": {"LL_elbo": 1e-10, "hat_Z": 1e-5}}
    print(json.dumps(res))
    if rccl is not None:
        rccl.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)

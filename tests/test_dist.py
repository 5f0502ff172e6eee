"""Multi-rank EM (vbhem_amd.dist + vbhem_amd.em) on the CPU with gloo.

Each rank owns a contiguous shard of base HMMs and runs the E-step on it (the
oracle stand-in engine here, the HIP engine on GPUs); the packed statistics are
SUM-all-reduced once per iteration.  All ranks must end with identical
posteriors, equal to a single-process run up to summation order.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cases import post_dict  # noqa: F401  (ensures tests/ is importable in workers)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_em(name, N, world, rank, outdir, port):
    import torch
    import torch.distributed as dist

    import pkgload
    from oracle_engine import OracleEngine

    vb = pkgload.load()
    from vbhem_amd.dist import make_allreduce, shard_range
    from vbhem_amd.em import vbhem_h3m_c_step_fc

    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    base, P, opt = vb.synth_workload(name, N=N)
    lo, hi = shard_range(N, rank, world)
    eng = OracleEngine(base.shard(lo, hi), P.K, P.S, opt["tau"], nthreads=1)
    res = vbhem_h3m_c_step_fc(P, eng, dict(opt, max_iter=8), total_N=N,
                              allreduce=make_allreduce())
    np.savez(os.path.join(outdir, f"r{rank}_w{world}.npz"), LogLs=np.array(res.LogLs),
             m=res.post.m, W=res.post.W, alpha=res.post.alpha, epsilon=res.post.epsilon,
             hatZ=res.hatZ.numpy(), lo=lo, hi=hi)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    del torch


def _worker(rank, name, N, world, outdir, port):
    _run_em(name, N, world, rank, outdir, port)


@pytest.mark.slow
@pytest.mark.parametrize("name", ["C2", "C3"])
def test_gloo_two_ranks_match_single_process(tmp_path, name):
    N = 30
    _run_em(name, N, 1, 0, str(tmp_path), 0)
    port = _free_port()
    mp.spawn(_worker, args=(name, N, 2, str(tmp_path), port), nprocs=2, join=True)
    single = np.load(tmp_path / "r0_w1.npz")
    r0 = np.load(tmp_path / "r0_w2.npz")
    r1 = np.load(tmp_path / "r1_w2.npz")
    for k in ("LogLs", "m", "W", "alpha", "epsilon"):
        np.testing.assert_array_equal(r0[k], r1[k])         # replicated host math
        np.testing.assert_allclose(r0[k], single[k], rtol=1e-10, err_msg=k)
    hz = np.concatenate([r0["hatZ"], r1["hatZ"]])
    np.testing.assert_allclose(hz, single["hatZ"], rtol=1e-9, atol=1e-300)
    assert int(r0["hi"]) == int(r1["lo"])


def _run_trials(N, world, rank, outdir, port):
    import torch.distributed as dist

    import pkgload
    from oracle_engine import OracleEngine

    vb = pkgload.load()
    from vbhem_amd.dist import make_allreduce, shard_range
    from vbhem_amd.em import vbhem_h3m_c_trials

    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    base, P, opt = vb.synth_workload("C2", N=N)
    posts = [P.copy()]
    for r in (1, 2):
        Q = P.copy()
        rng = np.random.default_rng(r)
        Q.m = Q.m + rng.normal(0.0, 0.5, Q.m.shape)
        posts.append(Q)
    lo, hi = shard_range(N, rank, world)
    eng = OracleEngine(base.shard(lo, hi), 3 * P.K, P.S, opt["tau"], nthreads=1, trials=3)
    tr = vbhem_h3m_c_trials(posts, eng, dict(opt, max_iter=6), total_N=N,
                            allreduce=make_allreduce())
    np.savez(os.path.join(outdir, f"t{rank}_w{world}.npz"), LLall=tr.LLall, best=tr.best,
             m=np.stack([r.post.m for r in tr.results]),
             LogLs=np.stack([np.pad(r.LogLs, (0, 7 - len(r.LogLs))) for r in tr.results]))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _trials_worker(rank, N, world, outdir, port):
    _run_trials(N, world, rank, outdir, port)


@pytest.mark.slow
def test_gloo_two_ranks_batched_trials(tmp_path):
    """Batched trials (one statistics vector of R sections, one all-reduce per
    iteration) on 2 gloo ranks vs one process."""
    N = 30
    _run_trials(N, 1, 0, str(tmp_path), 0)
    port = _free_port()
    mp.spawn(_trials_worker, args=(N, 2, str(tmp_path), port), nprocs=2, join=True)
    single = np.load(tmp_path / "t0_w1.npz")
    r0, r1 = np.load(tmp_path / "t0_w2.npz"), np.load(tmp_path / "t1_w2.npz")
    for k in ("LLall", "m", "LogLs"):
        np.testing.assert_array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], single[k], rtol=1e-10, err_msg=k)
    assert int(r0["best"]) == int(single["best"])


def _rccl_id_worker(rank, world, port, outdir):
    import torch.distributed as dist

    import pkgload
    pkgload.load()
    from vbhem_amd.dist import RcclComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = RcclComm.exchange_id(rank, world)
    with open(os.path.join(outdir, f"id{rank}.bin"), "wb") as f:
        f.write(uid)
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_id_exchange_two_ranks_gloo(tmp_path):
    """The native communicator's set-up (dist.RcclComm.exchange_id): rank 0's RCCL
    id (vbhem_rccl_unique_id, which needs no GPU) reaches every rank of a gloo
    group unchanged -- the bytes every rank then hands to ncclCommInitRank."""
    world = 2
    mp.spawn(_rccl_id_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ids = [open(tmp_path / f"id{r}.bin", "rb").read() for r in range(world)]
    assert len(ids[0]) == 128 and ids[0] == ids[1] and any(ids[0])


def _ready_worker(rank, world, port, bad_rank, outdir):
    import torch.distributed as dist

    import pkgload
    pkgload.load()
    from vbhem_amd import _capi
    from vbhem_amd.dist import RcclComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # this rank's own readiness (RCCL bound, device visible), faked so the test needs
    # neither a GPU nor RCCL: rank bad_rank cannot take part
    RcclComm.local_status = staticmethod(lambda dev: "no RCCL here" if rank == bad_rank else None)
    msg = "ok"
    try:
        RcclComm.check_ranks_ready(rank, world, 0)
    except _capi.VbhemError as ex:
        msg = str(ex)
    with open(os.path.join(outdir, f"ready{rank}.txt"), "w") as f:
        f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("bad_rank", [None, 1])
def test_rccl_readiness_agreed_before_init(tmp_path, bad_rank):
    """RcclComm's set-up gathers every rank's readiness before any rank enters
    ncclCommInitRank: when one rank (here the non-zero one) cannot bind RCCL, every
    rank raises naming it, instead of rank 0 waiting for it forever."""
    world = 2
    mp.spawn(_ready_worker, args=(world, _free_port(), bad_rank, str(tmp_path)), nprocs=world,
             join=True)
    msgs = [open(tmp_path / f"ready{r}.txt").read() for r in range(world)]
    if bad_rank is None:
        assert msgs == ["ok", "ok"]
    else:
        assert all("rank 1: no RCCL here" in m for m in msgs), msgs

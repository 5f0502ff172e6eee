"""The C++ EM loop (vbhem_em_run, include/vbhem_em.h) on 2 ranks: each rank runs
the device E-step on its shard of base HMMs and the loop's all-reduce callback
(vbhem_allreduce_fn) SUM-reduces the packed statistics over a gloo process group
(host-staged), once per iteration -- the --gpus N path of bench.py with the C++
loop in place of the Python one.  Both ranks share cuda:0 (one GPU per box), so
this checks the exchange and the replicated host math, not xGMI.

All ranks must end with identical posteriors and bounds, equal to one process
over the whole base set up to the all-reduce's summation order."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(name, N, world, rank, outdir, port, iters):
    import torch
    import torch.distributed as dist

    import pkgload
    vb = pkgload.load()
    from vbhem_amd import native_em
    from vbhem_amd.dist import shard_range
    from vbhem_amd.estep import EStepEngine

    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = [0]

    def allreduce(t):  # host-staged gloo all-reduce of the device statistics
        calls[0] += 1
        if world == 1:
            return
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM)
        t.copy_(h)

    base, P, opt = vb.synth_workload(name, N=N)
    lo, hi = shard_range(N, rank, world)
    eng = EStepEngine(base.shard(lo, hi), P.K, P.S, opt["tau"], device="cuda:0")
    res = native_em.run(P, eng, dict(opt, max_iter=iters), total_N=N, allreduce=allreduce)
    torch.cuda.synchronize()
    np.savez(os.path.join(outdir, f"r{rank}_w{world}.npz"), LogLs=np.array(res.LogLs),
             m=res.post.m, W=res.post.W, alpha=res.post.alpha, epsilon=res.post.epsilon,
             eta=res.post.eta, hatZ=res.hatZ.cpu().numpy(), L_elbo=res.L_elbo.cpu().numpy(),
             iters=res.iters, calls=calls[0], lo=lo, hi=hi)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _worker(rank, name, N, world, outdir, port, iters):
    _run(name, N, world, rank, outdir, port, iters)


@pytest.mark.parametrize("name,N", [("C3", 2000), ("C4", 1000), ("C4", 1003)])
def test_native_em_two_ranks_gloo(tmp_path, name, N):
    import torch.multiprocessing as mp
    iters = 4
    _run(name, N, 1, 0, str(tmp_path), 0, iters)
    mp.spawn(_worker, args=(name, N, 2, str(tmp_path), _free_port(), iters), nprocs=2, join=True)
    single = np.load(tmp_path / "r0_w1.npz")
    r0, r1 = np.load(tmp_path / "r0_w2.npz"), np.load(tmp_path / "r1_w2.npz")
    assert int(r0["iters"]) == int(r1["iters"]) == int(single["iters"])
    # one callback per E-step on every rank
    assert int(r0["calls"]) == int(r1["calls"]) == int(single["calls"]) >= int(single["iters"])
    for k in ("LogLs", "m", "W", "alpha", "epsilon", "eta"):
        np.testing.assert_array_equal(r0[k], r1[k], err_msg=k)      # replicated host math
        np.testing.assert_allclose(r0[k], single[k], rtol=1e-10, err_msg=k)
    assert int(r0["hi"]) == int(r1["lo"]) and int(r1["hi"]) == N
    # the shards' responsibilities and bounds are the single run's rows
    for k, tol in (("hatZ", 1e-8), ("L_elbo", 1e-10)):
        got = np.concatenate([r0[k], r1[k]])
        np.testing.assert_allclose(got, single[k], rtol=tol, atol=1e-300, err_msg=k)

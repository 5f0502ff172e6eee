"""The EM host loop in C++ (include/vbhem_em.h, vbhem_amd.native_em).

CPU: each host step of the library (psi prelude, M-step, lower bound) against
the Python host path (vbhem_amd.host, itself checked against the oracle's
restatement of the MATLAB code) on oracle-generated statistics.
GPU: the whole loop (vbhem_em_run) against the Python EM loop on the device
E-step, and against the oracle EM (north-star tolerance)."""
import numpy as np
import pytest

from cases import make_case
from conftest import RTOL_NORTH_STAR, hatz_err, post_err, rel_err


def packed_stats(vb, vo, cs, cov):
    """The fused E-step's packed vector [Nj | N1 | M | Lt1 Lt7 | U], built from the oracle."""
    base, consts, post, T = cs["base"], cs["consts"], cs["post"], cs["T"]
    N = base["prior"].shape[0]
    K, S = consts["logPi"].shape
    d = base["centres"].shape[2]
    pairs = vo.c_estep_pairs(base, consts, T)
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, post["alpha"])
    st = vo.c_statistics(Z, pairs, cov)
    NU = vb.host.stats_nu(d, cov)
    U = np.zeros((K, S, NU))
    U[..., 0] = st["Nr"]
    U[..., 1:1 + d] = st["Y"]
    if cov == 1:
        iu = np.triu_indices(d)
        U[..., 1 + d:] = st["SC"][..., iu[0], iu[1]]
    else:
        U[..., 1 + d:] = st["SC"]
    Lt1 = float((Z * pairs["LL_elbo"]).sum())
    Lt7 = float((hz * np.log(hz)).sum())
    vec = np.concatenate([st["Nj"], st["N1"].ravel(), st["M"].ravel(), [Lt1, Lt7], U.ravel()])
    assert vec.size == vb.host.stats_len(K, S, d, cov)
    return vec


CASES = [("full", 1, 3), ("diag", 0, 3), ("full_S1", 1, 1)]


@pytest.mark.parametrize("name,cov,S", CASES, ids=[c[0] for c in CASES])
def test_prelude_matches_host(vb, name, cov, S):
    from vbhem_amd import native_em
    cs = make_case(6, 3, S, 3, 3, cov, seed=11 + cov)
    got = native_em.prelude(cs["P"], cov)
    ref = vb.host.cluster_constants(cs["P"], cov)
    for k in ("logA", "logPi", "m", "P", "c", "logLambdaTilde"):
        assert rel_err(got[k], ref[k]) < 1e-13, k
    assert rel_err(got["logOmega"], vb.host.log_omega_tilde(cs["P"].alpha)) < 1e-14


@pytest.mark.parametrize("name,cov,S", CASES, ids=[c[0] for c in CASES])
def test_mstep_and_bound_match_host(vb, vo, name, cov, S):
    from vbhem_amd import native_em
    cs = make_case(8, 3, S, 3, 3, cov, seed=21 + cov, tau=6)
    K, d = 3, 3
    vec = packed_stats(vb, vo, cs, cov)
    P, opt = cs["P"], cs["opt"]
    # M-step
    got = native_em.mstep(vec, P, opt, cov)
    st = vb.host.unpack_stats(vec, K, S, d, cov)
    ref = vb.host.mstep(vb.host.finish_statistics(st, cov), st["Nj"] + 1e-50, opt, cov, P.W0mode)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert rel_err(getattr(got, k), getattr(ref, k)) < 1e-12, k
    # lower bound
    consts = vb.host.cluster_constants(P, cov)
    logOm = vb.host.log_omega_tilde(P.alpha)
    Lref = vb.host.lower_bound(st["Lt1"], st["Lt7"], st["Nj"] + 1e-50, logOm, P, consts, opt, cov)
    Lgot = native_em.lower_bound(vec, P, opt, cov, dict(consts, logOmega=logOm))
    assert abs(Lgot - Lref) <= 1e-11 * abs(Lref)


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [1, 0])
def test_native_em_matches_python_em(vb, cov):
    """vbhem_em_run (C++ loop) vs em.vbhem_h3m_c_step_fc (Python loop), same device E-step."""
    import torch
    from vbhem_amd import native_em
    from vbhem_amd.em import vbhem_h3m_c_step_fc
    from vbhem_amd.estep import EStepEngine
    cs = make_case(300, 4, 3, 3, 2, cov, seed=31 + cov, tau=8)
    opt = dict(cs["opt"], max_iter=6)
    e1 = EStepEngine(cs["bs"], 4, 3, 8, device="cuda:0")
    ref = vbhem_h3m_c_step_fc(cs["P"], e1, opt)
    e2 = EStepEngine(cs["bs"], 4, 3, 8, device="cuda:0")
    got = native_em.run(cs["P"], e2, opt)
    assert got.iters == ref.iters and got.stable == ref.stable
    np.testing.assert_allclose(got.LogLs, ref.LogLs, rtol=1e-11)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert rel_err(getattr(got.post, k), getattr(ref.post, k)) < 1e-10, k
    assert torch.equal(got.label, ref.label)


@pytest.mark.gpu
def test_native_em_c4_slice_vs_oracle(vb, vo):
    """Three EM iterations on a 2,000-base C4 slice: the C++ loop vs the oracle EM."""
    from vbhem_amd import native_em
    from vbhem_amd.estep import EStepEngine
    from cases import post_dict
    base, P, opt = vb.synth_workload("C4", N=2000)
    opt = dict(opt, max_iter=3)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device="cuda:0")
    res = native_em.run(P, eng, opt)
    ref = vo.em_step_fc(post_dict(P), base.numpy(), opt)
    np.testing.assert_allclose(res.LogLs, ref["LogLs"], rtol=RTOL_NORTH_STAR)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert post_err(getattr(res.post, k), ref["post"][k]) < RTOL_NORTH_STAR, k


@pytest.mark.parametrize("name,cov,S", CASES, ids=[c[0] for c in CASES])
def test_host_iteration_matches_steps(vb, vo, name, cov, S):
    """vbhem_em_host_iteration (one call: bound, M-step, next prelude) equals the
    three host steps in sequence, and a NaN bound leaves the posterior untouched."""
    from vbhem_amd import native_em
    cs = make_case(8, 3, S, 3, 3, cov, seed=51 + cov, tau=6)
    vec = packed_stats(vb, vo, cs, cov)
    P, opt = cs["P"], cs["opt"]
    hi = native_em.HostIteration(P, opt, cov)
    L = hi(vec)
    pre = native_em.prelude(P, cov)
    assert L == native_em.lower_bound(vec, P, opt, cov, pre)
    post1 = native_em.mstep(vec, P, opt, cov)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert np.array_equal(hi.pb.a[k], getattr(post1, k)), k
    pre1 = native_em.prelude(post1, cov)
    for k, v in pre1.items():
        assert np.array_equal(hi.pre[k], v), k
    bad = vec.copy()
    K = 3
    bad[K + K * S + K * S * S] = np.nan          # Lt1
    before = {k: v.copy() for k, v in hi.pb.a.items()}
    assert np.isnan(hi(bad))
    for k, v in before.items():
        assert np.array_equal(hi.pb.a[k], v, equal_nan=True), k


@pytest.mark.gpu
def test_native_em_timestamps_and_reused_buffers(vb):
    """vbhem_em_run_ext's per-iteration host clock: one stamp per accepted
    iteration, increasing; repeated runs on one engine reuse its workspace (no
    per-run allocation) and give identical results."""
    from vbhem_amd import native_em
    from vbhem_amd.estep import EStepEngine
    cs = make_case(300, 4, 3, 3, 2, 1, seed=33, tau=8)
    opt = dict(cs["opt"], max_iter=6, minDiff=0.0)
    eng = EStepEngine(cs["bs"], 4, 3, 8, device="cuda:0")
    r1 = native_em.run(cs["P"], eng, opt, timestamps=True)
    ws = eng._em_ws
    r2 = native_em.run(cs["P"], eng, opt, timestamps=True)
    assert eng._em_ws is ws
    assert r1.iters == r2.iters == 7 and r1.LogLs == r2.LogLs
    for r in (r1, r2):
        t = r.iter_seconds
        assert t.shape == (r.iters,) and np.all(np.diff(t) > 0) and t[0] > 0


@pytest.mark.gpu
def test_native_em_rccl_one_rank(vb):
    """The in-loop RCCL all-reduce (RcclComm, vbhem_rccl_*) on a one-rank
    communicator: the statistics pass through ncclAllReduce every E-step and the
    run equals the run without a collective bit for bit."""
    import torch
    from vbhem_amd import native_em
    from vbhem_amd.dist import RcclComm
    from vbhem_amd.estep import EStepEngine
    cs = make_case(300, 4, 3, 3, 2, 1, seed=34, tau=8)
    opt = dict(cs["opt"], max_iter=5)
    eng = EStepEngine(cs["bs"], 4, 3, 8, device="cuda:0")
    ref = native_em.run(cs["P"], eng, opt)
    comm = RcclComm(torch.device("cuda", 0), rank=0, world=1)
    try:
        got = native_em.run(cs["P"], eng, opt, comm=comm)
        x = torch.arange(10, dtype=torch.float64, device="cuda:0")
        comm.allreduce(x)
        torch.cuda.synchronize()
        assert torch.equal(x, torch.arange(10, dtype=torch.float64, device="cuda:0"))
        # allreduce_to (bench.py's multi-rank E-step tail): the reduced statistics
        # written by a kernel into the engine's pinned host buffer
        st = eng.fused(torch.full((300,), 100.0, dtype=torch.float64, device="cuda:0"))
        want = st.clone()
        hs = eng.host_stats_buffer()
        hs.fill_(-1.0)
        comm.allreduce_to(st, eng.stats_address(hs))
        torch.cuda.synchronize()
        assert torch.equal(hs, want.cpu()) and torch.equal(st, want)
    finally:
        comm.close()
    assert got.iters == ref.iters and got.LogLs == ref.LogLs
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert np.array_equal(getattr(got.post, k), getattr(ref.post, k)), k
    with pytest.raises(ValueError):
        native_em.run(cs["P"], eng, opt, comm=comm, allreduce=lambda t: None)


@pytest.mark.gpu
def test_native_em_unstable_device_path(vb, monkeypatch):
    """A NaN bound on the device EM path (the next iteration already queued): the
    run stops unstable with L = -inf, the posterior is the one before the failing
    iteration's M-step, and hat_Z is that iteration's -- as the host-math path
    (VBHEM_EM_HOST_MATH) gives."""
    import torch
    from vbhem_amd import native_em
    from vbhem_amd.estep import EStepEngine
    cs = make_case(200, 3, 3, 3, 2, 1, seed=35, tau=6)
    P = cs["P"].copy()
    P.alpha[0] = np.nan          # logOmega NaN -> every bound NaN from iteration 0
    opt = dict(cs["opt"], max_iter=5)
    eng = EStepEngine(cs["bs"], 3, 3, 6, device="cuda:0")
    dev = native_em.run(P, eng, opt, calc_deriv=True)
    hz_dev = dev.hatZ.clone()
    monkeypatch.setenv("VBHEM_EM_HOST_MATH", "1")
    host = native_em.run(P, eng, opt, calc_deriv=True)
    for r in (dev, host):
        assert not r.stable and r.LL == -np.inf and r.iters == 0 and r.LogLs == []
        assert all(np.isnan(np.atleast_1d(v)).all() for v in r.dLL.values())
    for k in ("eta", "epsilon", "lam", "v", "m", "W"):
        assert np.array_equal(getattr(dev.post, k), getattr(P, k)), k
        assert np.array_equal(getattr(host.post, k), getattr(P, k)), k
    assert torch.equal(torch.isnan(hz_dev), torch.isnan(host.hatZ))
    torch.testing.assert_close(torch.nan_to_num(hz_dev), torch.nan_to_num(host.hatZ), rtol=1e-12,
                               atol=0)

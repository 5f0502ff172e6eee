"""Host-side math of the product package (vbhem_amd.host / h3m / em) against
the oracle's loop-style restatements of the MATLAB sources (CPU only)."""
import numpy as np
import pytest
import torch

from cases import make_case, post_dict
from conftest import RTOL_NORTH_STAR, rel_err
from oracle_engine import OracleEngine, pack_stats


def random_vbhmms(n, S_max, d, seed, with_none=True):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        if with_none and k == 1:
            out.append(None)
            continue
        S = int(rng.integers(1, S_max + 1))
        L = rng.normal(size=(S, d, d))
        covs = L @ np.swapaxes(L, 1, 2) + 0.3 * np.eye(d)
        out.append(dict(prior=rng.dirichlet(np.ones(S)), trans=rng.dirichlet(np.ones(S), size=S),
                        pdf=[dict(mean=rng.normal(size=d), cov=covs[s]) for s in range(S)],
                        varpar=dict(alpha=rng.uniform(1, 30, S), epsilon=rng.uniform(1, 50, (S, S)),
                                    beta=rng.uniform(2, 100, S))))
    return out


@pytest.mark.parametrize("cov", [0, 1])
@pytest.mark.parametrize("use_post", [True, False])
def test_hmms_to_h3m_hem(vb, vo, cov, use_post):
    hmms = random_vbhmms(6, 4, 3, seed=4, with_none=True)
    got = vb.hmms_to_h3m_hem(hmms, covmode=cov, use_post=use_post).numpy()
    ref = vo.hmms_to_h3m_hem(hmms, cov, use_post=use_post)
    for k in ("nstates", "prior", "A", "centres", "covars", "omega"):
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-14, atol=0, err_msg=k)
    assert got["omega"][1] == 0.0 and abs(got["omega"].sum() - 1) < 1e-15


def test_default_options_reject_small_v0(vb):
    with pytest.raises(ValueError):
        vb.default_options(4, 3, 8, v0=5.0)
    vb.default_options(4, 3, 8, v0=10.0)


def test_clip_hyps(vb, vo):
    opt = vb.default_options(3, 2, 2, alpha0=1e20, eta0=1e-20, W0=np.array([1e-30, 2.0]))
    a = vb.clip_hyps(opt)
    b = vo.clip_hyps(opt)
    for k in ("alpha0", "eta0", "epsilon0", "v0", "lambda0", "W0"):
        np.testing.assert_array_equal(np.asarray(a[k]), np.asarray(b[k]))
    assert a["alpha0"] == 1.0686e13 and a["eta0"] == 1.0686e-13


@pytest.mark.parametrize("cov", [0, 1])
def test_baseem_init(vb, vo, cov):
    bs = vb.synth_base_set(20, 3, 4, 3, cov, seed=3, ragged=True)
    opt = vb.default_options(3, 4, 3, covmode=cov)
    rb, rg, om = vb.baseem_draws(bs, 3, 4, seed=9)
    assert (rg < bs.nstates.numpy()[rb]).all()
    got = post_dict(vb.baseem_init(bs, opt, rb, rg, om))
    ref = vo.baseem_init(bs.numpy(), opt, rb, rg, om)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-13, err_msg=k)


@pytest.mark.parametrize("cov", [0, 1])
def test_cluster_constants(vb, vo, cov):
    cs = make_case(4, 5, 4, 3, 3, cov, seed=2)
    got = vb.host.cluster_constants(cs["P"], cov)
    ref = vo.prelude(cs["post"], cov)
    for k in ("logLambdaTilde", "c", "logA", "logPi", "m", "P"):
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-13, atol=1e-13, err_msg=k)


def _oracle_stats(vo, cs, tN):
    cov = cs["base"]["covmode"]
    pairs = vo.c_estep_pairs(cs["base"], cs["consts"], cs["T"])
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, cov)
    return pairs, logOmega, hz, Z, Nj, st


@pytest.mark.parametrize("cov", [0, 1])
def test_stats_layout_roundtrip(vb, vo, cov):
    K, S, d = 3, 4, 3
    cs = make_case(10, K, S, 3, d, cov, seed=6)
    tN = 100 * 10 * cs["base"]["omega"]
    pairs, logOmega, hz, Z, Nj, st = _oracle_stats(vo, cs, tN)
    vec = pack_stats(st["Nj"], st["N1"], st["M"], 1.5, -2.5, st["Nr"], st["Y"], st["SC"], cov)
    assert vec.size == vb.host.stats_len(K, S, d, cov)
    u = vb.host.unpack_stats(vec, K, S, d, cov)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        np.testing.assert_array_equal(u[k], st[k], err_msg=k)
    assert u["Lt1"] == 1.5 and u["Lt7"] == -2.5


@pytest.mark.parametrize("cov", [0, 1])
@pytest.mark.parametrize("S", [1, 4])
def test_finish_statistics_and_mstep(vb, vo, cov, S):
    K, d = 3, 3
    cs = make_case(10, K, S, 3, d, cov, seed=7)
    tN = 100 * 10 * cs["base"]["omega"]
    pairs, logOmega, hz, Z, Nj, st = _oracle_stats(vo, cs, tN)
    syn = vb.host.finish_statistics(st, cov)
    post = vb.host.mstep(syn, Nj, cs["opt"], cov, "iid")
    for j in range(K):
        pj = {k: pairs[k][:, j] for k in ("sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")}
        ref = vo.compute_statistics(Z[:, j], pj, S, d, cov)
        for k in ref:
            np.testing.assert_allclose(syn[k][j], ref[k], rtol=1e-12, atol=1e-12, err_msg=k)
        h = vo.mstep_component(ref, cs["opt"], cov)
        for k in ("eta", "epsilon", "lam", "v", "m", "W"):
            np.testing.assert_allclose(getattr(post, k)[j], h[k], rtol=1e-11, atol=1e-14, err_msg=k)
    np.testing.assert_allclose(post.alpha, cs["opt"]["alpha0"] + Nj, rtol=1e-15)


@pytest.mark.parametrize("cov", [0, 1])
def test_lower_bound(vb, vo, cov):
    cs = make_case(10, 3, 4, 3, 3, cov, seed=8)
    tN = 100 * 10 * cs["base"]["omega"]
    pairs, logOmega, hz, Z, Nj, st = _oracle_stats(vo, cs, tN)
    ref = vo.lower_bound(hz, Z, Nj, pairs["LL_elbo"], logOmega, cs["post"], cs["consts"], cs["opt"])
    Lt1 = float((Z * pairs["LL_elbo"]).sum())
    Lt7 = float((hz * np.log(hz)).sum())
    consts = vb.host.cluster_constants(cs["P"], cov)
    got = vb.host.lower_bound(Lt1, Lt7, Nj, vb.host.log_omega_tilde(cs["P"].alpha), cs["P"], consts,
                              cs["opt"], cov)
    assert abs(got - ref) <= 1e-12 * abs(ref)


@pytest.mark.parametrize("cov", [0, 1])
def test_convert_to_point(vb, vo, cov):
    cs = make_case(4, 3, 4, 3, 3, cov, seed=9)
    got = vb.host.convert_to_point(cs["P"], cov)
    ref = vo.convert_to_point(cs["post"], cov)
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-13, err_msg=k)


@pytest.mark.parametrize("cov,name", [(1, "C2"), (0, "C3")])
def test_em_loop_matches_oracle_em(vb, vo, cov, name):
    """Product EM loop (vbhem_amd.em, vectorised host math) driven by the
    oracle stand-in engine vs the oracle's loop-style em_step_fc."""
    from vbhem_amd.em import vbhem_h3m_c_step_fc

    N = 60 if name == "C2" else 40
    base, P, opt = vb.synth_workload(name, N=N)
    opt = dict(opt, max_iter=12)
    eng = OracleEngine(base, P.K, P.S, opt["tau"])
    res = vbhem_h3m_c_step_fc(P, eng, opt)
    ref = vo.em_step_fc(post_dict(P), base.numpy(), opt)
    assert res.iters == ref["iters"]
    np.testing.assert_allclose(res.LogLs, ref["LogLs"], rtol=1e-10)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert rel_err(getattr(res.post, k), ref["post"][k]) < RTOL_NORTH_STAR * 1e-3, k
    np.testing.assert_array_equal(res.label.numpy(), ref["label"])
    assert rel_err(res.hatZ.numpy(), ref["hat_Z"]) < 1e-10
    for k in ("prior", "A", "centres", "covars", "omega"):
        assert rel_err(res.point[k], ref["point"][k]) < 1e-9, k


def test_em_unstable_model_stops(vb):
    """NaN lower bound -> LL = -inf, stable = False, no M-step (step_fc.m:338-374)."""
    from vbhem_amd.em import vbhem_h3m_c_step_fc

    base, P, opt = vb.synth_workload("C2", N=8)
    eng = OracleEngine(base, P.K, P.S, opt["tau"])
    orig = eng.fused

    def nan_fused(tN):
        out = orig(tN)
        K, S = P.K, P.S
        out[K + K * S + K * S * S] = float("nan")     # Lt1
        return out

    eng.fused = nan_fused
    res = vbhem_h3m_c_step_fc(P, eng, opt)
    assert not res.stable and res.LL == -np.inf and res.iters == 0 and res.point is None


def test_shard_range_partitions(vb):
    from vbhem_amd.dist import shard_range

    for N in (0, 1, 7, 100, 101):
        for w in (1, 2, 3, 8):
            rs = [shard_range(N, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(rs[k][1] == rs[k + 1][0] for k in range(w - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("N", [300, 6000])
def test_synth_workload_shards_consistent(vb, N):
    """A shard generated alone equals the same rows of the whole set only in
    shape/semantics (per-shard seeding); the cluster posterior is identical on
    every shard -- and, above 4096 bases, identical to the unsharded run -- so
    all ranks of a multi-GPU run start from the same h3m_r."""
    h = N // 2
    b0, P0, _ = vb.synth_workload("C3", N=N, shard=(0, h))
    b1, P1, _ = vb.synth_workload("C3", N=N, shard=(h, N))
    assert b0.N == h and b1.N == N - h
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        np.testing.assert_array_equal(getattr(P0, k), getattr(P1, k))
    if N > 4096:
        _, Pu, _ = vb.synth_workload("C3", N=N)
        for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
            np.testing.assert_array_equal(getattr(P0, k), getattr(Pu, k))
    np.testing.assert_allclose((b0.omega.sum() + b1.omega.sum()).item(), 1.0, rtol=1e-13)
    assert torch.equal(b0.omega, b1.omega)


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [0, 1])
@pytest.mark.parametrize("use_post", [True, False])
def test_hmms_to_h3m_hem_device(vb, vo, cov, use_post):
    """hmms_to_h3m_hem.m on the device (vbhem_hmms_to_h3m, csrc/vbhem_h3m.hip) against
    the oracle's restatement: ragged state counts, an empty entry (weight 0, the
    one-state dummy), 1e-13 (the device psi / exp against SciPy's)."""
    hmms = random_vbhmms(40, 5, 3, seed=6, with_none=True)
    got = vb.h3m.hmms_to_h3m_hem_device(hmms, covmode=cov, use_post=use_post, device="cuda:0").numpy()
    ref = vo.hmms_to_h3m_hem(hmms, cov, use_post=use_post)
    for k in ("nstates", "prior", "A", "centres", "covars", "omega"):
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-13, atol=0, err_msg=k)
    assert got["omega"][1] == 0.0 and abs(got["omega"].sum() - 1) < 1e-15

"""The clustering driver (vbhem_amd.cluster: vbhem_h3m_cluster.m, vbhem_h3m_c.m)
and the hyperparameter learner (vbhem_amd.hyp: vbhem_h3m_c_hyp.m) on the CPU,
with the oracle stand-in engine (tests/oracle_engine.py) in place of the
device E-step: model selection over K and S (+gammaln), trials and their best
bound, groups, and a short L-BFGS hyperparameter run."""
import numpy as np
import pytest
from scipy.special import gammaln

from oracle_engine import OracleEngine


def _factory(base, K, S, T, trials=1):
    return OracleEngine(base, K, S, T, nthreads=2, trials=trials)


def _exprmt1(vb, N=16):
    return vb.synth_base_set(N, 2, 2, 2, vb.COV_FULL, seed=1002, exprmt1=True)


OPT = dict(alpha0=1e6, eta0=1.0, epsilon0=1.0, lambda0=1.0, v0=5.0, W0=1.0, m0=[1.5, 1.5],
           tau=20, Nv=100, seed=1001, trials=3, max_iter=30, minDiff=1e-5, learn_hyps=0)


def test_cluster_model_selection(vb):
    from vbhem_amd import cluster, em
    base = _exprmt1(vb)
    res = cluster.vbhem_h3m_cluster(None, [1, 2], [1, 2], dict(OPT, initmode="baseem"), base=base,
                                    engine_factory=_factory)
    # per-K raw bounds (each the best S of its run) + gammaln(K+1) select K
    raw = np.array([o["LL"] for o in res["model_all"]])
    np.testing.assert_allclose(res["model_LL"], raw + gammaln(np.array([2.0, 3.0])))
    assert res["model_bestK"] == [1, 2][int(np.argmax(res["model_LL"]))]
    for o in res["model_all"]:
        np.testing.assert_allclose(o["model_LL_S"],
                                   np.array([x["LL"] for x in o["model_all_s"]]) + gammaln([2.0, 3.0]))
    assert res["group_size"].sum() == base.N
    # the chosen model is its best trial: re-run it alone from the same initialisation
    K, S = res["K"], res["S"]
    o = vb.default_options(K, S, 2, **{k: v for k, v in OPT.items()})
    rb, rg, om = vb.baseem_draws(base, K, S, seed=OPT["seed"] + res["best"] + 1)
    P = vb.baseem_init(base, o, rb, rg, om)
    one = em.vbhem_h3m_c_step_fc(P, _factory(base, K, S, OPT["tau"]), o)
    assert one.iters == res["result"].iters
    np.testing.assert_allclose(one.LogLs, res["result"].LogLs, rtol=1e-12)
    assert res["LL"] == max(res["LLall"])


def test_trials_chunking_matches_one_launch(vb):
    """Batched trials (one launch for all) equal the same trials run one per launch."""
    from vbhem_amd import cluster
    base = _exprmt1(vb, N=10)
    o = vb.default_options(2, 2, 2, **dict(OPT, trials=4, max_iter=8))
    a = cluster.vbhem_h3m_c(base, o, engine_factory=_factory)
    b_results = []
    for r in range(4):  # one trial per launch
        oo = dict(o, trials=1, seed=o["seed"] + r)
        b_results.append(cluster.vbhem_h3m_c(base, oo, engine_factory=_factory)["LL"])
    np.testing.assert_allclose(a["LLall"], b_results, rtol=1e-12)


def test_hyp_learning_cpu(vb):
    from vbhem_amd import em, hyp
    base = _exprmt1(vb, N=12)
    o = vb.default_options(2, 2, 2, **dict(OPT, max_iter=40, minDiff=1e-8, learn_hyps=1))
    rb, rg, om = vb.baseem_draws(base, 2, 2, seed=7)
    P = vb.baseem_init(base, o, rb, rg, om)
    eng = _factory(base, 2, 2, o["tau"])
    start = em.vbhem_h3m_c_step_fc(P, eng, o)
    out = hyp.vbhem_h3m_c_hyp(base, o, start.post, eng, length=3)
    assert out["evaluations"] >= 2 and np.isfinite(out["result"].LL)
    # the optimiser's recorded objective never increases (it minimises -LL)
    assert np.all(np.diff(out["fX"]) <= 1e-9 * np.abs(out["fX"][:-1]))
    # the final run uses the optimised hyperparameters, clipped into range
    for name in ("alpha0", "eta0", "epsilon0", "lambda0"):
        assert o["hyps_min"][name] <= out["vbopt"][name] <= o["hyps_max"][name]


def test_hyp_best_only_among_reoptimised(vb, monkeypatch):
    """vbhem_h3m_c.m:102-105, 157-164: after hyperparameter learning every bound is
    NaN except those of the unique (re-optimised) trials, so a duplicate trial
    whose original bound beats the re-optimised one can not win."""
    from vbhem_amd import cluster, em, hyp
    base = _exprmt1(vb, N=10)
    o = vb.default_options(2, 2, 2, **dict(OPT, trials=3, max_iter=6, learn_hyps=1))
    fake_ll = iter([-100.0, -100.0, -50.0])          # trial bounds: 0 and 1 are duplicates

    real = em.vbhem_h3m_c_trials

    def trials(posts, eng, opt):
        out = real(posts, eng, opt)
        out.LLall = np.array([next(fake_ll) for _ in posts])
        return out

    calls = []

    def fake_hyp(base_, opt_, post, eng):
        calls.append(post)
        r = em.vbhem_h3m_c_step_fc(post, eng, dict(opt_, max_iter=2))
        r.LL = -1e9                                   # re-optimised bound far below the rest
        return dict(result=r)

    monkeypatch.setattr(em, "vbhem_h3m_c_trials", trials)
    monkeypatch.setattr(hyp, "vbhem_h3m_c_hyp", fake_hyp)
    out = cluster.vbhem_h3m_c(base, o, engine_factory=_factory)
    # unique trials: 0 and 2 (1 duplicates 0); both re-optimised to -1e9
    assert len(calls) == 2
    assert np.isnan(out["LLall"][1]) and out["best"] in (0, 2) and out["LL"] == -1e9
    assert out["hyp"] is not None


def test_cluster_vector_k_without_opt(vb):
    """vbhem_h3m_cluster with a vector of K and opt=None (defaults) runs."""
    from vbhem_amd import cluster
    base = _exprmt1(vb, N=8)
    calls = []

    def fake_c(base_, o, device, engine_factory):
        calls.append((o["K"], o["S"]))
        return dict(LL=-float(o["K"]), K=o["K"], S=o["S"])

    import unittest.mock as um
    with um.patch.object(cluster, "vbhem_h3m_c", fake_c):
        res = cluster.vbhem_h3m_cluster(None, [1, 2], 2, None, base=base)
    # (the default initmode 'auto': baseem, gmmNew, wtkmeans for each K)
    assert calls == [(1, 2)] * 3 + [(2, 2)] * 3 and res["model_bestK"] in (1, 2)


def test_weighted_kmeans_vs_loop_restatement(vb):
    """h3m.weighted_kmeans against oracle/h3m_init_oracle.py (my_weighted_kmeans.m in
    loops): the same assignments, centres to 1e-12."""
    import h3m_init_oracle as wo
    rng = np.random.default_rng(3)
    for K, n in ((2, 30), (3, 45), (4, 60)):
        pts = np.concatenate([rng.normal(loc, 0.7, (n // K, 2)) for loc in rng.uniform(-6, 6, (K, 2))])
        w = rng.uniform(0.1, 1.0, pts.shape[0])
        init = pts[rng.choice(pts.shape[0], K, replace=False)]
        got_c, got_cen, _ = vb.weighted_kmeans(K, 100, pts, w / w.sum(), init)
        ref_c, ref_cen = wo.weighted_kmeans(K, 100, pts.tolist(), (w / w.sum()).tolist(), init.tolist())
        assert got_c.tolist() == ref_c
        np.testing.assert_allclose(got_cen, np.array(ref_cen), rtol=1e-12, atol=1e-12)


def test_wtkmeans_init_structure(vb):
    """vbhemhmm_init.m:294-425 around the k-means centres: counts NJ = (Nv Kb) Kb / K,
    one W for every state, prior / A rows summing to NJ plus the pseudo-counts, and
    state centres drawn from the base means of well separated groups."""
    base = _exprmt1(vb, N=16)
    o = vb.default_options(2, 2, 2, **dict(OPT, initmode="wtkmeans"))
    P = vb.wtkmeans_init(base, o, 1005)
    Kb, NJ = base.N, o["Nv"] * base.N * base.N / 2
    np.testing.assert_allclose(P.alpha, o["alpha0"] + NJ)
    np.testing.assert_allclose(P.eta.sum(1), NJ + 2 * o["eta0"])
    np.testing.assert_allclose(P.epsilon.sum(2), NJ + 2 * o["epsilon0"])
    np.testing.assert_allclose(P.v, o["v0"] + NJ / 2 + 1)
    np.testing.assert_allclose(P.lam, o["lambda0"] + NJ / 2)
    W11 = np.linalg.inv((o["v0"] + NJ / 2 + 1 - 3) * base.covars[0, 0].numpy())
    np.testing.assert_allclose(P.W, np.broadcast_to(W11, P.W.shape))
    # exprmt1: ground-truth means {0, 3}; each cluster's centres sit near one of them
    cm = np.sort(P.m.mean(1)[:, 0])
    np.testing.assert_allclose(cm, [0.0, 3.0], atol=0.5)
    # deterministic in the seed
    np.testing.assert_array_equal(vb.wtkmeans_init(base, o, 1005).m, P.m)


def test_cluster_wtkmeans_and_auto(vb):
    from vbhem_amd import cluster
    base = _exprmt1(vb, N=12)
    o = vb.default_options(2, 2, 2, **dict(OPT, initmode="wtkmeans", trials=3, max_iter=20))
    r = cluster.vbhem_h3m_c(base, o, engine_factory=_factory)
    assert np.isfinite(r["LLall"]).all() and r["LL"] == max(r["LLall"])
    d = np.diff(r["result"].LogLs)
    assert (d >= -1e-9 * np.abs(r["result"].LogLs[1:])).all()
    auto = cluster.vbhem_h3m_cluster(None, 2, 2, dict(OPT, initmode="auto", trials=3, max_iter=20),
                                     base=base, engine_factory=_factory)
    assert auto["initmode"] in ("baseem", "gmmNew", "wtkmeans")
    assert auto["LL"] == max(auto["init_trials_LL"])
    np.testing.assert_allclose(auto["init_trials_LL"][2], r["LL"], rtol=1e-12)
    # keep_best_random_trial (default 1): every mode's run kept (vbhem_h3m_cluster.m:391-393)
    assert [t["Initmodes"] for t in auto["h3m_out_trials"]] == ["baseem", "gmmNew", "wtkmeans"]
    assert [t["LL"] for t in auto["h3m_out_trials"]] == auto["init_trials_LL"]
    # opt.initmodes needs opt.initopts (vbhem_h3m_cluster.m:366-368); one mode alone
    with pytest.raises(ValueError):
        cluster.vbhem_h3m_cluster(None, 2, 2, dict(OPT, initmode="auto", initmodes=["wtkmeans"],
                                                   trials=3, max_iter=20),
                                  base=base, engine_factory=_factory)
    one = cluster.vbhem_h3m_cluster(None, 2, 2, dict(OPT, initmode="auto", initmodes=["wtkmeans"],
                                                     initopts=["r0"], trials=3, max_iter=20,
                                                     keep_best_random_trial=0),
                                    base=base, engine_factory=_factory)
    np.testing.assert_allclose(one["LL"], r["LL"], rtol=1e-12)
    assert "h3m_out_trials" not in one


def test_hier_em_vs_loop_restatement(vb):
    """h3m.gmm_mix_hier_em (GMM_MixHierEM.m) against the loop restatement in
    oracle/h3m_init_oracle.py from the same initial centres (full covariance)."""
    import h3m_init_oracle as wo
    rng = np.random.default_rng(5)
    X = np.concatenate([rng.normal(loc, 0.4, (8, 2)) for loc in ([0, 0], [4, 1], [1, 5])])
    C = np.stack([(lambda a: a @ a.T + 0.2 * np.eye(2))(rng.normal(size=(2, 2)) * 0.3) for _ in X])
    init = X[[0, 9, 17]]
    pri, cen, cov, _ = vb.gmm_mix_hier_em(X, C, True, 3, 100.0 * 24, 30, rng, init_centres=init)
    rp, rc, rv = wo.hier_em_full(X, C, 3, 100.0 * 24, 30, init)
    np.testing.assert_allclose(pri, rp, rtol=1e-10)
    np.testing.assert_allclose(cen, np.stack(rc), rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(cov, np.stack(rv), rtol=1e-10, atol=1e-12)
    # three well separated groups: the reduced components sit on them
    np.testing.assert_allclose(np.sort(cen[:, 0]), [0, 1, 4], atol=0.4)


def test_gmmnew_init_and_auto(vb):
    from vbhem_amd import cluster
    base = _exprmt1(vb, N=12)
    o = vb.default_options(2, 2, 2, **dict(OPT, initmode="gmmNew", trials=3, max_iter=20))
    P = vb.gmmnew_init(base, o, 1002)
    Nv = o["Nv"] * base.N
    np.testing.assert_allclose(P.alpha.sum(), 2 * o["alpha0"] + Nv)
    np.testing.assert_allclose(P.m[0], P.m[1])                 # shared reduced components
    np.testing.assert_allclose(np.sort(P.m[0][:, 0]), [0.0, 3.0], atol=0.5)
    r = cluster.vbhem_h3m_c(base, o, engine_factory=_factory)
    assert np.isfinite(r["LLall"]).all()
    auto = cluster.vbhem_h3m_cluster(None, 2, 2, dict(OPT, initmode="auto", trials=3, max_iter=20),
                                     base=base, engine_factory=_factory)
    assert len(auto["init_trials_LL"]) == 3 and auto["LL"] == max(auto["init_trials_LL"])
    np.testing.assert_allclose(auto["init_trials_LL"][1], r["LL"], rtol=1e-12)

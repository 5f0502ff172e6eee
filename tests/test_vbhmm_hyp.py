"""VB-HMM hyperparameter learning (vbhmm_learn.m learn_hyps: vbhmm_em_hyp.m,
get_hypinfo.m, uniqueLL.m, vbhmm_em_lb.m:260-400).

No reference output holds a learned-hyperparameter run, so the derivatives are
pinned by central finite differences of the bound itself (vbhmm_em_lb.m:74-257,
whose value is pinned against the oracle in test_vbhmm_em.py), and the
optimiser by its contract: the bound at the optimum is >= the bound at the
start, and the final EM run reproduces the optimiser's best value.

CPU: finite differences of every transformed derivative (iid and diag W0,
the sqrt and log W0 transforms); uniqueLL; vbhmm_em_hyp and vbhmm_learn with
learn_hyps driven by the C restatement of vbhmm_fb_mex.c in place of the GPU
forward-backward (host logic only).
GPU: the same learn_hyps run on the GPU forward-backward agrees with the CPU one.
"""
import numpy as np
import pytest

import vbhem_oracle as vo
from test_vbhmm_em import DEMO_VBHEMOPT, DEMO_VBOPT, demo_subjects


def _opts(dim=2, **over):
    from vbhem_amd.vbhmm_em import vbhmm_default_options
    return vbhmm_default_options(dim, **dict(DEMO_VBOPT, **over))


def _synthetic_state(rng, K, dim, W0mode):
    """A valid posterior + fbstats with every field vbhmm_em_lb reads."""
    N, T = 4, 6
    W = np.stack([(lambda a: (a @ a.T + np.eye(dim)) * 3e-3)(rng.normal(size=(dim, dim)) * 0.3)
                  for _ in range(K)])
    vp = dict(v=rng.uniform(dim + 2, dim + 20, K), W=W, epsilon=rng.uniform(0.5, 5, (K, K)),
              alpha=rng.uniform(0.5, 5, K), m=np.array([150.0, 200.0][:dim]) + rng.normal(0, 3, (K, dim)),
              beta=rng.uniform(1, 30, K))
    g = rng.uniform(0.01, 1, (K, N, T))
    g /= g.sum(0, keepdims=True)
    fb = dict(logLambdaTilde=rng.normal(-10, 1, K), logPiTilde=np.log(rng.dirichlet(np.ones(K))),
              logATilde=np.log(rng.dirichlet(np.ones(K), K)), gamma_all=g,
              logrho_Saved=rng.normal(-12, 2, (K, N, T)), phi_norm=rng.normal(-30, 3, N))
    st = dict(dim=dim, K=K, N=N, W0mode=W0mode, t1_S=np.stack([np.eye(dim) * 0.5] * K),
              xbar=vp["m"] + rng.normal(0, 0.5, (K, dim)), Nk=g.sum((1, 2)), M=rng.uniform(0, 5, (K, K)))
    return st, vp, fb


def _lb_at(X, st, opt, vp, fb, info):
    from vbhem_amd.vbhmm_em import _set_hyps, vbhmm_em_lb
    o = _set_hyps(X, opt, info)
    W0 = np.asarray(o["W0"], float)
    dim = st["dim"]
    st = dict(st, W0inv=np.linalg.inv(float(W0) * np.eye(dim) if W0.size == 1 else np.diag(W0.reshape(-1))))
    return vbhmm_em_lb(st, o, vp, fb, do_deriv=True)


@pytest.mark.parametrize("W0mode,wname", [("iid", "W0"), ("diag", "W0"), ("iid", "W0log"),
                                          ("diag", "W0log")])
def test_bound_derivatives_finite_difference(vb, W0mode, wname):
    from vbhem_amd import hyp
    from vbhem_amd.vbhmm_em import vbhmm_hypinfo
    rng = np.random.default_rng(11 + len(W0mode) + len(wname))
    K, dim = 3, 2
    opt = _opts(alpha0=0.7, epsilon0=1.3, beta0=2.0, v0=6.0,
                W0=0.002 if W0mode == "iid" else np.array([0.002, 0.004]), mu0=[150.0, 200.0])
    st, vp, fb = _synthetic_state(rng, K, dim, W0mode)
    info = vbhmm_hypinfo(["alpha0", "epsilon0", "v0", "beta0", wname, "mu0"], opt)
    X0 = hyp.init_x(opt, info)
    _, d = _lb_at(X0, st, opt, vp, fb, info)
    grad = np.concatenate([np.atleast_1d(d[i.derivname]).reshape(-1) for i in info])
    assert grad.size == X0.size
    LB0 = _lb_at(X0, st, opt, vp, fb, info)[0]
    assert abs(LB0) < 1e4                      # keeps the rounding of the differences ~1e-9
    for j in range(X0.size):
        h = 1e-4 * max(1.0, abs(X0[j]))
        e = np.zeros_like(X0)
        e[j] = h
        fd = (_lb_at(X0 + e, st, opt, vp, fb, info)[0] - _lb_at(X0 - e, st, opt, vp, fb, info)[0]) / (2 * h)
        assert abs(fd - grad[j]) <= 1e-6 * max(1.0, abs(grad[j])), (j, fd, grad[j])


def test_clipped_derivative_zeroed(vb):
    from vbhem_amd.vbhmm_em import vbhmm_em_lb
    rng = np.random.default_rng(3)
    st, vp, fb = _synthetic_state(rng, 2, 2, "iid")
    st["W0inv"] = np.eye(2) / 0.002
    opt = _opts(W0=0.002)
    _, d = vbhmm_em_lb(st, opt, vp, fb, do_deriv=True)
    up = d["d_logalpha0"][0] > 0
    _, d2 = vbhmm_em_lb(st, opt, vp, fb, do_deriv=True, clipped={"alpha0": 1 if up else -1})
    assert d2["d_logalpha0"][0] == 0.0
    _, d3 = vbhmm_em_lb(st, opt, vp, fb, do_deriv=True, clipped={"alpha0": -1 if up else 1})
    assert d3["d_logalpha0"][0] == d["d_logalpha0"][0]


def test_unique_ll(vb):
    from vbhem_amd.cluster import unique_ll
    LL = np.array([-1000.0, -1000.0001, -1010.0, -999.99999, -1010.00001, -1200.0])
    assert unique_ll(LL, 2e-4) == [0, 2, 5]
    assert unique_ll(LL, 0.0) == [0, 1, 2, 3, 4, 5]


def _cpu_fb(data, vp, batch=None):
    """vbhmm.vbhmm_fb's contract, computed by the C restatement of vbhmm_fb_mex.c."""
    pre = vo.vbhmm_prelude(vp)
    f = vo.c_vbhmm_fb(data, vp, pre)
    return dict(gamma_all=f["gamma"].transpose(2, 1, 0), logrho_Saved=f["logrho"].transpose(2, 1, 0),
                xi_sum=f["xi_sum"].transpose(1, 2, 0), phi_norm=f["phi_norm"],
                logLambdaTilde=pre["logLambdaTilde"], logPiTilde=pre["logPiTilde"],
                logATilde=pre["logATilde"])


@pytest.fixture
def cpu_fb(vb, monkeypatch):
    from vbhem_amd import vbhmm_em as vme
    monkeypatch.setattr(vme.vbhmm, "vbhmm_fb", _cpu_fb)
    monkeypatch.setattr(vme.vbhmm, "SequenceBatch", lambda data, dim, device: None)
    return vme


def _learn_hyps_case(vme):
    data = demo_subjects()[2]
    opt = _opts(learn_hyps=1, hyp_length=8, maxIter=60)
    start = vme.vbhmm_em(data, 2, opt, gmm=vme.random_gmm(data, 2, np.random.default_rng(5)))
    return data, opt, start, vme.vbhmm_em_hyp(data, 2, opt, start)


def test_em_hyp_raises_bound_cpu(cpu_fb):
    data, opt, start, h = _learn_hyps_case(cpu_fb)
    lh = h["learn_hyps"]
    assert lh["hypinfo"] == ["alpha0", "epsilon0", "v0", "beta0", "W0", "mu0"]
    assert lh["opt_transhyp"].size == 7
    assert h["LL"] >= start["LL"] - 1e-9 * abs(start["LL"])
    assert h["LL"] > start["LL"] + 1.0            # the demo's hyperparameters are not optimal
    np.testing.assert_allclose(h["LL"], lh["opt_L"], rtol=1e-12)
    assert np.all(np.diff(lh["fX"]) <= 1e-9 * np.abs(lh["fX"][1:]))
    assert lh["vbopt"]["v0"] > 1.0 and lh["vbopt"]["alpha0"] > 0


def test_learn_with_hyps_cpu(cpu_fb):
    data = demo_subjects()[6]
    opt = _opts(learn_hyps=["alpha0", "epsilon0"], hyp_length=5, numtrials=3, maxIter=40,
                keep_best_random_trial=1)
    out = cpu_fb.vbhmm_learn(data, 2, opt)
    assert np.isfinite(out["trials_LL"]).sum() >= 1
    assert out["LL"] >= np.nanmax(out["trials_LL_random"]) - 1e-9 * abs(out["LL"])
    assert out["learn_hyps"]["hypinfo"] == ["alpha0", "epsilon0"]
    assert "hmm_best_random_trial" in out["learn_hyps"]


@pytest.mark.gpu
def test_em_hyp_gpu_matches_cpu_fb(vb, monkeypatch):
    from vbhem_amd import vbhmm_em as vme
    _, _, start_g, h_g = _learn_hyps_case(vme)
    monkeypatch.setattr(vme.vbhmm, "vbhmm_fb", _cpu_fb)
    monkeypatch.setattr(vme.vbhmm, "SequenceBatch", lambda data, dim, device: None)
    _, _, start_c, h_c = _learn_hyps_case(vme)
    np.testing.assert_allclose(start_g["LL"], start_c["LL"], rtol=1e-9)
    np.testing.assert_allclose(h_g["LL"], h_c["LL"], rtol=1e-6)
    np.testing.assert_allclose(h_g["learn_hyps"]["opt_transhyp"], h_c["learn_hyps"]["opt_transhyp"],
                               rtol=1e-3, atol=1e-3)


def test_learn_hyps_batch_cpu(cpu_fb):
    """vbhmm_learn_batch.m learn_hyps_batch: one hyperparameter set for all subjects."""
    from scipy.special import gammaln
    subs = demo_subjects()
    datas = [subs[1], subs[4]]
    opt = _opts(learn_hyps_batch=["alpha0", "epsilon0", "mu0"], numtrials=2, maxIter=40)
    hmms, Ls = cpu_fb.vbhmm_learn_batch(datas, [1, 2], opt)
    lh = hmms[0]["learn_hyps_batch"]
    assert lh["hypinfo"] == ["alpha0", "epsilon0", "mu0"] and lh["opt_transhyp"].size == 4
    assert lh["fX"][-1] < lh["fX"][0]                     # the shared bound went up
    np.testing.assert_allclose(hmms[0]["vbopt"]["mu0"], hmms[1]["vbopt"]["mu0"])
    # the optimiser's value is the mean over subjects of -(LL + gammaln(K+1))
    nL = np.mean([-(h["LL"] + gammaln(len(h["pdf"]) + 1)) for h in hmms])
    np.testing.assert_allclose(nL, lh["fX"][-1], rtol=1e-12)
    np.testing.assert_allclose(Ls, [h["LL"] for h in hmms])
    # without the shared learning the same subjects give the per-subject path
    hmms0, _ = cpu_fb.vbhmm_learn_batch(datas, [1, 2], dict(opt, learn_hyps_batch=0))
    assert "learn_hyps_batch" not in hmms0[0]


@pytest.mark.gpu
def test_c1_demo_with_learn_hyps(vb, monkeypatch):
    """vbdemo_face.m as written (vbopt.learn_hyps = 1, K = 1:3; vbhemopt 'wtkmeans' x 50
    with its default learn_hyps = 1, K = 1:5, S = 1:3), except 3 injected random GMMs per
    K instead of 50 trials in the HMM stage and the k-means stand-in inside 'wtkmeans':
    the GPU HMM stage agrees with the same run on the C forward-backward, every K's
    optimised bound is >= its best random trial, and the learned HMMs cluster."""
    from vbhem_amd import cluster
    from vbhem_amd import vbhmm_em as vme
    subjects = demo_subjects()
    opt = _opts(learn_hyps=1, numtrials=3)
    gmms = []
    for i, d in enumerate(subjects):
        rng = np.random.default_rng(1000 + i)
        gmms.append({K: [vme.random_gmm(d, K, np.random.default_rng(int(rng.integers(1 << 30))))
                         for _ in range(1 if K == 1 else 3)] for K in (1, 2, 3)})
    hmms, Ls = vme.vbhmm_learn_batch(subjects, [1, 2, 3], opt, device="cuda:0", gmms=gmms)
    assert len(hmms) == 10 and np.isfinite(Ls).all()
    for h in hmms:
        for o in h["model_all"]:
            assert np.nanmax(o["trials_LL"]) >= o["trials_LL_random"].max() - 1e-9 * abs(o["LL"])
            assert "learn_hyps" in o
    with monkeypatch.context() as m:
        m.setattr(vme.vbhmm, "vbhmm_fb", _cpu_fb)
        m.setattr(vme.vbhmm, "SequenceBatch", lambda data, dim, device: None)
        _, Ls_c = vme.vbhmm_learn_batch(subjects, [1, 2, 3], opt, gmms=gmms)
    np.testing.assert_allclose(Ls, Ls_c, rtol=1e-6)
    # the clustering stage as the demo writes it: 'wtkmeans' x 50 trials, vbhemopt.learn_hyps
    # left at its default, 1
    hopt = dict(DEMO_VBHEMOPT, initmode="wtkmeans", trials=50, max_iter=200, minDiff=1e-5,
                learn_hyps=1)
    res = cluster.vbhem_h3m_cluster(hmms, [1, 2, 3, 4, 5], [1, 2, 3], hopt, device="cuda:0")
    assert 1 <= res["model_bestK"] <= 5 and 1 <= res["model_bestS"] <= 3
    assert np.isfinite(res["model_LL"]).all() and sum(res["group_size"]) == 10
    assert res["hyp"] is not None


def test_vbhmm_standardize(vb):
    """vbhmm_standardize.m / vbhmm_permute.m on a hand-made 3-state HMM."""
    from vbhem_amd.vbhmm_em import vbhmm_permute, vbhmm_prob_steadystate, vbhmm_standardize
    hmm = dict(prior=np.array([0.2, 0.5, 0.3]), trans=np.array([[0.1, 0.2, 0.7], [0.6, 0.1, 0.3],
                                                                   [0.3, 0.6, 0.1]]),
               N=np.array([5.0, 9.0, 7.0]), N1=np.array([1.0, 2.0, 3.0]), M=np.arange(9.0).reshape(3, 3),
               pdf=[dict(mean=np.array([x, 0.0]), cov=np.eye(2)) for x in (3.0, 1.0, 2.0)],
               gamma=[np.array([[0.2], [0.5], [0.3]])],
               varpar=dict(alpha=np.array([1.0, 2.0, 3.0]), epsilon=np.arange(9.0).reshape(3, 3),
                           beta=np.ones(3), v=np.array([4.0, 5.0, 6.0]), m=np.eye(3)[:, :2],
                           W=np.stack([np.eye(2) * k for k in (1, 2, 3)])))
    f = vbhmm_standardize(hmm, "f")          # prior argmax 1, then row 1 -> 0, then 2
    np.testing.assert_allclose(f["prior"], [0.5, 0.2, 0.3])
    np.testing.assert_allclose(f["trans"], hmm["trans"][np.ix_([1, 0, 2], [1, 0, 2])])
    assert [q["mean"][0] for q in f["pdf"]] == [1.0, 3.0, 2.0]
    np.testing.assert_allclose(f["varpar"]["W"][:, 0, 0], [2, 1, 3])
    np.testing.assert_allclose(f["gamma"][0][:, 0], [0.5, 0.2, 0.3])
    np.testing.assert_allclose(vbhmm_standardize(f, "f")["prior"], f["prior"])   # idempotent
    assert list(vbhmm_standardize(hmm, "e")["N"]) == [9.0, 7.0, 5.0]
    assert [q["mean"][0] for q in vbhmm_standardize(hmm, "l")["pdf"]] == [1.0, 2.0, 3.0]
    p = vbhmm_prob_steadystate(hmm)
    np.testing.assert_allclose(p @ hmm["trans"], p, atol=1e-12)
    np.testing.assert_allclose(p.sum(), 1.0)
    back = vbhmm_permute(vbhmm_permute(hmm, [2, 0, 1]), [1, 2, 0])
    np.testing.assert_allclose(back["varpar"]["epsilon"], hmm["varpar"]["epsilon"])


@pytest.mark.gpu
def test_learn_hyps_batch_gpu_matches_cpu_fb(vb, monkeypatch):
    """learn_hyps_batch on the GPU forward-backward agrees with the same run on the C
    restatement of vbhmm_fb_mex.c (bounds 1e-6, shared hyperparameters 1e-3)."""
    from vbhem_amd import vbhmm_em as vme
    subs = demo_subjects()
    datas = [subs[1], subs[4]]
    opt = _opts(learn_hyps_batch=["alpha0", "epsilon0", "mu0"], numtrials=2, maxIter=40)
    hmms_g, Ls_g = vme.vbhmm_learn_batch(datas, [1, 2], opt, device="cuda:0")
    with monkeypatch.context() as m:
        m.setattr(vme.vbhmm, "vbhmm_fb", _cpu_fb)
        m.setattr(vme.vbhmm, "SequenceBatch", lambda data, dim, device: None)
        hmms_c, Ls_c = vme.vbhmm_learn_batch(datas, [1, 2], opt)
    np.testing.assert_allclose(Ls_g, Ls_c, rtol=1e-6)
    np.testing.assert_allclose(hmms_g[0]["learn_hyps_batch"]["opt_transhyp"],
                               hmms_c[0]["learn_hyps_batch"]["opt_transhyp"], rtol=1e-3, atol=1e-3)

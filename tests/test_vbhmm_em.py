"""VB-HMM learning of the base HMMs and config C1 end to
end (demo/vbdemo_face.m: fixations -> vbhmm_learn_batch -> vbhem_h3m_cluster).

The oracle is oracle/vbhmm_em_oracle.py, a loop restatement of vbhmm_em.m +
vbhmm_em_lb.m + vbhmm_init.m driving the C restatement of vbhmm_fb_mex.c.
MATLAB's gmdistribution.fit (the 'random' initialiser) is absent, so both
sides get the same injected GMM; parity of the initialiser itself is unpinned.

CPU: the oracle with the C forward-backward vs with the numpy twin of
vbhmm_fb.m; the variational bound never decreases; the GMM stand-in and
vbhmm_remove_empty on known inputs.
GPU: vbhmm_em (GPU forward-backward) vs the oracle per iteration, and C1: the
demo's 10 subjects through vbhmm_learn_batch (K = 1:3) and vbhem_h3m_cluster
(K = 1:5, S = 1:3), each subject's bound and the selected clustering's ELBO
trajectory checked against the oracles.
"""
import os

import numpy as np
import pytest

import vbhmm_em_oracle as vho
from conftest import GOLDEN_DIR, RTOL_NORTH_STAR, hatz_err, post_err

# demo/vbdemo_face.m:21-31 (mu0 = image size / 2 of ave_face120.png, 320 x 420)
DEMO_VBOPT = dict(alpha0=1.0, mu0=[160.0, 210.0], W0=0.001, beta0=1.0, v0=10.0, epsilon0=1.0,
                  seed=100)
# demo/vbdemo_face.m:49-61
DEMO_VBHEMOPT = dict(alpha0=1.0, eta0=1.0, m0=[160.0, 210.0], W0=0.001, lambda0=1.0, v0=10.0,
                     epsilon0=1.0, seed=1001, Nv=10, tau=5)


def demo_subjects():
    fx = np.load(os.path.join(GOLDEN_DIR, "demo_fixations.npz"))
    off, x, subj = fx["offsets"], fx["x"], fx["subject"]
    seqs = [x[off[n]:off[n + 1]] for n in range(off.size - 1)]
    return [[s for s, g in zip(seqs, subj) if g == i] for i in range(len(fx["names"]))]


def _opts(vb, **over):
    from vbhem_amd.vbhmm_em import vbhmm_default_options
    return vbhmm_default_options(2, **dict(DEMO_VBOPT, **over))


def _gmm(vb, data, K, seed):
    from vbhem_amd.vbhmm_em import random_gmm
    return random_gmm(data, K, np.random.default_rng(seed))


def test_oracle_c_vs_twin_fb(vb):
    subjects = demo_subjects()
    opt = _opts(vb, maxIter=30)
    for i, K in ((0, 2), (3, 3)):
        g = _gmm(vb, subjects[i], K, 7 + i)
        a = vho.em(subjects[i], K, opt, g, fb_fn="c")
        b = vho.em(subjects[i], K, opt, g, fb_fn="twin")
        assert a["iters"] == b["iters"]
        np.testing.assert_allclose(a["LLs"], b["LLs"], rtol=1e-10)


def test_bound_never_decreases(vb):
    subjects = demo_subjects()
    opt = _opts(vb, maxIter=60, minDiff=1e-9)
    for i, K in ((1, 2), (4, 3), (7, 3)):
        r = vho.em(subjects[i], K, opt, _gmm(vb, subjects[i], K, 30 + i))
        d = np.diff(r["LLs"])
        assert (d >= -1e-9 * np.abs(r["LLs"][1:])).all(), (i, K, d.min())


def test_gmm_standin_recovers_clusters(vb):
    from vbhem_amd.vbhmm_em import gmm_fit_randsample
    rng = np.random.default_rng(1)
    X = np.concatenate([rng.normal([0, 0], 1.0, (300, 2)), rng.normal([20, 5], 2.0, (200, 2))])
    g = gmm_fit_randsample(X, 2, np.random.default_rng(4))
    order = np.argsort(g["mean"][:, 0])
    np.testing.assert_allclose(g["mean"][order], [[0, 0], [20, 5]], atol=0.5)
    np.testing.assert_allclose(np.sort(g["prior"]), [0.4, 0.6], atol=0.02)


def test_remove_empty(vb):
    from vbhem_amd.vbhmm_em import vbhmm_remove_empty
    K = 3
    hmm = dict(N=np.array([5.0, 1e-5, 2.0]), M=np.arange(9.0).reshape(3, 3), N1=np.ones(3),
               gamma=[np.array([[0.5, 0.2], [0.1, 0.1], [0.4, 0.7]])],
               pdf=[dict(mean=np.zeros(2) + k, cov=np.eye(2)) for k in range(K)],
               varpar=dict(alpha=np.array([2.0, 1.0, 3.0]), epsilon=np.arange(1.0, 10.0).reshape(3, 3),
                           beta=np.ones(3), v=np.full(3, 5.0), m=np.zeros((3, 2)),
                           W=np.stack([np.eye(2)] * 3)))
    out = vbhmm_remove_empty(hmm, 1e-3)
    assert out["N"].tolist() == [5.0, 2.0]
    np.testing.assert_allclose(out["prior"], [0.4, 0.6])
    np.testing.assert_allclose(out["trans"], [[1 / 4, 3 / 4], [7 / 16, 9 / 16]])
    np.testing.assert_allclose(out["gamma"][0].sum(0), 1.0)
    assert [p["mean"][0] for p in out["pdf"]] == [0.0, 2.0]


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 2, 3])
def test_vbhmm_em_matches_oracle(vb, K):
    from vbhem_amd.vbhmm_em import vbhmm_em
    subjects = demo_subjects()
    opt = _opts(vb)
    for i in (0, 5, 9):
        g = _gmm(vb, subjects[i], K, 100 + i)
        got = vbhmm_em(subjects[i], K, opt, gmm=g, device="cuda:0")
        ref = vho.em(subjects[i], K, opt, g)
        assert got["iters"] == ref["iters"], (i, K)
        np.testing.assert_allclose(got["LLs"], ref["LLs"], rtol=1e-9)
        for k in ("alpha", "epsilon", "beta", "v", "m", "W"):
            assert post_err(got["varpar"][k], ref["varpar"][k]) < 1e-8, (i, K, k)


@pytest.mark.gpu
def test_c1_demo_end_to_end(vb, vo):
    """vbdemo_face.m: 10 subjects -> vbhmm_learn_batch(K = 1:3) -> vbhem_h3m_cluster(K = 1:5,
    S = 1:3), both stages without learn_hyps so that every bound can be re-run by
    the oracles (test_vbhmm_hyp.test_c1_demo_with_learn_hyps runs the demo with
    it); the clustering with the 'baseem' initialiser and 8 trials per (K, S)
    instead of 'wtkmeans' x 50 (Statistics Toolbox); everything else follows the
    demo's options."""
    from cases import post_dict
    from vbhem_amd import cluster
    from vbhem_amd.vbhmm_em import vbhmm_learn_batch, vbhmm_remove_empty
    subjects = demo_subjects()
    opt = _opts(vb, numtrials=3)
    gmms = []
    for i, d in enumerate(subjects):
        rng = np.random.default_rng(1000 + i)
        gmms.append({K: [_gmm(vb, d, K, int(rng.integers(1 << 30))) for _ in range(1 if K == 1 else 3)]
                     for K in (1, 2, 3)})
    hmms, Ls = vbhmm_learn_batch(subjects, [1, 2, 3], opt, device="cuda:0", gmms=gmms)
    assert len(hmms) == 10 and np.isfinite(Ls).all()
    # every subject's selected model: its bound equals the oracle EM from the same GMM
    from scipy.special import gammaln
    for i, h in enumerate(hmms):
        K = h["model_bestK"]
        best = int(np.argmax(h["model_all"][[1, 2, 3].index(K)]["trials_LL"]))
        ref = vho.em(subjects[i], K, opt, gmms[i][K][best])
        assert abs(h["LL"] - (ref["LL"] + gammaln(K + 1))) <= 1e-9 * abs(ref["LL"]), i
    # clustering: K = 1:5, S = 1:3 over the learned HMMs
    hopt = dict(DEMO_VBHEMOPT, initmode="baseem", trials=8, max_iter=200, minDiff=1e-5, learn_hyps=0)
    res = cluster.vbhem_h3m_cluster(hmms, [1, 2, 3, 4, 5], [1, 2, 3], hopt, device="cuda:0")
    bestK, bestS = res["model_bestK"], res["model_bestS"]
    assert 1 <= bestK <= 5 and 1 <= bestS <= 3
    assert len(res["model_LL"]) == 5 and np.isfinite(res["model_LL"]).all()
    assert sum(res["group_size"]) == 10
    # the selected (K, S): its best trial re-run by the oracle EM from the same initialisation
    base = vb.hmms_to_h3m_hem([vbhmm_remove_empty(h, 1e-3) for h in hmms], vb.COV_FULL, True)
    o = vb.default_options(bestK, bestS, 2, **{k: v for k, v in hopt.items()})
    rb, rg, om = vb.baseem_draws(base, bestK, bestS, seed=hopt["seed"] + res["best"] + 1)
    P = vb.baseem_init(base, o, rb, rg, om)
    ref = vo.em_step_fc(post_dict(P), base.numpy(), o)
    r = res["result"]
    assert r.iters == ref["iters"]
    np.testing.assert_allclose(r.LogLs, ref["LogLs"], rtol=RTOL_NORTH_STAR)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert post_err(getattr(r.post, k), ref["post"][k]) < RTOL_NORTH_STAR, k
    assert hatz_err(r.hatZ.cpu().numpy(), ref["hat_Z"]) < RTOL_NORTH_STAR

"""Clustering scores (vbhem_amd.evaluate: valid_RandIndex.m, Purity.m) on hand
checked cases, and the reference's synthetic experiment 1 as an end-to-end
recovery check: base HMMs from the two ground-truth HMMs of
exprmt1_sampledata.m:20-43 (20 per group in the reference; here N = 80), VBHEM
with K = 2, S = 2 and batched trials; the best trial's labels must recover the
ground-truth grouping (Rand index 1, purity 1), as syn_evluate.m scores it."""
import numpy as np
import pytest


def test_rand_index_known_values(vb):
    from vbhem_amd.evaluate import purity, rand_index
    a = [1, 1, 2, 2]
    RI, AR, MI, HI = rand_index(a, [5, 5, 7, 7])       # same partition, other names
    assert RI == 1.0 and AR == 1.0 and MI == 0.0 and HI == 1.0
    RI, AR, MI, HI = rand_index(a, [1, 2, 1, 2])       # 6 pairs: 2 agreements
    assert abs(RI - 2 / 6) < 1e-15 and abs(MI - 4 / 6) < 1e-15 and abs(HI + 2 / 6) < 1e-15
    assert abs(AR - (-0.5)) < 1e-12
    assert purity(a, [1, 1, 1, 1]) == 0.5 and purity(a, [3, 3, 4, 4]) == 1.0
    assert purity([1, 1, 2, 2, 2], [1, 1, 1, 2, 2]) == 0.8
    with pytest.raises(ValueError):
        rand_index([1], [1])


@pytest.mark.gpu
def test_exprmt1_recovery(vb):
    import torch
    from vbhem_amd import em, host
    from vbhem_amd.estep import EStepEngine
    from vbhem_amd.evaluate import purity, rand_index
    N, K, S, R = 80, 2, 2, 8
    base = vb.synth_base_set(N, K, 2, 2, vb.COV_FULL, seed=1002, exprmt1=True)
    opt = vb.default_options(K, S, 2, tau=50, Nv=100, covmode=vb.COV_FULL, alpha0=1e6, eta0=1.0,
                             epsilon0=1.0, lambda0=1.0, v0=5.0, W0=1.0, m0=[1.5, 1.5])
    posts = []
    for r in range(R):
        rb, rg, om = vb.baseem_draws(base, K, S, seed=100 + r)
        posts.append(vb.baseem_init(base, opt, rb, rg, om))
    eng = EStepEngine(base, R * K, S, opt["tau"], device="cuda:0", trials=R)
    tr = em.vbhem_h3m_c_trials(posts, eng, opt)
    best = tr.results[tr.best]
    assert best.stable and np.isfinite(best.LL)
    truth = np.arange(N) % 2                      # synth_base_set's ground-truth index
    labels = best.label.cpu().numpy()
    RI, AR, _, _ = rand_index(truth, labels)
    assert RI == 1.0 and AR == 1.0, (RI, AR)
    assert purity(truth, labels) == 1.0
    del torch, host

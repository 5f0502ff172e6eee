"""Batched EM trials (vbhem_h3m_c.m:28-67 `parfor it = 1:numits`):
R trials of K clusters each run as ONE fused launch over R*K clusters
(vbhem_estep_fused_trials).  Checked against R separate fused calls (each
already pinned to the oracle by test_gpu_parity.py) and, for the EM loop,
against R separate vbhem_h3m_c_step_fc runs: the same per-pair arithmetic,
so only the epilogue's summation trees and the emission GEMM's mean shift
differ (tolerance 1e-12)."""
import ctypes

import numpy as np
import pytest
import torch

from cases import make_case
from conftest import hatz_err, rel_err, stat_err

DEV = "cuda:0"


def _trial_posts(cs, R, seed):
    """R cluster posteriors over the same base set: the case's posterior and R-1
    re-perturbed copies (distinct initialisations, as the trials of vbhem_h3m_c.m)."""
    posts = [cs["P"].copy()]
    for r in range(1, R):
        P = cs["P"].copy()
        rng = np.random.default_rng(seed * 100 + r)
        P.epsilon = P.epsilon * rng.uniform(0.3, 1.7, P.epsilon.shape)
        P.eta = P.eta * rng.uniform(0.3, 1.7, P.eta.shape)
        P.m = P.m + rng.normal(0.0, 0.5, P.m.shape)
        P.alpha = P.alpha * rng.uniform(0.5, 1.5, P.alpha.shape)
        posts.append(P)
    return posts


def test_trials_workspace_and_arguments(capi_lib):
    from vbhem_amd import _capi
    p = 1 << 20
    b = _capi.BaseT(10, 3, 2, 1, p, p, p, p, p)
    c = _capi.ClusterT(6, 3, p, p, p, p, p)
    one = capi_lib.vbhem_fused_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 10)
    assert capi_lib.vbhem_fused_trials_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 1, 10) == one
    assert capi_lib.vbhem_fused_trials_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 3, 10) > 0
    assert capi_lib.vbhem_fused_trials_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 4, 10) == 0
    assert capi_lib.vbhem_fused_trials_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 0, 10) == 0
    v = ctypes.c_void_p(p)
    rc = capi_lib.vbhem_estep_fused_trials(ctypes.byref(b), ctypes.byref(c), 4, 10, v, v, v, v, v,
                                           v, ctypes.c_size_t(1 << 40), None)
    assert rc != 0 and b"multiple" in capi_lib.vbhem_last_error()


TRIAL_SHAPES = [  # (name, N, K, S, Sb, d, cov, T, ragged, R)
    ("full_small", 7, 3, 3, 3, 2, 1, 6, False, 3),
    ("ragged_diag", 40, 3, 4, 4, 3, 0, 7, True, 4),
    ("C3like", 300, 8, 5, 5, 2, 0, 10, False, 5),
    ("C4like", 200, 16, 8, 8, 8, 1, 10, False, 4),
    ("K1", 30, 1, 3, 3, 2, 1, 5, False, 6),
    ("many", 500, 5, 4, 4, 2, 1, 8, False, 12),
]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", TRIAL_SHAPES, ids=[s[0] for s in TRIAL_SHAPES])
def test_fused_trials_match_separate(vb, shape):
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    name, N, K, S, Sb, d, cov, T, ragged, R = shape
    cs = make_case(N, K, S, Sb, d, cov, seed=len(name), ragged=ragged, tau=T)
    posts = _trial_posts(cs, R, len(name))
    bs = vb.BaseSet.from_numpy(cs["base"])
    tN = torch.as_tensor(100.0 * N * cs["base"]["omega"], device=DEV)
    consts = [host.cluster_constants(P, cov) for P in posts]
    logOm = [host.log_omega_tilde(P.alpha) for P in posts]
    from vbhem_amd.em import _stack_constants
    eng = EStepEngine(bs, R * K, S, T, device=DEV, trials=R)
    eng.set_clusters(_stack_constants(consts))
    eng.set_log_omega(np.concatenate(logOm))
    vec = eng.fused(tN).cpu().numpy()
    SL = host.stats_len(K, S, d, cov)
    assert vec.size == R * SL
    for r in range(R):
        one = EStepEngine(bs, K, S, T, device=DEV)
        one.set_clusters(consts[r])
        one.set_log_omega(logOm[r])
        ref = one.fused(tN).cpu().numpy()
        got = vec[r * SL:(r + 1) * SL]
        a = host.unpack_stats(got, K, S, d, cov)
        b = host.unpack_stats(ref, K, S, d, cov)
        for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
            assert rel_err(a[k], b[k]) < 1e-12, (name, r, k, rel_err(a[k], b[k]))
            assert stat_err(a[k], b[k]) < 1e-10, (name, r, k, stat_err(a[k], b[k]))
        for k in ("Lt1", "Lt7"):
            assert abs(a[k] - b[k]) <= 1e-12 * abs(b[k]) + 1e-12, (name, r, k)
        cols = slice(r * K, (r + 1) * K)
        # elementwise: log_Z = tilde_N (logOmega + L_elbo) ~ 1e4..1e5 carries ~1e-11
        # absolute rounding from the last-bit L_elbo differences noted below
        assert rel_err(eng.hatZ[:, cols].cpu().numpy(), one.hatZ.cpu().numpy()) < 1e-12
        assert hatz_err(eng.hatZ[:, cols].cpu().numpy(), one.hatZ.cpu().numpy()) < 1e-9
        # the emission GEMM shifts every mean by the average of ALL cluster means
        # (R*K of them here): shift-invariant algebra, last-bit differences in E
        assert rel_err(eng.LL[:, cols].cpu().numpy(), one.LL.cpu().numpy()) < 1e-13


@pytest.mark.gpu
def test_em_trials_match_separate_runs(vb):
    from vbhem_amd import em
    from vbhem_amd.estep import EStepEngine
    N, K, S, Sb, d, cov, T, R = 60, 3, 3, 3, 2, 1, 8, 4
    cs = make_case(N, K, S, Sb, d, cov, seed=11, tau=T)
    posts = _trial_posts(cs, R, 11)
    opt = dict(cs["opt"], max_iter=40, minDiff=1e-6)
    bs = vb.BaseSet.from_numpy(cs["base"])
    eng = EStepEngine(bs, R * K, S, T, device=DEV, trials=R)
    tr = em.vbhem_h3m_c_trials(posts, eng, opt)
    singles = []
    for r in range(R):
        one = EStepEngine(bs, K, S, T, device=DEV)
        singles.append(em.vbhem_h3m_c_step_fc(posts[r], one, opt))
    for r, (a, b) in enumerate(zip(tr.results, singles)):
        assert a.iters == b.iters, (r, a.iters, b.iters)
        assert np.allclose(a.LogLs, b.LogLs, rtol=1e-10, atol=0), r
        assert np.allclose(a.post.m, b.post.m, rtol=1e-9, atol=1e-12)
        assert hatz_err(a.hatZ.cpu().numpy(), b.hatZ.cpu().numpy()) < 1e-8
    assert tr.best == int(np.argmax([s.LL for s in singles]))


def test_em_trials_host_logic_cpu(vb):
    """vbhem_h3m_c_trials on the oracle stand-in engine (CPU): every trial follows
    vbhem_h3m_c_step_fc exactly (iterations, bounds, posteriors, labels), a trial
    that stops early keeps its own last E-step, and the best trial is argmax LL."""
    from oracle_engine import OracleEngine
    from vbhem_amd import em
    N, K, S, Sb, d, cov, T, R = 24, 3, 3, 3, 2, 1, 6, 3
    cs = make_case(N, K, S, Sb, d, cov, seed=5, tau=T)
    posts = _trial_posts(cs, R, 5)
    opt = dict(cs["opt"], max_iter=15, minDiff=1e-5)
    bs = vb.BaseSet.from_numpy(cs["base"])
    tr = em.vbhem_h3m_c_trials(posts, OracleEngine(bs, R * K, S, T, nthreads=1, trials=R), opt)
    iters = []
    for r in range(R):
        one = em.vbhem_h3m_c_step_fc(posts[r], OracleEngine(bs, K, S, T, nthreads=1), opt)
        a = tr.results[r]
        assert a.iters == one.iters
        np.testing.assert_array_equal(a.LogLs, one.LogLs)
        np.testing.assert_array_equal(a.post.m, one.post.m)
        np.testing.assert_array_equal(a.hatZ.numpy(), one.hatZ.numpy())
        np.testing.assert_array_equal(a.label.numpy(), one.label.numpy())
        iters.append(one.iters)
    assert tr.best == int(np.argmax(tr.LLall))

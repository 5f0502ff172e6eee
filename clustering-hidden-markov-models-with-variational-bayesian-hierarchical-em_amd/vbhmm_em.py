"""VB-HMM learning of the base HMMs (config C1).

The upstream stage that produces the HMMs VBHEM clusters:
``vbhmm_learn_batch`` -> ``vbhmm_learn`` -> ``vbhmm_em`` -> ``vbhmm_fb`` ->
``vbhmm_fb_mex`` (src/hmm/).  The forward-backward runs on the GPU through the
C-ABI (:func:`vbhmm.vbhmm_fb`, one lane per sequence); the per-iteration
statistics, lower bound and M-step are O(K^2 + K dim^2 + total fixations) host
work, restated here from:

* vbhmm_em.m:112-414  the EM loop (E-step :133-246, bound :251-275, convergence
  and NaN handling :277-349, M-step :352-408) and the output model :426-491;
* vbhmm_em_lb.m:74-257  the lower bound, :260-400 its derivatives with respect to
  the (transformed) hyperparameters;
* vbhmm_em_hyp.m + get_hypinfo.m  hyperparameter learning (``learn_hyps``): the
  bound maximised over the transformed hyperparameters with minimize_new.m's BFGS
  (:func:`hyp.minimize`), every evaluation an EM run from the trial's HMM
  ('inithmm', vbhmm_init.m:154-161) with the derivatives at its last E-step;
  vbhmm_learn.m:482-552 runs it on each unique random trial (uniqueLL.m);
* vbhmm_init.m:122-204  the initial posterior from a GMM; :27-43 the K = 1 and
  N <= K special cases of the 'random' mode;
* vbhmm_clip_hyps.m:20-85, vbhmm_learn.m:252-310 (defaults), :440-480 (random
  trials, best LL), :367-405 (model selection over K with +gammaln(K+1));
* vbhmm_learn_batch.m (one vbhmm_learn per subject);
* vbhmm_remove_empty.m (states with N < thresh removed, as vbhem_h3m_cluster.m:116-134).

The 'random' initialisation fits a GMM with MATLAB's ``gmdistribution.fit``
(Statistics Toolbox, 'Start' 'randSample', TolFun 1e-5; vbhmm_init.m:59-60),
which is not part of the reference.  :func:`gmm_fit_randsample` restates that
published algorithm (random data rows as means, uniform weights, diagonal
covariances of the data variances, EM until the relative log-likelihood change
is below 1e-5); MATLAB's random stream cannot be reproduced, so the draws come
from a seeded numpy generator and parity tests inject the same GMM into both
sides.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
from scipy.special import digamma, gammaln

from . import vbhmm


# ----------------------------------------------------------------------------
# options
# ----------------------------------------------------------------------------
def vbhmm_default_options(dim: int, **over) -> dict:
    """vbhmm_learn.m:252-310 (the fields the EM loop reads)."""
    defmu = {2: [256.0, 192.0], 3: [256.0, 192.0, 150.0]}.get(dim, [0.0] * dim)
    opt = dict(alpha0=0.1, mu0=defmu, W0=0.005, beta0=1.0, v0=5.0, epsilon0=0.1,
               initmode="random", numtrials=50, maxIter=100, minDiff=1e-5, seed=None,
               fix_clusters=0, fix_cov=None, verbose=0, learn_hyps=0, calc_LLderiv=0,
               minimizer="minimize-bfgs", hyp_length=100, sortclusters="f")
    opt["hyps_max"] = dict(alpha0=1.0686e13, epsilon0=1.0686e13, v0=1e4, beta0=1.0686e13,
                           W0=1.0686e13)
    opt["hyps_min"] = dict(alpha0=1.0686e-13, epsilon0=1.0686e-13, v0=2.0612e-09 + dim - 1,
                           beta0=1.0686e-13, W0=1.0686e-13)
    opt.update(over)
    opt["mu0"] = np.asarray(opt["mu0"], dtype=np.float64).reshape(-1)
    if opt["v0"] <= dim - 1:
        raise ValueError("v0 not large enough...should be > D-1")  # vbhmm_learn.m:319-321
    return opt


def vbhmm_clip_hyps(opt: dict):
    """vbhmm_clip_hyps.m:20-85: clip each hyperparameter into [min, max];
    returns (clipped options, clipped flags: +1 at max, -1 at min)."""
    out = dict(opt)
    clipped = {}
    for name in ("alpha0", "epsilon0", "v0", "beta0", "W0"):
        val = np.array(opt[name], dtype=np.float64, ndmin=1)
        flag = np.zeros(val.size)
        hi, lo = opt["hyps_max"][name], opt["hyps_min"][name]
        flag[val >= hi] = +1
        val = np.where(val >= hi, hi, val)
        flag[val <= lo] = -1
        val = np.where(val <= lo, lo, val)
        out[name] = val if np.ndim(opt[name]) else float(val[0])
        clipped[name] = flag
    return out, clipped


# ----------------------------------------------------------------------------
# initialisation
# ----------------------------------------------------------------------------
def gmm_fit_randsample(X: np.ndarray, K: int, rng: np.random.Generator, tolfun: float = 1e-5,
                       max_iter: int = 100, reg: float = 0.0) -> dict:
    """Stand-in for MATLAB gmdistribution.fit(X, K, 'Start', 'randSample',
    'Options', struct('TolFun', 1e-5)) (vbhmm_init.m:59-60): K random rows of X
    as means, uniform proportions, every covariance diag(var(X)); full-covariance
    EM until |dLL| <= TolFun * |LL|.  Returns dict(prior [K], mean [K][dim],
    cov [K][dim][dim])."""
    N, dim = X.shape
    mu = X[rng.choice(N, K, replace=False)].copy()
    var = X.var(axis=0, ddof=1) if N > 1 else np.ones(dim)
    cov = np.repeat(np.diag(var)[None], K, axis=0)
    pi = np.full(K, 1.0 / K)
    last = -np.inf
    for _ in range(max_iter):
        logp = np.zeros((N, K))
        for k in range(K):
            L = np.linalg.cholesky(cov[k] + reg * np.eye(dim))
            z = np.linalg.solve(L, (X - mu[k]).T)
            logp[:, k] = (np.log(pi[k]) - 0.5 * (z * z).sum(0) - np.log(np.diag(L)).sum()
                          - 0.5 * dim * np.log(2 * np.pi))
        mx = logp.max(1, keepdims=True)
        lse = mx[:, 0] + np.log(np.exp(logp - mx).sum(1))
        ll = lse.sum()
        post = np.exp(logp - lse[:, None])
        nk = post.sum(0) + 1e-300
        pi = nk / N
        mu = (post.T @ X) / nk[:, None]
        for k in range(K):
            d = X - mu[k]
            cov[k] = (d * post[:, k:k + 1]).T @ d / nk[k] + reg * np.eye(dim)
            cov[k] = 0.5 * (cov[k] + cov[k].T)
        if abs(ll - last) <= tolfun * abs(ll):
            break
        last = ll
    return dict(prior=pi, mean=mu, cov=cov)


def random_gmm(data: Sequence[np.ndarray], K: int, rng: np.random.Generator) -> dict:
    """The 'random' initmode's GMM (vbhmm_init.m:27-91): one Gaussian for K = 1,
    the data points themselves when N <= K, else a GMM fit."""
    X = np.concatenate([np.asarray(a, dtype=np.float64) for a in data], axis=0)
    N, dim = X.shape
    if K == 1:
        return dict(prior=np.ones(1), mean=X.mean(0, keepdims=True),
                    cov=np.cov(X.T, ddof=1).reshape(1, dim, dim))
    if N <= K:
        tmp = np.concatenate([np.ones(N), 1e-6 * np.ones(K - N)])
        mean = np.concatenate([X, np.zeros((K - N, dim))])
        v = X.var(axis=0, ddof=1) if N > 1 else np.ones(dim)
        return dict(prior=tmp / tmp.sum(), mean=mean,
                    cov=np.repeat((np.mean(v) * np.eye(dim))[None], K, axis=0))
    try:
        return gmm_fit_randsample(X, K, rng)
    except np.linalg.LinAlgError:  # ill-conditioned: regularised fit (vbhmm_init.m:63-70)
        return gmm_fit_randsample(X, K, rng, reg=1e-10)


def vbhmm_init(data: Sequence[np.ndarray], K: int, opt: dict, gmm: dict) -> dict:
    """vbhmm_init.m:122-204: the initial variational posterior from a GMM
    (prior [K], mean [K][dim], cov [K][dim][dim]), or ('inithmm') an HMM's own."""
    X = np.concatenate([np.asarray(a, dtype=np.float64) for a in data], axis=0)
    N, dim = X.shape
    if len(opt["mu0"]) != dim:
        raise ValueError(f"vbopt.mu0 should have dimension D={dim}")
    W0 = np.asarray(opt["W0"], dtype=np.float64)
    W0m = float(W0) * np.eye(dim) if W0.size == 1 else np.diag(W0.reshape(-1))
    W0inv = np.linalg.inv(W0m)
    beta0, v0, m0 = float(opt["beta0"]), float(opt["v0"]), opt["mu0"]
    W0mode = "iid" if W0.size == 1 else "diag"
    if opt.get("initmode") == "inithmm":  # vbhmm_init.m:154-161: the HMM's own posterior
        vp = opt["inithmm"]["varpar"]
        return dict(alpha=np.array(vp["alpha"], float), epsilon=np.array(vp["epsilon"], float),
                    beta=np.array(vp["beta"], float), v=np.array(vp["v"], float),
                    m=np.array(vp["m"], float), W=np.array(vp["W"], float), W0inv=W0inv,
                    W0mode=W0mode)
    Nk = N * np.asarray(gmm["prior"], dtype=np.float64).reshape(-1)
    Nk2 = np.full(K, N / K)
    xbar = np.asarray(gmm["mean"], dtype=np.float64).reshape(K, dim)
    S = np.asarray(gmm["cov"], dtype=np.float64).reshape(K, dim, dim)
    alpha = opt["alpha0"] + Nk2
    epsilon = np.repeat((opt["epsilon0"] + Nk2)[None, :], K, axis=0)
    beta = beta0 + Nk
    v = v0 + Nk + 1
    m = (beta0 * m0[None, :] + Nk[:, None] * xbar) / beta[:, None]
    W = np.zeros((K, dim, dim))
    for k in range(K):
        mult1 = beta0 * Nk[k] / (beta0 + Nk[k])
        diff3 = xbar[k] - m0
        W[k] = np.linalg.inv(W0inv + Nk[k] * S[k] + mult1 * np.outer(diff3, diff3))
    return dict(alpha=alpha, epsilon=epsilon, beta=beta, v=v, m=m, W=W, W0inv=W0inv,
                W0mode=W0mode)


# ----------------------------------------------------------------------------
# lower bound (vbhmm_em_lb.m) and its hyperparameter derivatives
# ----------------------------------------------------------------------------
def vbhmm_em_lb(st: dict, opt: dict, vp: dict, fb: dict, do_deriv: bool = False,
                clipped: Optional[dict] = None):
    """vbhmm_em_lb.m:74-257 (usegroups = 0); with ``do_deriv`` also :260-400, the
    bound's derivatives with respect to the hyperparameters at this posterior
    (returns (LB, dLB), dLB keyed as the reference's d_LB: d_logalpha0,
    d_logepsilon0, d_logv0D1, d_sqrtv0D1, d_logbeta0, d_sqrtbeta0, d_sqrtW0inv,
    d_logW0, d_m0), a derivative set to 0 where its hyperparameter is clipped and
    moving past the limit would raise the bound."""
    dim, K = st["dim"], st["K"]
    alpha0, epsilon0, beta0, v0 = opt["alpha0"], opt["epsilon0"], opt["beta0"], opt["v0"]
    m0, W0inv = opt["mu0"], st["W0inv"]
    v, W, eps, alpha, m, beta = vp["v"], vp["W"], vp["epsilon"], vp["alpha"], vp["m"], vp["beta"]
    lLT, lPi, lA = fb["logLambdaTilde"], fb["logPiTilde"], fb["logATilde"]
    logdetW0inv = (dim * np.log(W0inv[0, 0]) if st["W0mode"] == "iid"
                   else np.log(np.diag(W0inv)).sum())
    q = np.arange(1, dim + 1)
    logCalpha0 = gammaln(K * alpha0) - K * gammaln(alpha0)
    logCepsilon0 = np.full(K, gammaln(K * epsilon0) - K * gammaln(epsilon0))
    logB0 = ((v0 / 2) * logdetW0inv - (v0 * dim / 2) * np.log(2) - (dim * (dim - 1) / 4) * np.log(np.pi)
             - gammaln(0.5 * (v0 + 1 - q)).sum())
    logCalpha = gammaln(alpha.sum()) - gammaln(alpha).sum()
    logCeps = gammaln(eps.sum(1)) - gammaln(eps).sum(1)
    H = 0.0
    trSW = np.zeros(K)
    xWx = np.zeros(K)
    mWm = np.zeros(K)
    trW0W = np.zeros(K)
    for k in range(K):
        logBk = (-(v[k] / 2) * np.log(np.linalg.det(W[k])) - (v[k] * dim / 2) * np.log(2)
                 - (dim * (dim - 1) / 4) * np.log(np.pi) - gammaln(0.5 * (v[k] + 1 - q)).sum())
        H = H - logBk - 0.5 * (v[k] - dim - 1) * lLT[k] + 0.5 * v[k] * dim
        trSW[k] = np.trace(st["t1_S"][k] @ W[k])
        dx = st["xbar"][k] - m[k]
        xWx[k] = dx @ W[k] @ dx
        dm = m[k] - m0
        mWm[k] = dm @ W[k] @ dm
        trW0W[k] = np.trace(W0inv @ W[k])
    Nk = st["Nk"]
    Lt1 = 0.5 * (Nk * (lLT - dim / beta - v * trSW - v * xWx - dim * np.log(2 * np.pi))).sum()
    gamma1 = fb["gamma_all"][:, :, 0]
    Lt2a = (gamma1 * lPi[:, None]).sum()
    Lt2b = (st["M"] * lA).sum()
    Lt2 = Lt2a + Lt2b
    Lt3 = logCalpha0 + (alpha0 - 1) * lPi.sum()
    Lt4 = (logCepsilon0 + (epsilon0 - 1) * lA.sum(1)).sum()
    Lt51 = 0.5 * (dim * np.log(beta0 / (2 * np.pi)) + lLT - dim * beta0 / beta - beta0 * v * mWm).sum()
    Lt52 = K * logB0 + 0.5 * (v0 - dim - 1) * lLT.sum() - 0.5 * (v * trW0W).sum()
    Lt5 = Lt51 + Lt52
    Lt63 = (fb["gamma_all"] * fb["logrho_Saved"]).sum()
    Lt64 = fb["phi_norm"].sum()
    Lt6 = Lt2a + Lt2b + Lt63 - Lt64
    Lt7 = ((alpha - 1) * lPi).sum() + logCalpha + (((eps - 1) * lA).sum(1) + logCeps).sum()
    Lt8 = 0.5 * (lLT + dim * np.log(beta / (2 * np.pi))).sum() - 0.5 * dim * K - H
    LB = float(Lt1 + Lt2 + Lt3 + Lt4 + Lt5 - Lt6 - Lt7 - Lt8)
    if not do_deriv:
        return LB
    # vbhmm_em_lb.m:263-320: the partial derivatives of Lt3 (alpha0), Lt4 (epsilon0)
    # and Lt5 (v0, beta0, W0, m0) -- the only terms holding hyperparameters
    d = {}
    d["alpha0"] = np.atleast_1d(K * digamma(K * alpha0) - K * digamma(alpha0) + lPi.sum())
    d["epsilon0"] = np.atleast_1d(K * (K * digamma(K * epsilon0) - K * digamma(epsilon0)) + lA.sum())
    dlogB0_dv0 = 0.5 * logdetW0inv - (dim / 2) * np.log(2) - 0.5 * digamma(0.5 * (v0 + 1 - q)).sum()
    d["v0"] = np.atleast_1d(K * dlogB0_dv0 + 0.5 * lLT.sum())
    d["beta0"] = np.atleast_1d(0.5 * (dim / beta0 - dim / beta - v * mWm).sum())
    trW = np.array([np.trace(W[k]) for k in range(K)])
    if st["W0mode"] == "iid":
        myW0inv = W0inv[0, 0]
        d_trW0invW = -(myW0inv ** 2) * trW                                  # [K]
        d["W0"] = np.atleast_1d(K * (-0.5 * v0 * dim * myW0inv) - 0.5 * (v * d_trW0invW).sum())
    else:
        myW0inv = np.diag(W0inv).copy()
        d_trW0invW = -(myW0inv[:, None] ** 2) * np.stack([np.diag(W[k]) for k in range(K)], 1)  # [dim][K]
        d["W0"] = K * (-0.5 * v0 * myW0inv) - 0.5 * (v[None, :] * d_trW0invW).sum(1)
    myW0 = 1.0 / myW0inv
    d["m0"] = sum(beta0 * v[k] * (W[k] @ (m[k] - m0)) for k in range(K))
    # :326-341: a clipped hyperparameter's derivative is zeroed where moving further
    # past its limit would raise the bound
    for name, flags in (clipped or {}).items():
        g = d[name]
        for j, fl in enumerate(np.atleast_1d(flags)):
            if (fl == +1 and g[j] > 0) or (fl == -1 and g[j] < 0):
                g[j] = 0.0
    # :387-398: derivatives of the transformed hyperparameters
    dLB = dict(d_logalpha0=d["alpha0"] * alpha0, d_logepsilon0=d["epsilon0"] * epsilon0,
               d_logv0D1=d["v0"] * (v0 - dim + 1), d_sqrtv0D1=d["v0"] * 2 * np.sqrt(v0 - dim + 1),
               d_logbeta0=d["beta0"] * beta0, d_sqrtbeta0=d["beta0"] * 2 * np.sqrt(beta0),
               d_sqrtW0inv=d["W0"] * (myW0 ** 1.5) * (-2), d_logW0=d["W0"] * myW0,
               d_m0=np.asarray(d["m0"], dtype=np.float64))
    return LB, dLB


# ----------------------------------------------------------------------------
# EM
# ----------------------------------------------------------------------------
def vbhmm_em(data: Sequence[np.ndarray], K: int, opt: dict, gmm: Optional[dict] = None,
             rng: Optional[np.random.Generator] = None, device="cuda",
             batch: Optional["vbhmm.SequenceBatch"] = None) -> dict:
    """vbhmm_em.m:1-491 (usegroups = 0): EM from the posterior vbhmm_init builds
    out of ``gmm`` (or a 'random' GMM drawn with ``rng``; or opt['inithmm'] when
    opt['initmode'] == 'inithmm').  Returns the output HMM (prior, trans, pdf, LL,
    gamma, M, N1, N, varpar) plus the bound trajectory ``LLs``, and with
    opt['calc_LLderiv'] the bound's hyperparameter derivatives ``dLL``."""
    data = [np.asarray(a, dtype=np.float64).reshape(-1, len(opt["mu0"])) for a in data]
    opt, clipped = vbhmm_clip_hyps(opt)
    if gmm is None and opt.get("initmode") != "inithmm":
        gmm = random_gmm(data, K, rng if rng is not None else np.random.default_rng(0))
    mix = vbhmm_init(data, K, opt, gmm)
    dim = len(opt["mu0"])
    lens = np.array([a.shape[0] for a in data])
    N, maxT = len(data), int(lens.max())
    X = np.concatenate(data, axis=0)
    n_idx = np.repeat(np.arange(N), lens)
    t_idx = np.concatenate([np.arange(n) for n in lens])
    sb = batch if batch is not None else vbhmm.SequenceBatch(data, dim, device)
    alpha, eps, beta, v, m, W = (mix[k].copy() for k in ("alpha", "epsilon", "beta", "v", "m", "W"))
    alpha0, eps0, beta0, v0, m0 = opt["alpha0"], opt["epsilon0"], opt["beta0"], opt["v0"], opt["mu0"]
    W0inv = mix["W0inv"]
    L = lastL = -np.finfo(float).max
    LLs: List[float] = []
    dLL = None
    C = np.zeros((K, dim, dim))
    unstable = False
    for it in range(1, int(opt["maxIter"]) + 1):
        vp = dict(v=v, W=W, epsilon=eps, alpha=alpha, m=m, beta=beta)
        fb = vbhmm.vbhmm_fb(data, vp, batch=sb)                      # GPU (vbhmm_fb_mex.c)
        g_all = fb["gamma_all"]                                       # [K, N, maxT]
        Nk1 = g_all[:, :, 0].sum(1) + 1e-50
        Nk = g_all.sum(axis=(1, 2)) + 1e-50
        M = fb["xi_sum"].sum(2)
        G = g_all[:, n_idx, t_idx]                                    # gamma_block [K, totalT]
        xbar = (G @ X) / Nk[:, None]
        t1_S = np.zeros((K, dim, dim))
        for k in range(K):
            d1 = X - xbar[k]
            t1_S[k] = (d1 * G[k][:, None]).T @ d1 / Nk[k]
        if it > 1:
            lastL = L
        st = dict(dim=dim, K=K, N=N, W0inv=W0inv, W0mode=mix["W0mode"], t1_S=t1_S, xbar=xbar,
                  Nk=Nk, M=M)
        L = vbhmm_em_lb(st, opt, vp, fb)
        do_break = False
        if it > 1 and abs((L - lastL) / lastL) <= opt["minDiff"]:
            do_break = True
        if it == opt["maxIter"]:
            do_break = True
        if np.isnan(L):  # vbhmm_em.m:314-330
            do_break, unstable, L = True, True, -np.inf
        LLs.append(L)
        if do_break and opt.get("calc_LLderiv", 0):
            # vbhmm_em.m:332-343: the derivatives at the last E-step, before its M-step
            # (NaN when the run went unstable)
            _, dLL = vbhmm_em_lb(st, opt, vp, fb, do_deriv=True, clipped=clipped)
            if unstable:
                dLL = {k: np.full_like(np.asarray(g, dtype=float), np.nan) for k, g in dLL.items()}
        if do_break and unstable:
            break
        # M-step (vbhmm_em.m:352-408)
        alpha = alpha0 + Nk1
        eps = eps0 + M
        if not opt.get("fix_clusters", 0):
            beta = beta0 + Nk
            v = v0 + Nk + 1
            m = (beta0 * m0[None, :] + Nk[:, None] * xbar) / beta[:, None]
            for k in range(K):
                if opt.get("fix_cov") is None:
                    mult1 = beta0 * Nk[k] / (beta0 + Nk[k])
                    diff3 = xbar[k] - m0
                    Wk = np.linalg.inv(W0inv + Nk[k] * t1_S[k] + mult1 * np.outer(diff3, diff3))
                    W[k] = 0.5 * (Wk + Wk.T)
                else:
                    W[k] = np.linalg.inv(opt["fix_cov"]) / (v[k] - dim - 1)
        for k in range(K):
            Ck = np.linalg.inv(W[k]) / ((v[k] - dim - 1) if v[k] > dim + 1 else v[k])
            C[k] = 0.5 * (Ck + Ck.T)
        if do_break:
            break
    prior = alpha / alpha.sum()
    sc = eps.sum(1, keepdims=True)
    trans = eps / np.where(sc == 0, 1.0, sc)
    return dict(prior=prior, trans=trans,
                pdf=[dict(mean=m[k].copy(), cov=C[k].copy()) for k in range(K)],
                LL=float(L), LLs=np.array(LLs), iters=it, unstable=unstable,
                gamma=[g_all[:, n, :lens[n]].copy() for n in range(N)], M=M, N1=Nk1, N=Nk,
                varpar=dict(epsilon=eps, alpha=alpha, beta=beta, v=v, m=m, W=W.copy()),
                clipped=clipped, dLL=dLL)


# ----------------------------------------------------------------------------
# hyperparameter learning (vbhmm_em_hyp.m, get_hypinfo.m, uniqueLL.m)
# ----------------------------------------------------------------------------
VBHMM_HYPS = ("alpha0", "epsilon0", "v0", "beta0", "W0", "mu0")


def vbhmm_hypinfo(learn_hyps, opt: dict) -> list:
    """get_hypinfo.m:13-79: per learnable hyperparameter its optimiser-space
    transform, inverse, derivative key and size ('W0' = the sqrt(W0inv) transform)."""
    from .hyp import HypInfo
    dim = len(opt["mu0"])
    names = VBHMM_HYPS if (learn_hyps is True or (np.isscalar(learn_hyps) and learn_hyps == 1)) \
        else tuple(learn_hyps)
    out = []
    for h in names:
        if h in ("alpha0", "epsilon0", "beta0"):
            out.append(HypInfo(h, "d_log" + h, np.exp, np.log, 1))
        elif h == "v0":
            out.append(HypInfo("v0", "d_logv0D1", lambda x: np.exp(x) + dim - 1,
                               lambda x: np.log(x - dim + 1), 1))
        elif h in ("W0", "W0isqrt"):
            out.append(HypInfo("W0", "d_sqrtW0inv", lambda x: x ** (-2.0),
                               lambda x: 1.0 / np.sqrt(x), int(np.size(opt["W0"]))))
        elif h == "W0log":
            out.append(HypInfo("W0", "d_logW0", np.exp, np.log, int(np.size(opt["W0"]))))
        elif h == "mu0":
            out.append(HypInfo("mu0", "d_m0", lambda x: x, lambda x: x, dim))
        else:
            raise ValueError("bad value of learn_hyp")
    return out


def _set_hyps(X: np.ndarray, opt: dict, info: list) -> dict:
    """vbhmm_em_hyp.m set_vbopt: optimiser vector -> options."""
    o = dict(opt)
    i = 0
    for h in info:
        with np.errstate(over="ignore"):  # a line-search probe may overflow; clipped later
            val = np.asarray(h.trans(X[i:i + h.dims]), dtype=np.float64)
        o[h.optname] = float(val[0]) if (h.dims == 1 and np.ndim(opt[h.optname]) == 0) else val
        i += h.dims
    o["mu0"] = np.asarray(o["mu0"], dtype=np.float64).reshape(-1)
    return o


def vbhmm_em_hyp(data: Sequence[np.ndarray], K: int, opt: dict, inithmm: dict, device="cuda",
                 batch: Optional["vbhmm.SequenceBatch"] = None) -> dict:
    """vbhmm_em_hyp.m:15-126: maximise the bound over the transformed
    hyperparameters (minimize_new.m, p.length = opt['hyp_length'], BFGS by default),
    every evaluation an EM run from ``inithmm`` with its derivatives (vbhmm_grad,
    :172-190), then one EM run at the optimum; the result carries ``learn_hyps``
    (hypinfo names, opt_transhyp, opt_L, the optimised hyperparameters)."""
    from . import hyp
    dim = len(opt["mu0"])
    data = [np.asarray(a, dtype=np.float64).reshape(-1, dim) for a in data]
    sb = batch if batch is not None else vbhmm.SequenceBatch(data, dim, device)
    info = vbhmm_hypinfo(opt.get("learn_hyps", 1) or 1, opt)
    base = dict(opt, initmode="inithmm", inithmm=inithmm)
    n_eval = [0]

    def grad(X):
        o = _set_hyps(X, base, info)
        o["calc_LLderiv"] = 1
        h = vbhmm_em(data, K, o, batch=sb)
        n_eval[0] += 1
        return -h["LL"], np.concatenate([-np.atleast_1d(h["dLL"][i.derivname]).reshape(-1) for i in info])

    methods = {"minimize-bfgs": "BFGS", "minimize-lbfgs": "LBFGS", "minimize-cg": "CG"}
    name = opt.get("minimizer", "minimize-bfgs")
    if name not in methods:  # 'fminunc' needs MATLAB's Optimization Toolbox
        raise ValueError("bad minimizer specified")
    X0 = hyp.init_x(opt, info)
    Xopt, fX, nls = hyp.minimize(X0, grad, length=int(opt.get("hyp_length", 100)), method=methods[name])
    o2 = _set_hyps(Xopt, base, info)
    o2["calc_LLderiv"] = 0
    h = vbhmm_em(data, K, o2, batch=sb)
    h["learn_hyps"] = dict(hypinfo=[i.optname for i in info], opt_transhyp=Xopt, opt_L=-fX[-1],
                           fX=fX, line_searches=nls, evaluations=n_eval[0],
                           vbopt={i.optname: o2[i.optname] for i in info})
    return h


def vbhmm_learn(data: Sequence[np.ndarray], Ks, opt: dict, device="cuda",
                gmms: Optional[dict] = None) -> dict:
    """vbhmm_learn.m (initmode 'random'): for each K, numtrials EM runs from random
    GMMs (seeded by opt['seed'], vbhmm_learn.m:443-451; K = 1 needs one); with
    opt['learn_hyps'] every unique trial (uniqueLL, 2 minDiff 10 apart) is re-run
    through :func:`vbhmm_em_hyp` (:482-552); keep the best bound; over several K,
    select by LL + gammaln(K+1) (:367-405).  ``gmms[K]`` = list of GMMs to inject
    instead of random draws."""
    Ks = [int(k) for k in np.atleast_1d(Ks)]
    dim = len(opt["mu0"])
    data = [np.asarray(a, dtype=np.float64).reshape(-1, dim) for a in data]
    sb = vbhmm.SequenceBatch(data, dim, device)
    out_all = []
    for K in Ks:
        rng = np.random.default_rng(opt["seed"])
        if gmms is not None and K in gmms:
            inits = list(gmms[K])
        else:
            numits = 1 if K == 1 else int(opt["numtrials"])
            inits = [random_gmm(data, K, rng) for _ in range(numits)]
        trials = [vbhmm_em(data, K, opt, gmm=g, batch=sb) for g in inits]
        LLall = np.array([h["LL"] for h in trials])
        LLall_random, trials_random = LLall.copy(), list(trials)
        learn = _do_learn_hyps(opt.get("learn_hyps", 0))
        if learn or opt.get("keep_suboptimal_hmms", 0):
            from .cluster import unique_ll   # uniqueLL.m
            uniq = unique_ll(LLall, 2 * opt["minDiff"] * 10)
        if learn:
            LLall = np.full(len(trials), np.nan)
            for it in uniq:
                trials[it] = vbhmm_em_hyp(data, K, opt, trials_random[it], batch=sb)
                LLall[it] = trials[it]["LL"]
        best = trials[int(np.nanargmax(LLall))]
        best["trials_LL"] = LLall
        if opt.get("keep_suboptimal_hmms", 0):  # vbhmm_learn.m:600-602 (the random trials)
            best["suboptimal_hmms"] = [trials_random[it] for it in uniq]
        if learn:
            best["trials_LL_random"] = LLall_random
            if opt.get("keep_best_random_trial", 0):  # vbhmm_learn.m:587-596
                tmp = trials_random[int(np.argmax(LLall_random))]
                if opt.get("sortclusters"):
                    tmp = vbhmm_standardize(tmp, opt["sortclusters"])
                best["learn_hyps"]["hmm_best_random_trial"] = tmp
        if opt.get("sortclusters"):  # vbhmm_learn.m:635-640
            best = vbhmm_standardize(best, opt["sortclusters"])
        out_all.append(best)
    if len(Ks) == 1:
        return out_all[0]
    LLk = np.array([h["LL"] for h in out_all]) + gammaln(np.array(Ks) + 1.0)
    ind = int(np.argmax(LLk))
    h = dict(out_all[ind])
    h.update(model_LL=LLk, model_k=Ks, model_bestK=Ks[ind], model_all=out_all, LL=float(LLk[ind]))
    if opt.get("keep_suboptimal_hmms", 0):  # :417-424: every K's unique trials
        h["suboptimal_hmms"] = [q for o in out_all for q in o["suboptimal_hmms"]]
    if opt.get("sortclusters"):  # :635-640 (again; idempotent for the sub-calls' order)
        h = vbhmm_standardize(h, opt["sortclusters"])
    return h


def vbhmm_permute(hmm: dict, cl) -> dict:
    """vbhmm_permute.m (usegroups = 0): the states reordered by ``cl`` (0-based)."""
    cl = np.asarray(cl, dtype=np.int64)
    out = dict(hmm)
    out["prior"] = np.asarray(hmm["prior"])[cl]
    out["trans"] = np.asarray(hmm["trans"])[np.ix_(cl, cl)]
    for k in ("M",):
        if k in hmm:
            out[k] = np.asarray(hmm[k])[np.ix_(cl, cl)]
    for k in ("N1", "N"):
        if k in hmm:
            out[k] = np.asarray(hmm[k])[cl]
    out["pdf"] = [hmm["pdf"][k] for k in cl]
    if "gamma" in hmm:
        out["gamma"] = [np.asarray(g)[cl] for g in hmm["gamma"]]
    if "varpar" in hmm:
        vp = hmm["varpar"]
        out["varpar"] = dict(vp, epsilon=np.asarray(vp["epsilon"])[np.ix_(cl, cl)],
                             alpha=np.asarray(vp["alpha"])[cl], beta=np.asarray(vp["beta"])[cl],
                             v=np.asarray(vp["v"])[cl], m=np.asarray(vp["m"])[cl],
                             W=np.asarray(vp["W"])[cl])
    return out


def vbhmm_prob_steadystate(hmm: dict) -> np.ndarray:
    """vbhmm_prob_steadystate.m computep: the stationary distribution (least squares
    of [A' - I; 1] p = [0; 1]), or the prior for an identity transition matrix."""
    A = np.asarray(hmm["trans"], dtype=float)
    d = A.shape[0]
    if np.all(np.abs(A - np.eye(d)) < 1e-6):
        return np.asarray(hmm["prior"], dtype=float)
    M = np.vstack([A.T - np.eye(d), np.ones((1, d))])
    return np.linalg.lstsq(M, np.r_[np.zeros(d), 1.0], rcond=None)[0]


def vbhmm_standardize(hmm: dict, mode: str) -> dict:
    """vbhmm_standardize.m: reorder the states -- 'e' (or 'd') by size N, 's' by the
    steady-state probability, 'p' by the prior (all descending, stable), 'f' along the
    most likely fixation path (the prior's argmax, then each row's argmax among the
    states not visited yet), 'l' / 'r' by the first mean coordinate ascending /
    descending."""
    if mode in ("d", "e"):
        wi = np.argsort(-np.asarray(hmm["N"], dtype=float), kind="stable")
    elif mode == "s":
        wi = np.argsort(-vbhmm_prob_steadystate(hmm), kind="stable")
    elif mode == "p":
        wi = np.argsort(-np.asarray(hmm["prior"], dtype=float).reshape(-1), kind="stable")
    elif mode == "f":
        A = np.array(hmm["trans"], dtype=float)
        p = np.asarray(hmm["prior"], dtype=float).reshape(-1)
        wi = []
        for t in range(p.size):
            cur = int(np.argmax(p)) if t == 0 else int(np.argmax(A[cur]))
            wi.append(cur)
            A[:, cur] = -1.0
    elif mode in ("l", "r"):
        x = np.array([np.asarray(q["mean"]).reshape(-1)[0] for q in hmm["pdf"]])
        wi = np.argsort(x if mode == "l" else -x, kind="stable")
    else:
        raise ValueError("unknown mode")
    return vbhmm_permute(hmm, wi)


def _do_learn_hyps(v) -> bool:
    """vbhmm_learn.m:357-361: a list of names, or 1."""
    return isinstance(v, (list, tuple)) or (np.isscalar(v) and v == 1)


def vbhmm_learn_batch(datas: Sequence[Sequence[np.ndarray]], Ks, opt: dict, device="cuda",
                      gmms: Optional[list] = None):
    """vbhmm_learn_batch.m: one vbhmm_learn per subject; returns (hmms, LLs).  With
    opt['learn_hyps_batch'] (:84-189) one set of hyperparameters shared by every
    subject: each subject's unique random trials (keep_suboptimal_hmms) seed EM runs,
    and BFGS (minimize_new.m, length 100) minimises the mean over subjects of the
    best -(LL + gammaln(K+1)) among that subject's runs (vbhmm_grad_batch_parfor,
    :347-457); the returned HMMs are the final run's, each with its ``vbopt``."""
    lhb = opt.get("learn_hyps_batch", 0)
    if not (isinstance(lhb, (list, tuple)) or lhb):
        hmms = [vbhmm_learn(d, Ks, opt, device, gmms[i] if gmms is not None else None)
                for i, d in enumerate(datas)]
        return hmms, np.array([h["LL"] for h in hmms])
    from . import hyp
    if not isinstance(lhb, (list, tuple)):
        if lhb != 1:
            raise ValueError("learn_hyps_batch not set properly")
        lhb = list(VBHMM_HYPS)
    opt = dict(opt, learn_hyps=0)            # :97-101: individual learning is switched off
    info = vbhmm_hypinfo(list(lhb), opt)
    dim = len(opt["mu0"])
    datas = [[np.asarray(a, dtype=np.float64).reshape(-1, dim) for a in d] for d in datas]
    batches = [vbhmm.SequenceBatch(d, dim, device) for d in datas]
    iopt = dict(opt, keep_suboptimal_hmms=1)
    inithmms = [vbhmm_learn(d, Ks, iopt, device, gmms[i] if gmms is not None else None)
                for i, d in enumerate(datas)]

    def grad_batch(X, keep=False):
        nL, dnL, out = 0.0, 0.0, []
        for n, d in enumerate(datas):
            o = _set_hyps(X, dict(opt, initmode="inithmm", calc_LLderiv=1), info)
            best = None
            for q in inithmms[n]["suboptimal_hmms"]:
                K = len(q["pdf"])
                qh = vbhmm_em(d, K, dict(o, inithmm=q), batch=batches[n])
                qnL = -qh["LL"] - gammaln(K + 1)
                if best is None or qnL < best[0]:   # MATLAB min: the first of equal values
                    best = (qnL, qh)
            nL += best[0]
            dnL = dnL - np.concatenate([np.atleast_1d(best[1]["dLL"][i.derivname]).reshape(-1) for i in info])
            if keep:
                best[1]["vbopt"] = {i.optname: o[i.optname] for i in info}
                out.append(best[1])
        N = len(datas)
        return (nL / N, dnL / N, out) if keep else (nL / N, dnL / N)

    methods = {"minimize-bfgs": "BFGS", "minimize-lbfgs": "LBFGS", "minimize-cg": "CG"}
    name = opt.get("minimizer", "minimize-bfgs")
    if name not in methods:
        raise ValueError("bad minimizer specified")
    X0 = hyp.init_x(opt, info)
    Xopt, fX, nls = hyp.minimize(X0, grad_batch, length=100, method=methods[name])
    _, _, hmms = grad_batch(Xopt, keep=True)
    for h in hmms:
        h["learn_hyps_batch"] = dict(hypinfo=[i.optname for i in info], opt_transhyp=Xopt,
                                     opt_L=-fX[-1], fX=fX, line_searches=nls)
    if opt.get("sortclusters"):  # vbhmm_learn_batch.m:202-209
        hmms = [vbhmm_standardize(h, opt["sortclusters"]) for h in hmms]
    return hmms, np.array([h["LL"] for h in hmms])


def vbhmm_remove_empty(hmm: dict, thresh: float = 1.0) -> dict:
    """vbhmm_remove_empty.m:32-103 (usegroups = 0): drop states with N < thresh,
    renormalise gamma, prior and trans from the kept variational parameters."""
    keep = np.flatnonzero(~(np.asarray(hmm["N"]) < thresh))
    if keep.size == len(hmm["N"]):
        return hmm
    vp = hmm["varpar"]
    nvp = dict(alpha=vp["alpha"][keep], epsilon=vp["epsilon"][np.ix_(keep, keep)],
               beta=vp["beta"][keep], v=vp["v"][keep], m=vp["m"][keep], W=vp["W"][keep])
    out = dict(hmm)
    out["varpar"] = nvp
    out["M"] = hmm["M"][np.ix_(keep, keep)]
    out["N1"] = hmm["N1"][keep]
    out["N"] = hmm["N"][keep]
    out["gamma"] = [g[keep] / g[keep].sum(0, keepdims=True) for g in hmm["gamma"]]
    out["prior"] = nvp["alpha"] / nvp["alpha"].sum()
    out["trans"] = nvp["epsilon"] / nvp["epsilon"].sum(1, keepdims=True)
    out["pdf"] = [hmm["pdf"][k] for k in keep]
    return out

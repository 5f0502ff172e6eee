"""Oracle (TEST INFRASTRUCTURE ONLY): a loop-for-loop CPU restatement of the
VB-HMM EM of src/hmm/vbhmm_em.m + vbhmm_em_lb.m + vbhmm_init.m (usegroups = 0,
no derivatives), written in the .m files' own order and index conventions
(column-major m [dim x K], W [dim x dim x K], gamma [K x N x maxT]).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
oracle/.  The forward-backward comes from the C restatement of vbhmm_fb_mex.c
(vbhem_oracle.c_vbhmm_fb) or the numpy twin of vbhmm_fb.m (twin_vbhmm_fb).
Parity unpinned at the MATLAB builtins (psi, gammaln, det, inv: SciPy/numpy
here) and at the GMM initialiser (gmdistribution.fit, absent): tests inject
the same GMM into the product and this oracle.
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln

import vbhem_oracle as vo


def init_from_gmm(data, K, opt, gmm):
    """vbhmm_init.m:122-204 ('random' / 'initgmm' branch after the GMM)."""
    X = np.concatenate([np.asarray(a, float) for a in data], axis=0)
    N, dim = X.shape
    m0 = np.asarray(opt["mu0"], float).reshape(dim, 1)
    W0 = np.asarray(opt["W0"], float)
    W0m = float(W0) * np.eye(dim) if W0.size == 1 else np.diag(W0.ravel())     # :135-146
    W0inv = np.linalg.inv(W0m)                                                   # :151
    PC = np.asarray(gmm["prior"], float).ravel()
    Nk = (N * PC).reshape(K, 1)                                                   # :165
    Nk2 = np.full((K, 1), N / K)                                                 # :166
    xbar = np.asarray(gmm["mean"], float).reshape(K, dim).T                       # :168 (dim x K)
    S = np.asarray(gmm["cov"], float).reshape(K, dim, dim).transpose(1, 2, 0)      # dim x dim x K
    alpha = opt["alpha0"] + Nk2                                                   # :187
    epsilon = np.zeros((K, K))
    for k in range(K):
        epsilon[k, :] = opt["epsilon0"] + Nk2[:, 0]                                # :188-190
    beta = opt["beta0"] + Nk                                                       # :191
    v = opt["v0"] + Nk + 1                                                         # :192
    m = ((opt["beta0"] * m0) @ np.ones((1, K)) + (np.ones((dim, 1)) @ Nk.T) * xbar) / (
        np.ones((dim, 1)) @ beta.T)                                                # :193
    W = np.zeros((dim, dim, K))
    for k in range(K):                                                             # :195-199
        mult1 = opt["beta0"] * Nk[k, 0] / (opt["beta0"] + Nk[k, 0])
        diff3 = xbar[:, k:k + 1] - m0
        W[:, :, k] = np.linalg.inv(W0inv + Nk[k, 0] * S[:, :, k] + mult1 * (diff3 @ diff3.T))
    return dict(alpha=alpha[:, 0], epsilon=epsilon, beta=beta[:, 0], v=v[:, 0], m=m, W=W,
                W0inv=W0inv, W0mode="iid" if W0.size == 1 else "diag", m0=m0)


def lower_bound(dim, K, alpha0, epsilon0, m0, beta0, v0, W0inv, W0mode, t1_S, xbar, Nk, M,
                v, W, epsilon, alpha, m, beta, fb):
    """vbhmm_em_lb.m:74-257 term by term (usegroups = 0)."""
    logrho, gam, phi = fb["logrho"], fb["gamma"], fb["phi_norm"]     # [K x N x maxT]
    lLT, lPi, lA = fb["logLambdaTilde"], fb["logPiTilde"], fb["logATilde"]
    N = gam.shape[1]
    if W0mode == "iid":
        logdetW0inv = dim * np.log(W0inv[0, 0])                                      # :77
    else:
        logdetW0inv = np.sum(np.log(np.diag(W0inv)))                                 # :79
    logCalpha0 = gammaln(K * alpha0) - K * gammaln(alpha0)                          # :84
    logCepsilon0 = [gammaln(K * epsilon0) - K * gammaln(epsilon0) for _ in range(K)]
    qq = np.arange(1, dim + 1)
    logB0 = ((v0 / 2) * logdetW0inv - (v0 * dim / 2) * np.log(2) - (dim * (dim - 1) / 4) * np.log(np.pi)
             - np.sum(gammaln(0.5 * (v0 + 1 - qq))))                                 # :88-89
    logCalpha = gammaln(np.sum(alpha)) - np.sum(gammaln(alpha))                      # :92
    logCepsilon = [gammaln(np.sum(epsilon[k, :])) - np.sum(gammaln(epsilon[k, :])) for k in range(K)]
    H = 0.0
    trSW = np.zeros(K)
    xbarWxbar = np.zeros(K)
    mWm = np.zeros(K)
    trW0invW = np.zeros(K)
    for k in range(K):                                                                # :107-118
        Wk = W[:, :, k]
        logBk = (-(v[k] / 2) * np.log(np.linalg.det(Wk)) - (v[k] * dim / 2) * np.log(2)
                 - (dim * (dim - 1) / 4) * np.log(np.pi) - np.sum(gammaln(0.5 * (v[k] + 1 - qq))))
        H = H - logBk - 0.5 * (v[k] - dim - 1) * lLT[k] + 0.5 * v[k] * dim
        trSW[k] = np.trace(t1_S[:, :, k] @ Wk)
        diff = xbar[k, :] - m[:, k]
        xbarWxbar[k] = diff @ Wk @ diff
        diff = m[:, k] - m0[:, 0]
        mWm[k] = diff @ Wk @ diff
        trW0invW[k] = np.trace(W0inv @ Wk)
    Lt1 = 0.5 * np.sum(Nk * (lLT - dim / beta - v * trSW - v * xbarWxbar - dim * np.log(2 * np.pi)))
    gamma1 = gam[:, :, 0]                                                             # :127
    Lt2a = 0.0
    for n in range(N):                                                                # :141-143
        for k in range(K):
            Lt2a += gamma1[k, n] * lPi[k]
    Lt2b = np.sum(M.ravel() * lA.ravel())                                             # :160
    Lt2 = Lt2a + Lt2b
    Lt3 = logCalpha0 + (alpha0 - 1) * np.sum(lPi)                                     # :174
    Lt4 = sum(logCepsilon0[k] + (epsilon0 - 1) * np.sum(lA[k, :]) for k in range(K))  # :184-187
    Lt51 = 0.5 * np.sum(dim * np.log(beta0 / (2 * np.pi)) + lLT - dim * beta0 / beta - beta0 * v * mWm)
    Lt52 = K * logB0 + 0.5 * (v0 - dim - 1) * np.sum(lLT) - 0.5 * np.sum(v * trW0invW)
    Lt5 = Lt51 + Lt52
    Lt63 = np.sum(gam * logrho)                                                       # :214
    Lt64 = np.sum(phi)                                                                # :217
    Lt6 = Lt2a + Lt2b + Lt63 - Lt64
    Lt71 = np.sum((alpha - 1) * lPi) + logCalpha                                      # :225
    Lt72 = sum(np.sum((epsilon[k, :] - 1) * lA[k, :]) + logCepsilon[k] for k in range(K))
    Lt7 = Lt71 + Lt72
    Lt8 = 0.5 * np.sum(lLT + dim * np.log(beta / (2 * np.pi))) - 0.5 * dim * K - H   # :253
    return Lt1 + Lt2 + Lt3 + Lt4 + Lt5 - Lt6 - Lt7 - Lt8


def em(data, K, opt, gmm, fb_fn="c"):
    """vbhmm_em.m:112-491.  fb_fn: 'c' (C restatement of vbhmm_fb_mex.c) or 'twin'."""
    dim = len(np.ravel(opt["mu0"]))
    data = [np.asarray(a, float).reshape(-1, dim) for a in data]
    N = len(data)
    datalen = [a.shape[0] for a in data]
    maxT = max(datalen)
    mix = init_from_gmm(data, K, opt, gmm)
    alpha0, epsilon0, beta0, v0 = opt["alpha0"], opt["epsilon0"], opt["beta0"], opt["v0"]
    m0, W0inv, W0mode = mix["m0"], mix["W0inv"], mix["W0mode"]
    alpha, epsilon, beta, v, m, W = (np.array(mix[k], copy=True)
                                     for k in ("alpha", "epsilon", "beta", "v", "m", "W"))
    C = np.zeros((dim, dim, K))
    L = -np.finfo(float).max
    lastL = -np.finfo(float).max
    LLs = []
    unstable = False
    for it in range(1, opt["maxIter"] + 1):
        varpar = dict(v=v, W=W.transpose(2, 0, 1), epsilon=epsilon, alpha=alpha, m=m.T, beta=beta)
        pre = vo.vbhmm_prelude(varpar)
        if fb_fn == "c":
            f = vo.c_vbhmm_fb(data, varpar, pre)
            gam = f["gamma"].transpose(2, 1, 0)                  # [maxT][N][K] -> [K][N][maxT]
            logrho = f["logrho"].transpose(2, 1, 0)
            xi_sum = f["xi_sum"].transpose(1, 2, 0)              # [N][K][K] -> [K][K][N]
        else:
            f = vo.twin_vbhmm_fb(data, varpar, pre)
            gam = f["gamma"].transpose(2, 1, 0)
            logrho = f["logrho"].transpose(2, 1, 0)
            xi_sum = f["xi_sum"].transpose(1, 2, 0)
        fb = dict(logrho=logrho, gamma=gam, phi_norm=f["phi_norm"],
                  logLambdaTilde=pre["logLambdaTilde"], logPiTilde=pre["logPiTilde"],
                  logATilde=pre["logATilde"])
        t_Nk1 = gam.sum(axis=1)                                   # [K x maxT] (:158)
        Nk1 = t_Nk1[:, 0] + 1e-50                                 # :162-163
        Nk = t_Nk1.sum(axis=1) + 1e-50                            # :171-172
        M = xi_sum.sum(axis=2)                                    # :178
        xbar = np.zeros((K, dim))                                 # :216-219
        for k in range(K):
            acc = np.zeros(dim)
            for n in range(N):
                for t in range(datalen[n]):
                    acc += data[n][t] * gam[k, n, t]
            xbar[k] = acc / Nk[k]
        t1_S = np.zeros((dim, dim, K))                            # :241-246
        for k in range(K):
            acc = np.zeros((dim, dim))
            for n in range(N):
                for t in range(datalen[n]):
                    d1 = data[n][t] - xbar[k]
                    acc += gam[k, n, t] * np.outer(d1, d1)
            t1_S[:, :, k] = acc / Nk[k]
        if it > 1:
            lastL = L
        L = lower_bound(dim, K, alpha0, epsilon0, m0, beta0, v0, W0inv, W0mode, t1_S, xbar, Nk, M,
                        v, W, epsilon, alpha, m, beta, fb)
        do_break = False
        if it > 1 and abs((L - lastL) / lastL) <= opt["minDiff"]:
            do_break = True
        if it == opt["maxIter"]:
            do_break = True
        if np.isnan(L):
            do_break, unstable, L = True, True, -np.inf
        LLs.append(L)
        if do_break and unstable:
            break
        alpha = alpha0 + Nk1                                      # :356
        epsilon = epsilon0 + M                                    # :357
        beta = beta0 + Nk                                         # :368
        v = v0 + Nk + 1                                           # :369
        for k in range(K):                                        # :370-372
            m[:, k] = (beta0 * m0[:, 0] + Nk[k] * xbar[k, :]) / beta[k]
        for k in range(K):                                        # :375-383
            mult1 = beta0 * Nk[k] / (beta0 + Nk[k])
            diff3 = (xbar[k, :] - m0[:, 0]).reshape(dim, 1)
            Wk = np.linalg.inv(W0inv + Nk[k] * t1_S[:, :, k] + mult1 * (diff3 @ diff3.T))
            W[:, :, k] = (Wk + Wk.T) / 2
        for k in range(K):                                        # :394-408
            if v[k] > dim + 1:
                Ck = np.linalg.inv(W[:, :, k]) / (v[k] - dim - 1)
            else:
                Ck = np.linalg.inv(W[:, :, k]) / v[k]
            C[:, :, k] = (Ck + Ck.T) / 2
        if do_break:
            break
    prior = alpha / np.sum(alpha)
    trans = epsilon.copy()
    for k in range(K):
        sc = np.sum(trans[k, :])
        trans[k, :] = trans[k, :] / (sc if sc != 0 else 1.0)
    return dict(prior=prior, trans=trans, mean=m.T.copy(), cov=C.transpose(2, 0, 1).copy(),
                LL=L, LLs=np.array(LLs), iters=it, N=Nk, N1=Nk1, M=M,
                varpar=dict(alpha=alpha, epsilon=epsilon, beta=beta, v=v, m=m.T.copy(),
                            W=W.transpose(2, 0, 1).copy()))

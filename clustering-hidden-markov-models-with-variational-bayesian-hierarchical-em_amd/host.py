"""Host-side math around the device E-step (vectorised over clusters/states).

Everything here is O(K*S*d^3) per EM iteration -- tiny next to the E-step --
and mirrors the MATLAB code that surrounds the MEX call:

* :func:`cluster_constants` -- psi prelude, vbhem_h3m_c_step_fc.m:118-165, 180-191
* :func:`log_omega_tilde`   -- vbhem_h3m_c_step_fc.m:271-273
* :func:`unpack_stats` / :func:`finish_statistics` -- vbhem_compute_Statistics.m:57-82
* :func:`mstep`             -- vbhem_mstep_component.m:42-70 and step_fc.m:396
* :func:`lower_bound`       -- vbhemh3m_lb.m:64-186
* :func:`convert_to_point`  -- convert_h3mrtoh3mb.m:9-79
"""
from __future__ import annotations

import numpy as np
from scipy.special import digamma, gammaln

from .h3m import COV_DIAG, COV_FULL, Posterior


def cluster_constants(post: Posterior, covmode: int) -> dict:
    """Per-cluster E-step constants for this iteration.

    logLambdaTilde = sum_q psi((v+1-q)/2) + d log 2 + log|W|  (:136,146)
    c  = -logLambdaTilde + d/lambda                              (:154)
    logA = psi(eps) - psi(sum_sigma eps);  logPi = psi(eta) - psi(sum eta)  (:156-161)
    P  = v * W                                                   (:189)
    Diag mode uses sum(log W): MATLAB's sum(log(diag(W))) on a 1xd row only
    runs for d == 1, where both agree."""
    K, S, d = post.m.shape
    q = np.arange(1, d + 1)
    t1 = digamma(0.5 * (post.v[..., None] + 1.0) - 0.5 * q).sum(-1)
    if covmode == COV_FULL:
        logdet = np.log(np.linalg.det(post.W))
    else:
        logdet = np.log(post.W).sum(-1)
    lLT = t1 + d * np.log(2.0) + logdet
    eps = post.epsilon
    logA = digamma(eps) - digamma(eps.sum(-1, keepdims=True))
    logPi = digamma(post.eta) - digamma(post.eta.sum(-1, keepdims=True))
    P = post.v[..., None, None] * post.W if covmode == COV_FULL else post.v[..., None] * post.W
    return dict(logLambdaTilde=lLT, c=-lLT + d / post.lam, logA=logA, logPi=logPi,
                m=np.ascontiguousarray(post.m), P=np.ascontiguousarray(P))


def vhem_cluster_constants(red: dict, covmode: int) -> dict:
    """E-step constants of the VHEM sibling (hem_hmm_bwd_fwd_mex.c) from point-estimate
    reduced HMMs red = {A [K][S][S], prior [K][S], centres [K][S][d], covars [K][S][d,d]|[K][S][d]}:
    logA = log(A) (:906-922), logPi = log(prior) (:1004-1019), m = centres, and
    full: P = inv(covars), c = log(det(covars))  (hem_h3m_c_step.m:198-205);
    diag: P = 1 ./ covars, c = sum(log(covars))  (hem_hmm_bwd_fwd_mex.c:711-733)."""
    A = np.asarray(red["A"], dtype=np.float64)
    prior = np.asarray(red["prior"], dtype=np.float64)
    cov = np.asarray(red["covars"], dtype=np.float64)
    with np.errstate(divide="ignore"):
        logA, logPi = np.log(A), np.log(prior)
    if covmode == COV_FULL:
        P = np.linalg.inv(cov)
        c = np.log(np.linalg.det(cov))
    else:
        P = 1.0 / cov
        c = np.log(cov).sum(-1)
    return dict(logA=logA, logPi=logPi, m=np.asarray(red["centres"], dtype=np.float64).copy(),
                P=P, c=c)


def log_omega_tilde(alpha: np.ndarray) -> np.ndarray:
    return digamma(alpha) - digamma(alpha.sum())


def stats_nu(d: int, covmode: int) -> int:
    return 1 + d + d * (d + 1) // 2 if covmode == COV_FULL else 1 + 2 * d


def stats_len(K: int, S: int, d: int, covmode: int) -> int:
    return K + K * S + K * S * S + 2 + K * S * stats_nu(d, covmode)


def unpack_stats(vec: np.ndarray, K: int, S: int, d: int, covmode: int) -> dict:
    """Split the packed E-step statistics (include/vbhem_estep.h) into arrays."""
    vec = np.asarray(vec, dtype=np.float64)
    o = 0
    Nj = vec[o:o + K]; o += K
    N1 = vec[o:o + K * S].reshape(K, S); o += K * S
    M = vec[o:o + K * S * S].reshape(K, S, S); o += K * S * S
    Lt1, Lt7 = vec[o], vec[o + 1]; o += 2
    NU = stats_nu(d, covmode)
    U = vec[o:o + K * S * NU].reshape(K, S, NU)
    Nr = U[..., 0]
    Y = U[..., 1:1 + d]
    if covmode == COV_FULL:
        SC = np.zeros((K, S, d, d))
        iu = np.triu_indices(d)
        SC[..., iu[0], iu[1]] = U[..., 1 + d:]
        SC[..., iu[1], iu[0]] = U[..., 1 + d:]
    else:
        SC = U[..., 1 + d:1 + 2 * d].copy()
    return dict(Nj=Nj.copy(), N1=N1.copy(), M=M.copy(), Lt1=float(Lt1), Lt7=float(Lt7),
                Nr=Nr.copy(), Y=Y.copy(), SC=SC)


def finish_statistics(st: dict, covmode: int) -> dict:
    """vbhem_compute_Statistics.m:57-82 on the gated sums (all clusters)."""
    S = st["N1"].shape[1]
    Nr = st["Nr"] + 1e-50
    y = st["Y"] / Nr[..., None]
    if covmode == COV_FULL:
        SC = st["SC"] / Nr[..., None, None] - y[..., :, None] * y[..., None, :]
    else:
        SC = st["SC"] / Nr[..., None] - y * y
    M = st["M"] if S > 1 else np.full_like(st["M"], 1e-12)
    return dict(Nj_rho1=st["N1"], Nj_rho2rho=M, Nj_rho=Nr, y_bar=y, S_plus_C=SC)


def _W0(opt: dict, d: int) -> np.ndarray:
    W0 = np.asarray(opt["W0"], dtype=float)
    return W0 * np.eye(d) if W0.size == 1 else np.diag(W0)


def mstep(syn: dict, Nj: np.ndarray, opt: dict, covmode: int, W0mode: str) -> Posterior:
    """vbhem_mstep_component.m:42-70 for every cluster, alpha = alpha0 + Nj (step_fc.m:396)."""
    d = syn["y_bar"].shape[-1]
    m0 = np.asarray(opt["m0"], dtype=float)
    lam0 = opt["lambda0"]
    W0inv = np.linalg.inv(_W0(opt, d))
    Nk = syn["Nj_rho"]
    lam = lam0 + Nk
    v = opt["v0"] + Nk + 1.0
    m = (lam0 * m0 + Nk[..., None] * syn["y_bar"]) / (lam0 + Nk)[..., None]
    mult1 = lam0 * Nk / (lam0 + Nk)
    diff = syn["y_bar"] - m0
    outer = diff[..., :, None] * diff[..., None, :]
    if covmode == COV_FULL:
        tW = np.linalg.inv(W0inv + Nk[..., None, None] * syn["S_plus_C"] + mult1[..., None, None] * outer)
        W = (tW + np.swapaxes(tW, -1, -2)) / 2
    else:
        diagSC = syn["S_plus_C"][..., :, None] * np.eye(d)
        tW = np.linalg.inv(W0inv + Nk[..., None, None] * diagSC + mult1[..., None, None] * outer)
        W = np.diagonal((tW + np.swapaxes(tW, -1, -2)) / 2, axis1=-2, axis2=-1).copy()
    eta = opt["eta0"] + syn["Nj_rho1"]
    epsilon = opt["epsilon0"] + syn["Nj_rho2rho"]
    return Posterior(alpha=opt["alpha0"] + Nj, eta=eta, epsilon=epsilon, lam=lam, v=v, m=m, W=W,
                     W0mode=W0mode)


def lower_bound(Lt1: float, Lt7: float, Nj: np.ndarray, logOmega: np.ndarray, post: Posterior,
                consts: dict, opt: dict, covmode: int) -> float:
    """vbhemh3m_lb.m:64-186 (value only).  Lt1 = sum Z.*L_elbo and
    Lt7 = sum hat_Z.*log(hat_Z) come reduced from the device."""
    K, S = post.K, opt["S"]
    d = len(opt["m0"])
    a0, e0, ep0, l0, v0 = opt["alpha0"], opt["eta0"], opt["epsilon0"], opt["lambda0"], opt["v0"]
    m0 = np.asarray(opt["m0"], dtype=float)
    W0inv = np.linalg.inv(_W0(opt, d))
    if np.size(opt["W0"]) == 1:
        logdetW0inv = d * np.log(W0inv[0, 0])
    else:
        logdetW0inv = np.log(np.diag(W0inv)).sum()
    q = np.arange(1, d + 1)
    logCalpha0 = gammaln(K * a0) - K * gammaln(a0)
    logCeta0 = gammaln(S * e0) - S * gammaln(e0)
    logCepsilon0 = gammaln(S * ep0) - S * gammaln(ep0)
    logB0 = (v0 / 2) * logdetW0inv - (v0 * d / 2) * np.log(2) - (d * (d - 1) / 4) * np.log(np.pi) \
        - gammaln(0.5 * (v0 + 1 - q)).sum()
    const2 = d * np.log(l0 / (2 * np.pi))
    alpha = post.alpha
    logCalpha = gammaln(alpha.sum()) - gammaln(alpha).sum()
    lLT = consts["logLambdaTilde"]
    Lt2 = Nj @ logOmega
    Lt3 = K * logCeta0 + (e0 - 1) * consts["logPi"].sum()
    Lt4 = K * S * logCepsilon0 + (ep0 - 1) * consts["logA"].sum()
    Lt6 = logCalpha0 + (a0 - 1) * logOmega.sum()
    Lt8 = logCalpha + (alpha - 1) @ logOmega
    Wf = post.W if covmode == COV_FULL else post.W[..., :, None] * np.eye(d)
    v, lam = post.v, post.lam
    logBk = -(v / 2) * np.log(np.linalg.det(Wf)) - (v * d / 2) * np.log(2) \
        - (d * (d - 1) / 4) * np.log(np.pi) - gammaln(0.5 * (v[..., None] + 1 - q)).sum(-1)
    H = (-logBk - 0.5 * (v - d - 1) * lLT + 0.5 * v * d).sum(-1)
    diff = post.m - m0
    mWm = np.einsum("ksa,ksab,ksb->ks", diff, Wf, diff)
    trW = np.einsum("ab,ksba->ks", W0inv, Wf)
    Lt51 = 0.5 * (const2 + lLT - d * l0 / lam - l0 * v * mWm).sum(-1)
    Lt52 = S * logB0 + 0.5 * (v0 - d - 1) * lLT.sum(-1) - 0.5 * (v * trW).sum(-1)
    Lt5 = (Lt51 + Lt52).sum()
    eta, eps = post.eta, post.epsilon
    logCeta = gammaln(eta.sum(-1)) - gammaln(eta).sum(-1)
    logCeps = gammaln(eps.sum(-1)) - gammaln(eps).sum(-1)
    Lt9 = (logCeta + ((eta - 1) * consts["logPi"]).sum(-1)).sum() \
        + (logCeps + ((eps - 1) * consts["logA"]).sum(-1)).sum()
    Lt10 = (0.5 * (lLT + d * np.log(lam / (2 * np.pi))).sum(-1) - 0.5 * d * S - H).sum()
    return float(Lt1 + Lt2 + Lt3 + Lt4 + Lt5 + Lt6 - Lt7 - Lt8 - Lt9 - Lt10)


def lower_bound_derivs(logOmega: np.ndarray, post: Posterior, consts: dict, opt: dict,
                       covmode: int, clipped: dict = None) -> dict:
    """vbhemh3m_lb.m:202-345: derivatives of the lower bound with respect to the
    hyperparameters (posterior held fixed), zeroed where a clipped hyperparameter
    would move further out of range (:326-343), then taken with respect to the
    transformed hyperparameters the optimiser works in (:345-356).

    W0 diag ('diag' W0mode): the reference's branch refers to undefined K*S and
    covmode and would error; here it uses Kr*Sr and the
    run's covariance mode, the evident intent."""
    K, S = post.K, opt["S"]
    d = len(opt["m0"])
    a0, e0, ep0, l0, v0 = opt["alpha0"], opt["eta0"], opt["epsilon0"], opt["lambda0"], opt["v0"]
    m0 = np.asarray(opt["m0"], dtype=float)
    W0 = np.asarray(opt["W0"], dtype=float)
    W0inv = np.linalg.inv(_W0(opt, d))
    iid = W0.size == 1
    logdetW0inv = d * np.log(W0inv[0, 0]) if iid else np.log(np.diag(W0inv)).sum()
    q = np.arange(1, d + 1)
    lLT = consts["logLambdaTilde"]
    v, lam = post.v, post.lam
    Wf = post.W if covmode == COV_FULL else post.W[..., :, None] * np.eye(d)
    diff = post.m - m0
    mWm = np.einsum("ksa,ksab,ksb->ks", diff, Wf, diff)
    dLt = {}
    dLt["alpha0"] = np.atleast_1d(K * digamma(K * a0) - K * digamma(a0) + logOmega.sum())
    dLt["eta0"] = np.atleast_1d(K * (S * digamma(S * e0) - S * digamma(e0)) + consts["logPi"].sum())
    dLt["epsilon0"] = np.atleast_1d(K * S * (S * digamma(S * ep0) - S * digamma(ep0))
                                    + consts["logA"].sum())
    d_logB0_v0 = 0.5 * logdetW0inv - (d / 2) * np.log(2) - 0.5 * digamma(0.5 * (v0 + 1 - q)).sum()
    dLt["v0"] = np.atleast_1d(K * S * d_logB0_v0 + 0.5 * lLT.sum())
    dLt["lambda0"] = np.atleast_1d((0.5 * (d / l0 - d / lam - v * mWm)).sum())
    if iid:
        myW0inv = W0inv[0, 0]
        myW0 = 1.0 / myW0inv
        trW = np.trace(Wf, axis1=-2, axis2=-1)
        d_tr = -v * myW0inv ** 2 * trW
        dLt["W0"] = np.atleast_1d(K * S * (-0.5 * v0 * d * myW0inv) - 0.5 * d_tr.sum())
    else:
        myW0inv = np.diag(W0inv)
        myW0 = 1.0 / myW0inv
        dgW = np.diagonal(Wf, axis1=-2, axis2=-1)                        # [K][S][d]
        d_tr = -v[..., None] * myW0inv ** 2 * dgW
        dLt["W0"] = K * S * (-0.5 * v0 * myW0inv) - 0.5 * d_tr.sum(axis=(0, 1))
    dLt["m0"] = (l0 * v[..., None] * np.einsum("ksab,ksb->ksa", Wf, post.m - m0)).sum(axis=(0, 1))
    return transform_derivs(dLt, opt, clipped)


def transform_derivs(dLt: dict, opt: dict, clipped: dict = None) -> dict:
    """vbhemh3m_lb.m:326-356 on raw derivatives (alpha0, eta0, epsilon0, v0,
    lambda0, W0, m0 -- host.lower_bound_derivs or the C++ loop's
    vbhem_em_lower_bound_derivs): zeroed where a clipped hyperparameter would
    move further out of range, then taken with respect to the transformed
    hyperparameters the optimiser works in."""
    d = len(opt["m0"])
    a0, e0, ep0, l0, v0 = opt["alpha0"], opt["eta0"], opt["epsilon0"], opt["lambda0"], opt["v0"]
    W0inv = np.linalg.inv(_W0(opt, d))
    myW0 = 1.0 / W0inv[0, 0] if np.asarray(opt["W0"]).size == 1 else 1.0 / np.diag(W0inv)
    dLt = {k: np.array(v, dtype=float) for k, v in dLt.items()}
    if clipped is not None:
        for name, fl in clipped.items():
            g = dLt[name]
            g[(fl == 1) & (g > 0)] = 0.0
            g[(fl == -1) & (g < 0)] = 0.0
    return dict(d_logalpha0=dLt["alpha0"] * a0, d_logeta0=dLt["eta0"] * e0,
                d_logepsilon0=dLt["epsilon0"] * ep0, d_logv0D1=dLt["v0"] * (v0 - d + 1),
                d_sqrtv0D1=dLt["v0"] * 2 * np.sqrt(v0 - d + 1),
                d_loglambda0=dLt["lambda0"] * l0, d_sqrtlambda0=dLt["lambda0"] * 2 * np.sqrt(l0),
                d_sqrtW0inv=dLt["W0"] * (myW0 ** 1.5) * (-2.0), d_logW0=dLt["W0"] * myW0,
                d_m0=dLt["m0"], raw=dLt)


def convert_to_point(post: Posterior, covmode: int) -> dict:
    """convert_h3mrtoh3mb.m:9-79: prior, A, centres, covars, omega point estimates."""
    K, S, d = post.m.shape
    prior = post.eta / post.eta.sum(-1, keepdims=True)
    sc = post.epsilon.sum(-1, keepdims=True)
    A = post.epsilon / np.where(sc == 0, 1.0, sc)
    den = np.where(post.v > d + 1, post.v - d - 1, post.v)
    if covmode == COV_FULL:
        tC = np.linalg.inv(post.W) / den[..., None, None]
        cov = (tC + np.swapaxes(tC, -1, -2)) / 2
    else:
        tC = (1.0 / post.W) / den[..., None]
        cov = (tC + tC) / 2
    return dict(prior=prior, A=A, centres=post.m.copy(), covars=cov,
                omega=post.alpha / post.alpha.sum())

"""oracle/vbhem_oracle.py -- TEST INFRASTRUCTURE ONLY.

Checker for the VBHEM-H3M E-step hot path and the MATLAB host math around it.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module; the product package never does.

PARITY UNPINNED.  The reference repository ships no tests, fixtures or golden
vectors; MATLAB/Octave are absent, and the reference MEX
(src/vbhem/vbhem_hmm_bwd_fwd_mex.c) needs mex.h/libmx, which the image lacks,
so it is not built here ("Oracle").  Two independent restatements
are kept instead and cross-checked against each other and against closed-form
known answers:

* ``liboracle.so`` (oracle/vbhem_oracle.c): loop-for-loop restatement of the
  MEX (USEPTRS branch) including its summation order;
* :func:`twin_pair_estep` below: numpy restatement of the MATLAB twin
  src/vbhem/vbhem_hmm_bwd_fwd_fast.m (vectorised per pair).

The host-side math (psi prelude, responsibilities, statistics, M-step, ELBO,
conversion, output) is restated loop-style from the MATLAB sources cited in
each docstring.  MATLAB ``psi``/``gammaln`` are replaced by
``scipy.special.digamma``/``gammaln`` (not pinned by any reference test).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
from scipy.special import digamma as psi
from scipy.special import gammaln

HERE = os.path.dirname(os.path.abspath(__file__))
COV_DIAG, COV_FULL = 0, 1

# ----------------------------------------------------------------------------
# C oracle (restated MEX) via ctypes
# ----------------------------------------------------------------------------
_LIB = None


def liboracle_path() -> str:
    return os.path.join(HERE, "liboracle.so")


def load_c_oracle(build_if_missing: bool = True):
    """Load oracle/liboracle.so (built by oracle/Makefile)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = liboracle_path()
    if not os.path.exists(path) and build_if_missing:
        subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(path)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int)
    lib.oracle_estep_pairs.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip,
        dp, dp, dp, dp, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp,
        ctypes.c_int, dp, dp, dp, dp, dp, dp, dp, ctypes.c_int]
    lib.oracle_estep_pairs.restype = ctypes.c_int
    lib.oracle_vhem_estep_pairs.argtypes = [
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip,
        dp, dp, dp, dp, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, dp,
        ctypes.c_int, ctypes.c_double, dp, dp, dp, dp, dp, dp, dp, ctypes.c_int]
    lib.oracle_vhem_estep_pairs.restype = ctypes.c_int
    lib.oracle_responsibilities.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp]
    lib.oracle_responsibilities.restype = None
    lib.oracle_statistics.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, dp, dp, dp, dp, dp, dp,
                                      dp, dp, dp, dp, dp, dp]
    lib.oracle_statistics.restype = None
    lib.oracle_vbhmm_fb.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, dp,
                                    dp, dp, dp, dp, dp, ctypes.c_double, dp, dp, dp, dp, dp, dp]
    lib.oracle_vbhmm_fb.restype = ctypes.c_int
    _LIB = lib
    return lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _c64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def c_estep_pairs(base: dict, consts: dict, T: int, nthreads: int = 1, want_tnu: bool = False):
    """MEX-equivalent per-pair outputs, layout [N][K][...] (see vbhem_oracle.c)."""
    lib = load_c_oracle()
    N, SB = base["prior"].shape
    d = base["centres"].shape[2]
    covmode = base["covmode"]
    K, S = consts["logPi"].shape
    dM = d * d if covmode == COV_FULL else d
    ns = np.ascontiguousarray(base["nstates"], dtype=np.int32)
    arrs = [_c64(base[k]) for k in ("prior", "A", "centres", "covars")]
    carrs = [_c64(consts[k]) for k in ("logA", "logPi", "m", "P", "c")]
    out = {
        "LL_elbo": np.zeros((N, K)),
        "sum_nu_1": np.zeros((N, K, S)),
        "sum_xi": np.zeros((N, K, S, S)),
        "emit_pr": np.zeros((N, K, S)),
        "emit_mu": np.zeros((N, K, S, d)),
        "emit_Mu": np.zeros((N, K, S, d, d) if covmode == COV_FULL else (N, K, S, d)),
    }
    tnu = np.zeros((N, K, S, SB)) if want_tnu else None
    rc = lib.oracle_estep_pairs(
        N, SB, d, covmode, ns.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
        *[_dp(a) for a in arrs], K, S, *[_dp(a) for a in carrs], int(T),
        _dp(out["LL_elbo"]), _dp(out["sum_nu_1"]), _dp(out["sum_xi"]),
        _dp(out["emit_pr"]), _dp(out["emit_mu"]), _dp(out["emit_Mu"]),
        _dp(tnu) if tnu is not None else ctypes.POINTER(ctypes.c_double)(),
        int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_estep_pairs failed rc={rc}")
    if want_tnu:
        out["sum_t_nu"] = tnu
    del dM
    return out


def c_vhem_estep_pairs(base: dict, red: dict, T: int, smooth: float = 1.0, nthreads: int = 1,
                       want_tnu: bool = False):
    """VHEM sibling (hem_hmm_bwd_fwd_mex.c) on point-estimate reduced HMMs
    red = {A [K][S][S], prior [K][S], centres [K][S][d], covars [K][S][d,d]|[K][S][d]}
    (+ logdetCov [K][S], invCov [K][S][d][d] computed here for full covariances, as
    hem_h3m_c_step.m:198-205 does).  Outputs [N][K][...]."""
    lib = load_c_oracle()
    N, SB = base["prior"].shape
    d = base["centres"].shape[2]
    covmode = base["covmode"]
    K, S = red["prior"].shape
    ns = np.ascontiguousarray(base["nstates"], dtype=np.int32)
    arrs = [_c64(base[k]) for k in ("prior", "A", "centres", "covars")]
    rarrs = [_c64(red[k]) for k in ("A", "prior", "centres", "covars")]
    if covmode == COV_FULL:
        cov = np.asarray(red["covars"], dtype=np.float64)
        logdet = _c64(np.log(np.linalg.det(cov)))
        inv = _c64(np.linalg.inv(cov))
    else:
        logdet = inv = _c64(np.zeros(1))
    out = {
        "LL_elbo": np.zeros((N, K)),
        "sum_nu_1": np.zeros((N, K, S)),
        "sum_xi": np.zeros((N, K, S, S)),
        "emit_pr": np.zeros((N, K, S)),
        "emit_mu": np.zeros((N, K, S, d)),
        "emit_Mu": np.zeros((N, K, S, d, d) if covmode == COV_FULL else (N, K, S, d)),
    }
    tnu = np.zeros((N, K, S, SB)) if want_tnu else None
    rc = lib.oracle_vhem_estep_pairs(
        N, SB, d, covmode, ns.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
        *[_dp(a) for a in arrs], K, S, *[_dp(a) for a in rarrs], _dp(logdet), _dp(inv), int(T),
        ctypes.c_double(float(smooth)),
        _dp(out["LL_elbo"]), _dp(out["sum_nu_1"]), _dp(out["sum_xi"]),
        _dp(out["emit_pr"]), _dp(out["emit_mu"]), _dp(out["emit_Mu"]),
        _dp(tnu) if tnu is not None else ctypes.POINTER(ctypes.c_double)(),
        int(nthreads))
    if rc != 0:
        raise ValueError(f"oracle_vhem_estep_pairs failed rc={rc}")
    if want_tnu:
        out["sum_t_nu"] = tnu
    return out


def c_responsibilities(LL_elbo, tildeN, logOmega):
    lib = load_c_oracle()
    N, K = LL_elbo.shape
    L = _c64(LL_elbo)
    tn = _c64(tildeN)
    lo = _c64(logOmega)
    hz = np.zeros((N, K))
    Z = np.zeros((N, K))
    lib.oracle_responsibilities(N, K, _dp(L), _dp(tn), _dp(lo), _dp(hz), _dp(Z))
    return hz, Z


def c_statistics(Z, pairs: dict, covmode: int):
    lib = load_c_oracle()
    N, K, S = pairs["sum_nu_1"].shape
    d = pairs["emit_mu"].shape[3]
    dM = d * d if covmode == COV_FULL else d
    out = {"Nj": np.zeros(K), "N1": np.zeros((K, S)), "M": np.zeros((K, S, S)),
           "Nr": np.zeros((K, S)), "Y": np.zeros((K, S, d)),
           "SC": np.zeros((K, S, d, d) if covmode == COV_FULL else (K, S, d))}
    ins = [_c64(Z)] + [_c64(pairs[k]) for k in ("sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")]
    lib.oracle_statistics(N, K, S, d, covmode, *[_dp(a) for a in ins],
                          *[_dp(out[k]) for k in ("Nj", "N1", "M", "Nr", "Y", "SC")])
    del dM
    return out


def base_subset(base: dict, idx) -> dict:
    """The base HMMs ``idx`` (an index array or a slice) of a packed base dict."""
    N = base["prior"].shape[0]
    return {k: (np.ascontiguousarray(v[idx]) if isinstance(v, np.ndarray) and v.ndim and
                v.shape[0] == N else v) for k, v in base.items()}


def c_fused(base: dict, consts: dict, T: int, tildeN, logOmega, nthreads: int = 1,
            chunk: int = 4096):
    """The fused E-step of one EM iteration on the CPU: per-pair recursions
    (oracle_estep_pairs), responsibilities (vbhem_h3m_c_step_fc.m:270-283) and
    the gated statistic sums (vbhem_compute_Statistics.m:33-55), with the ELBO
    partials Lt1 = sum Z .* L_elbo and Lt7 = sum hat_Z .* log(hat_Z)
    (vbhemh3m_lb.m:90, 107), over chunks of ``chunk`` bases so the per-pair
    outputs never exist for all N at once (C4 / C5 at full size).  The sums are
    additive over bases, so chunking changes only their summation order.
    Returns dict(LL_elbo [N][K], hat_Z [N][K], Nj, N1, M, Nr, Y, SC, Lt1, Lt7)."""
    N = base["prior"].shape[0]
    K = consts["logPi"].shape[0]
    tN = np.asarray(tildeN, dtype=np.float64)
    LL = np.zeros((N, K))
    hz = np.zeros((N, K))
    acc = None
    Lt1 = Lt7 = 0.0
    for i0 in range(0, N, chunk):
        i1 = min(N, i0 + chunk)
        b = base_subset(base, slice(i0, i1))
        pr = c_estep_pairs(b, consts, T, nthreads=nthreads)
        h, Z = c_responsibilities(pr["LL_elbo"], tN[i0:i1], logOmega)
        st = c_statistics(Z, pr, base["covmode"])
        LL[i0:i1] = pr["LL_elbo"]
        hz[i0:i1] = h
        Lt1 += float((Z * pr["LL_elbo"]).sum())
        Lt7 += float((h * np.log(h)).sum())
        acc = st if acc is None else {k: acc[k] + st[k] for k in acc}
        del pr
    out = dict(acc or {})
    out.update(LL_elbo=LL, hat_Z=hz, Lt1=Lt1, Lt7=Lt7)
    return out


# ----------------------------------------------------------------------------
# numpy restatement of the MATLAB twin (vbhem_hmm_bwd_fwd_fast.m)
# ----------------------------------------------------------------------------
def _logtrick_cols(lA):
    """logtrick.m:15-18 -- column-wise log-sum-exp with max shift."""
    mv = lA.max(axis=0)
    return mv + np.log(np.exp(lA - mv).sum(axis=0))


def twin_pair_estep(prior, A, centres, covars, covmode, T, m, W, v, lam,
                    logLambdaTilde, logATilde, logPiTilde):
    """One (base, cluster) pair as in vbhem_hmm_bwd_fwd_fast.m:1-398.

    prior [Sb], A [Sb,Sb], centres [Sb,d], covars [Sb,d,d] | [Sb,d];
    m [S,d], W [S,d,d] (full) | [S,d] (diag), v/lam/logLambdaTilde [S],
    logATilde [S,S], logPiTilde [S].  Returns the six MEX outputs plus sum_t_nu.
    """
    Sb = A.shape[0]
    S = m.shape[0]
    d = centres.shape[1]
    # emission expectation E3logN [Sb,S]  (fast.m:66-140)
    E = np.zeros((Sb, S))
    for rho in range(S):
        if covmode == COV_DIAG:
            wd = W[rho]
            ell = (covars * wd[None, :]).sum(1)
            ell = ell + (((centres - m[rho][None, :]) ** 2) * wd[None, :]).sum(1)
            ell = v[rho] * ell - logLambdaTilde[rho] + d / lam[rho] + d * np.log(2 * np.pi)
            E[:, rho] = -0.5 * ell
        else:
            Wr = W[rho]
            trcov = np.einsum("ab,kab->k", Wr, covars)
            diff = centres - m[rho][None, :]
            dterm = np.einsum("ka,ab,kb->k", diff, Wr, diff)
            E[:, rho] = -0.5 * (d * np.log(2 * np.pi) - logLambdaTilde[rho] + d / lam[rho]
                                + v[rho] * (trcov + dterm))
    return _twin_recursions(prior, A, centres, covars, covmode, T, E, logATilde, logPiTilde)


def twin_vhem_pair_estep(prior, A, centres, covars, covmode, T, smooth, Ar, priorr, centresr,
                         covarsr):
    """One pair of the VHEM sibling as in hem_hmm_bwd_fwd.m:1-200 (+ g3m_stats.m for
    one Gaussian per state): E[beta,rho] = E_b[log N(y | mu_r, Sigma_r)] / smooth
    (hem_hmm_bwd_fwd.m:76), then the recursions with log(Ar) (:104) and log(prior_r)."""
    Sb = A.shape[0]
    S = Ar.shape[0]
    d = centres.shape[1]
    E = np.zeros((Sb, S))
    for rho in range(S):
        diff = centres - centresr[rho][None, :]
        if covmode == COV_DIAG:
            sr = covarsr[rho]
            ell = (d * np.log(2 * np.pi) + np.log(sr).sum() + (covars / sr[None, :]).sum(1)
                   + ((diff ** 2) / sr[None, :]).sum(1))
        else:
            inv = np.linalg.inv(covarsr[rho])
            ell = (d * np.log(2 * np.pi) + np.log(np.linalg.det(covarsr[rho]))
                   + np.einsum("ab,kab->k", inv, covars) + np.einsum("ka,ab,kb->k", diff, inv, diff))
        E[:, rho] = -0.5 * ell
    E = E / smooth
    with np.errstate(divide="ignore"):
        lA, lP = np.log(Ar), np.log(priorr)
    return _twin_recursions(prior, A, centres, covars, covmode, T, E, lA, lP)


def _twin_recursions(prior, A, centres, covars, covmode, T, E, logATilde, logPiTilde):
    """K2-K5 of the twin (fast.m:170-380) given E [Sb,S], logA [S,S], logPi [S]."""
    Sb = A.shape[0]
    S = E.shape[1]
    # backward recursion (fast.m:170-227)
    Theta = np.zeros((S, S, Sb, T))
    LL_old = np.zeros((Sb, S))
    for t in range(T - 1, 0, -1):
        # logtheta_all(sigma, beta, rho) = logATilde(rho,sigma) + E(beta,sigma) + L(beta,sigma)
        lt = logATilde.T[:, None, :] + (E.T + LL_old.T)[:, :, None]
        mv = lt.max(axis=0)
        ls = mv + np.log(np.exp(lt - mv[None]).sum(axis=0))      # [Sb, S(rho)]
        LL_new = A @ ls                                          # [Sb(gamma), S(rho)]
        th = np.exp(lt - ls[None])                               # [sigma, beta, rho]
        Theta[:, :, :, t] = np.transpose(th, (2, 0, 1))          # [rho, sigma, beta]
        LL_old = LL_new
    # termination (fast.m:231-239)
    lt = logPiTilde[:, None] + E.T + LL_old.T
    ls = _logtrick_cols(lt)
    LL_elbo = float(prior @ ls)
    Theta_1 = np.exp(lt - ls[None, :])
    # forward recursion (fast.m:258-327)
    nu = prior[None, :] * Theta_1
    sum_nu_1 = nu.sum(1)
    sum_t_nu = nu.copy()
    sum_xi = np.zeros((S, S))
    for t in range(1, T):
        foo = nu @ A
        xi = foo[:, None, :] * Theta[:, :, :, t]
        sum_xi += xi.sum(2)
        nu = xi.sum(0)
        sum_t_nu += nu
    # emission statistics (fast.m:336-380)
    emit_pr = sum_t_nu.sum(1)
    emit_mu = sum_t_nu @ centres
    if covmode == COV_DIAG:
        emit_Mu = sum_t_nu @ (centres ** 2 + covars)
    else:
        Mu = centres[:, :, None] * centres[:, None, :] + covars
        emit_Mu = np.einsum("sb,bpq->spq", sum_t_nu, Mu)
    return dict(LL_elbo=LL_elbo, sum_nu_1=sum_nu_1, sum_xi=sum_xi, emit_pr=emit_pr,
                emit_mu=emit_mu, emit_Mu=emit_Mu, sum_t_nu=sum_t_nu)


def twin_estep_pairs(base: dict, post: dict, consts: dict, T: int):
    """All pairs through :func:`twin_pair_estep`; outputs [N][K][...]."""
    N = base["prior"].shape[0]
    K, S = consts["logPi"].shape
    covmode = base["covmode"]
    res = None
    for i in range(N):
        Sb = int(base["nstates"][i])
        for j in range(K):
            o = twin_pair_estep(base["prior"][i, :Sb], base["A"][i, :Sb, :Sb],
                                base["centres"][i, :Sb], base["covars"][i, :Sb], covmode, T,
                                post["m"][j], post["W"][j], post["v"][j], post["lam"][j],
                                consts["logLambdaTilde"][j], consts["logA"][j],
                                consts["logPi"][j])
            if res is None:
                res = {k: np.zeros((N, K) + np.shape(v)) for k, v in o.items() if k != "sum_t_nu"}
            for k, v in o.items():
                if k != "sum_t_nu":
                    res[k][i, j] = v
    return res


# ----------------------------------------------------------------------------
# host math restatements (MATLAB side of the E-step call)
# ----------------------------------------------------------------------------
def hmms_to_h3m_hem(hmms, covmode: int, use_post: bool = True):
    """hmms_to_h3m_hem.m:1-144 -> packed base set (zero-padded to max states)."""
    K = len(hmms)
    nin = None
    for h in hmms:
        if h is not None:
            nin = len(h["pdf"][0]["mean"])
            break
    SB = max(len(h["prior"]) if h is not None else 1 for h in hmms)
    d = nin
    prior = np.zeros((K, SB))
    A = np.zeros((K, SB, SB))
    cen = np.zeros((K, SB, d))
    cov = np.zeros((K, SB, d, d) if covmode == COV_FULL else (K, SB, d))
    ns = np.zeros(K, dtype=np.int32)
    omega = np.ones(K)
    for j, h in enumerate(hmms):
        if h is None:  # :113-133 dummy one-state HMM with weight 0
            ns[j] = 1
            prior[j, 0] = 1.0
            A[j, 0, 0] = 1.0
            cov[j, 0] = np.eye(d) if covmode == COV_FULL else np.ones(d)
            omega[j] = 0.0
            continue
        S = len(h["prior"])
        ns[j] = S
        if use_post:  # :42-58
            al = np.asarray(h["varpar"]["alpha"], float)
            ep = np.asarray(h["varpar"]["epsilon"], float)
            lA = np.zeros((S, S))
            for k in range(S):
                lA[k] = psi(ep[k]) - psi(ep[k].sum())
            prior[j, :S] = np.exp(psi(al) - psi(al.sum()))
            A[j, :S, :S] = np.exp(lA)
        else:
            prior[j, :S] = h["prior"]
            A[j, :S, :S] = h["trans"]
        for i in range(S):
            cen[j, i] = h["pdf"][i]["mean"]
            c = np.asarray(h["pdf"][i]["cov"], float)
            scale = 1.0
            if use_post:  # :82,88 tilde_beta = (beta+1)/beta
                be = float(h["varpar"]["beta"][i])
                scale = (be + 1) / be
            if covmode == COV_DIAG:
                cov[j, i] = scale * np.diag(c)
            else:
                cov[j, i] = scale * c
    omega = omega / omega.sum()  # :140
    return dict(nstates=ns, prior=prior, A=A, centres=cen, covars=cov, omega=omega,
                covmode=covmode)


def clip_hyps(opt: dict):
    """vbhem_clip_hyps.m:20-85 (clip to hyps_min/hyps_max)."""
    opt = dict(opt)
    for name in ("alpha0", "eta0", "epsilon0", "v0", "lambda0", "W0"):
        val = np.array(opt[name], dtype=float, ndmin=1)
        hi = opt["hyps_max"][name]
        lo = opt["hyps_min"][name]
        val = np.where(val >= hi, hi, val)
        val = np.where(val <= lo, lo, val)
        opt[name] = val if np.ndim(opt[name]) else float(val[0])
    return opt


def default_opt(K: int, S: int, d: int, **over):
    """Defaults of vbhem_h3m_cluster.m:150-229 used by the EM loop."""
    m0 = {2: [256.0, 192.0], 3: [256.0, 192.0, 150.0]}.get(d, [0.0] * d)
    opt = dict(K=K, S=S, alpha0=1.0, eta0=1.0, epsilon0=1.0, m0=np.array(m0), W0=0.005,
               lambda0=1.0, v0=5.0, max_iter=200, minDiff=1e-5, Nv=100, tau=10,
               covmode=COV_FULL, verbose=0)
    opt["hyps_max"] = dict(alpha0=1.0686e13, eta0=1.0686e13, epsilon0=1.0686e13, v0=1e4,
                           lambda0=1.0686e13, W0=1.0686e13)
    opt["hyps_min"] = dict(alpha0=1.0686e-13, eta0=1.0686e-13, epsilon0=1.0686e-13,
                           v0=2.0612e-09 + d - 1, lambda0=1.0686e-13, W0=1.0686e-13)
    opt.update(over)
    opt["m0"] = np.asarray(opt["m0"], float).reshape(-1)
    return opt


def baseem_init(base: dict, opt: dict, randomb, randomg, omega_rand):
    """vbhemhmm_init.m:58-100 ('baseem', initopt.mode='u') with injected draws.

    randomb/randomg: [K,S] 0-based indices of the base HMM / its state;
    omega_rand: [K] uniform draws."""
    opt = clip_hyps(opt)
    K, S = opt["K"], opt["S"]
    Kb = base["prior"].shape[0]
    d = base["centres"].shape[2]
    covmode = base["covmode"]
    Nv = opt["Nv"] * Kb
    NLr = Nv / K
    post = dict(lam=np.zeros((K, S)), v=np.zeros((K, S)), m=np.zeros((K, S, d)),
                W=np.zeros((K, S, d, d) if covmode == COV_FULL else (K, S, d)),
                eta=np.zeros((K, S)), epsilon=np.zeros((K, S, S)))
    for j in range(K):
        for n in range(S):
            b, g = int(randomb[j, n]), int(randomg[j, n])
            post["lam"][j, n] = opt["lambda0"] + NLr / S
            post["v"][j, n] = opt["v0"] + NLr / S + 1
            post["m"][j, n] = base["centres"][b, g]
            if covmode == COV_DIAG:
                post["W"][j, n] = 1.0 / ((post["v"][j, n] - d - 1) * base["covars"][b, g])
            else:
                post["W"][j, n] = np.linalg.inv((post["v"][j, n] - d - 1) * base["covars"][b, g])
        prior = np.ones(S) / S
        Au = np.ones((S, S)) / S
        post["eta"][j] = prior * NLr + opt["eta0"]
        post["epsilon"][j] = (Au * NLr) / S + opt["epsilon0"]
    omega = np.asarray(omega_rand, float)
    omega = omega / omega.sum()
    post["alpha"] = opt["alpha0"] + omega * Nv
    post["W0mode"] = "iid" if np.size(opt["W0"]) == 1 else "diag"
    return post


def prelude(post: dict, covmode: int):
    """vbhem_h3m_c_step_fc.m:118-165 and :180-191 (cluster constants)."""
    K, S, d = post["m"].shape
    out = dict(logLambdaTilde=np.zeros((K, S)), c=np.zeros((K, S)), logA=np.zeros((K, S, S)),
               logPi=np.zeros((K, S)), m=post["m"].copy(),
               P=np.zeros_like(post["W"]))
    const = d * np.log(2)
    for j in range(K):
        for k in range(S):
            v = post["v"][j, k]
            t1 = psi(0.5 * (v + 1) - 0.5 * np.arange(1, d + 1))
            if covmode == COV_DIAG:
                # MATLAB writes sum(log(diag(W))) on a 1xd row; the intended
                # value (and the d==1 value) is sum(log(W)) -- SURVEY 2.4-1.
                lL = t1.sum() + const + np.log(post["W"][j, k]).sum()
            else:
                lL = t1.sum() + const + np.log(np.linalg.det(post["W"][j, k]))
            out["logLambdaTilde"][j, k] = lL
            out["c"][j, k] = -lL + d / post["lam"][j, k]
            ep = post["epsilon"][j, k]
            out["logA"][j, k] = psi(ep) - psi(ep.sum())
            out["P"][j, k] = v * post["W"][j, k]
        eta = post["eta"][j]
        out["logPi"][j] = psi(eta) - psi(eta.sum())
    return out


def responsibilities(L_elbo, tildeN, alpha):
    """vbhem_h3m_c_step_fc.m:271-283."""
    logOmega = psi(alpha) - psi(alpha.sum())
    log_Z = tildeN[:, None] * (logOmega[None, :] + L_elbo)
    ls = _logtrick_cols(log_Z.T)
    hat_Z = np.exp(log_Z - ls[:, None]) + 1e-50
    Z = hat_Z * tildeN[:, None]
    Nj = Z.sum(0) + 1e-50
    return logOmega, hat_Z, Z, Nj


def compute_statistics(Zcol, pairs_j: dict, S: int, d: int, covmode: int):
    """vbhem_compute_Statistics.m:1-85 for one cluster (loop over i)."""
    N1 = np.zeros(S)
    M = np.zeros((S, S))
    Nr = np.zeros(S)
    y = np.zeros((S, d))
    SC = np.zeros((S, d, d) if covmode == COV_FULL else (S, d))
    for i in range(len(Zcol)):
        z = Zcol[i]
        if z > 1e-8:
            N1 = N1 + z * pairs_j["sum_nu_1"][i]
            M = M + z * pairs_j["sum_xi"][i]
            Nr = Nr + z * pairs_j["emit_pr"][i]
            y = y + z * pairs_j["emit_mu"][i]
            SC = SC + z * pairs_j["emit_Mu"][i]
    return finish_statistics(N1, M, Nr, y, SC, S, covmode)


def finish_statistics(N1, M, Nr, y, SC, S, covmode):
    """vbhem_compute_Statistics.m:57-82 (normalisation of the gated sums)."""
    Nr = Nr + 1e-50
    y = y / Nr[:, None]
    if covmode == COV_DIAG:
        SC = SC / Nr[:, None] - y * y
    else:
        SC = SC / Nr[:, None, None] - y[:, :, None] * y[:, None, :]
    if S == 1:
        M = np.full((1, 1), 1e-12)
    return dict(Nj_rho1=N1, Nj_rho2rho=M, Nj_rho=Nr, y_bar=y, S_plus_C=SC)


def _W0(opt, d):
    W0 = np.asarray(opt["W0"], float)
    return W0 * np.eye(d) if W0.size == 1 else np.diag(W0)


def mstep_component(st: dict, opt: dict, covmode: int):
    """vbhem_mstep_component.m:1-70 for one cluster; returns its new posterior."""
    S = st["Nj_rho"].shape[0]
    d = st["y_bar"].shape[1]
    m0 = opt["m0"]
    lam0 = opt["lambda0"]
    W0inv = np.linalg.inv(_W0(opt, d))
    out = dict(eta=opt["eta0"] + st["Nj_rho1"], epsilon=opt["epsilon0"] + st["Nj_rho2rho"],
               lam=np.zeros(S), v=np.zeros(S), m=np.zeros((S, d)),
               W=np.zeros((S, d, d) if covmode == COV_FULL else (S, d)))
    for k in range(S):
        Nk = st["Nj_rho"][k]
        out["lam"][k] = lam0 + Nk
        out["v"][k] = opt["v0"] + Nk + 1
        out["m"][k] = (lam0 * m0 + Nk * st["y_bar"][k]) / (lam0 + Nk)
        mult1 = lam0 * Nk / (lam0 + Nk)
        diff3 = st["y_bar"][k] - m0
        if covmode == COV_DIAG:
            tW = np.linalg.inv(W0inv + Nk * np.diag(st["S_plus_C"][k]) + mult1 * np.outer(diff3, diff3))
            out["W"][k] = np.diag((tW + tW.T) / 2)
        else:
            tW = np.linalg.inv(W0inv + Nk * st["S_plus_C"][k] + mult1 * np.outer(diff3, diff3))
            out["W"][k] = (tW + tW.T) / 2
    if np.ndim(out["epsilon"]) == 0:
        out["epsilon"] = np.full((S, S), float(out["epsilon"]))
    return out


def lower_bound(hat_Z, Z, Nj, L_elbo, logOmega, post: dict, consts: dict, opt: dict):
    """vbhemh3m_lb.m:1-186 (no derivatives)."""
    K = post["alpha"].shape[0]
    d = len(opt["m0"])
    S = opt["S"]
    covmode = opt["covmode"]
    a0, e0, ep0, m0, l0, v0 = (opt["alpha0"], opt["eta0"], opt["epsilon0"], opt["m0"],
                               opt["lambda0"], opt["v0"])
    W0 = _W0(opt, d)
    W0inv = np.linalg.inv(W0)
    if np.size(opt["W0"]) == 1:
        logdetW0inv = d * np.log(W0inv[0, 0])
    else:
        logdetW0inv = np.log(np.diag(W0inv)).sum()
    logCalpha0 = gammaln(K * a0) - K * gammaln(a0)
    logCeta0 = gammaln(S * e0) - S * gammaln(e0)
    logCepsilon0 = np.full(S, gammaln(S * ep0) - S * gammaln(ep0))
    q = np.arange(1, d + 1)
    logB0 = (v0 / 2) * logdetW0inv - (v0 * d / 2) * np.log(2) - (d * (d - 1) / 4) * np.log(np.pi) \
        - gammaln(0.5 * (v0 + 1 - q)).sum()
    const2 = d * np.log(l0 / (2 * np.pi))
    alpha = post["alpha"]
    logCalpha = gammaln(alpha.sum()) - gammaln(alpha).sum()
    lLT = consts["logLambdaTilde"]
    Lt1 = (Z * L_elbo).sum()
    Lt2 = Nj @ logOmega
    Lt3 = K * logCeta0 + (e0 - 1) * consts["logPi"].sum()
    Lt4 = K * logCepsilon0.sum() + (ep0 - 1) * consts["logA"].sum()
    Lt5 = 0.0
    Lt6 = logCalpha0 + (a0 - 1) * logOmega.sum()
    Lt7 = (hat_Z * np.log(hat_Z)).sum()
    Lt8 = logCalpha + (alpha - 1) @ logOmega
    Lt9 = 0.0
    Lt10 = 0.0
    for j in range(K):
        lam = post["lam"][j]
        v = post["v"][j]
        H = 0.0
        mWm = np.zeros(S)
        trW = np.zeros(S)
        for k in range(S):
            Wk = post["W"][j, k] if covmode == COV_FULL else np.diag(post["W"][j, k])
            logBk = -(v[k] / 2) * np.log(np.linalg.det(Wk)) - (v[k] * d / 2) * np.log(2) \
                - (d * (d - 1) / 4) * np.log(np.pi) - gammaln(0.5 * (v[k] + 1 - q)).sum()
            H = H - logBk - 0.5 * (v[k] - d - 1) * lLT[j, k] + 0.5 * v[k] * d
            diff = post["m"][j, k] - m0
            mWm[k] = diff @ Wk @ diff
            trW[k] = np.trace(W0inv @ Wk)
        eta = post["eta"][j]
        eps = post["epsilon"][j]
        logCeta = gammaln(eta.sum()) - gammaln(eta).sum()
        logCeps = np.array([gammaln(eps[k].sum()) - gammaln(eps[k]).sum() for k in range(S)])
        Lt51 = 0.5 * (const2 + lLT[j] - d * l0 / lam - l0 * v * mWm).sum()
        Lt52 = S * logB0 + 0.5 * (v0 - d - 1) * lLT[j].sum() - 0.5 * (v * trW).sum()
        Lt5 += Lt51 + Lt52
        Lt9a = logCeta + (eta - 1) @ consts["logPi"][j]
        Lt9b = logCeps + ((eps - 1) * consts["logA"][j]).sum(1)
        Lt9 += Lt9a + Lt9b.sum()
        Lt10 += 0.5 * (lLT[j] + d * np.log(lam / (2 * np.pi))).sum() - 0.5 * d * S - H
    return Lt1 + Lt2 + Lt3 + Lt4 + Lt5 + Lt6 - Lt7 - Lt8 - Lt9 - Lt10


def lower_bound_derivs(logOmega, post: dict, consts: dict, opt: dict, clipped=None):
    """vbhemh3m_lb.m:202-356 loop by loop (iid or diag W0; the diag branch with
    Kr*Sr for the reference's undefined K*S)."""
    from scipy.special import digamma as ps
    K = post["alpha"].shape[0]
    S = opt["S"]
    d = len(opt["m0"])
    covmode = opt["covmode"]
    a0, e0, ep0, m0, l0, v0 = (opt["alpha0"], opt["eta0"], opt["epsilon0"], np.asarray(opt["m0"], float),
                               opt["lambda0"], opt["v0"])
    W0 = _W0(opt, d)
    W0inv = np.linalg.inv(W0)
    iid = np.size(opt["W0"]) == 1
    logdetW0inv = d * np.log(W0inv[0, 0]) if iid else np.log(np.diag(W0inv)).sum()
    dLt = {}
    dLt["alpha0"] = K * ps(K * a0) - K * ps(a0) + np.sum(logOmega)                  # :206-212
    dLt["eta0"] = K * (S * ps(S * e0) - S * ps(e0)) + np.sum(consts["logPi"])        # :216-222
    dLt["epsilon0"] = K * S * (S * ps(S * ep0) - S * ps(ep0)) + np.sum(consts["logA"])  # :226-232
    dB = 0.5 * logdetW0inv - (d / 2) * np.log(2) - 0.5 * sum(ps(0.5 * (v0 + 1 - q)) for q in range(1, d + 1))
    dLt["v0"] = K * S * dB + 0.5 * np.sum(consts["logLambdaTilde"])                  # :236-237
    dl = 0.0
    for j in range(K):                                                                # :240-248
        for k in range(S):
            Wk = post["W"][j, k] if covmode == COV_FULL else np.diag(post["W"][j, k])
            diff = post["m"][j, k] - m0
            mWm = diff @ Wk @ diff
            dl += 0.5 * (d / l0 - d / post["lam"][j, k] - post["v"][j, k] * mWm)
    dLt["lambda0"] = dl
    if iid:                                                                           # :251-272
        w0i = W0inv[0, 0]
        myW0 = 1.0 / w0i
        acc = 0.0
        for j in range(K):
            for k in range(S):
                W = post["W"][j, k]
                tr = np.trace(W) if covmode == COV_FULL else np.sum(W)
                acc += -post["v"][j, k] * w0i ** 2 * tr
        dLt["W0"] = np.array([K * S * (-0.5 * v0 * d * w0i) - 0.5 * acc])
    else:                                                                             # :275-298
        w0i = np.diag(W0inv)
        myW0 = 1.0 / w0i
        acc = np.zeros(d)
        for j in range(K):
            for k in range(S):
                W = post["W"][j, k]
                dg = np.diag(W) if covmode == COV_FULL else W
                acc += -post["v"][j, k] * w0i ** 2 * dg
        dLt["W0"] = K * S * (-0.5 * v0 * w0i) - 0.5 * acc
    tmp = np.zeros(d)
    for j in range(K):                                                                # :304-314
        for k in range(S):
            Wk = post["W"][j, k] if covmode == COV_FULL else np.diag(post["W"][j, k])
            tmp += l0 * post["v"][j, k] * (Wk @ (post["m"][j, k] - m0))
    dLt["m0"] = tmp
    if clipped is not None:                                                           # :321-334
        for name, fl in clipped.items():
            g = np.atleast_1d(dLt[name]).astype(float)
            for i in range(len(fl)):
                if fl[i] == 1 and g[i] > 0:
                    g[i] = 0.0
                if fl[i] == -1 and g[i] < 0:
                    g[i] = 0.0
            dLt[name] = g
    return dict(d_logalpha0=dLt["alpha0"] * a0, d_logeta0=dLt["eta0"] * e0,            # :337-346
                d_logepsilon0=dLt["epsilon0"] * ep0, d_logv0D1=dLt["v0"] * (v0 - d + 1),
                d_loglambda0=dLt["lambda0"] * l0, d_sqrtW0inv=dLt["W0"] * (myW0 ** 1.5) * (-2),
                d_logW0=dLt["W0"] * myW0, d_m0=dLt["m0"])


def convert_to_point(post: dict, covmode: int):
    """convert_h3mrtoh3mb.m:9-79 (posterior -> point-estimate HMMs)."""
    K, S, d = post["m"].shape
    prior = post["eta"] / post["eta"].sum(1, keepdims=True)
    A = post["epsilon"].copy()
    for j in range(K):
        for k in range(S):
            sc = A[j, k].sum()
            A[j, k] = A[j, k] / (sc if sc != 0 else 1.0)
    cov = np.zeros_like(post["W"])
    for j in range(K):
        for k in range(S):
            v = post["v"][j, k]
            den = (v - d - 1) if v > d + 1 else v
            if covmode == COV_DIAG:
                tC = (1.0 / post["W"][j, k]) / den
                cov[j, k] = (tC + tC) / 2
            else:
                tC = np.linalg.inv(post["W"][j, k]) / den
                cov[j, k] = (tC + tC.T) / 2
    omega = post["alpha"] / post["alpha"].sum()
    return dict(prior=prior, A=A, centres=post["m"].copy(), covars=cov, omega=omega)


def em_step_fc(post: dict, base: dict, opt: dict, estep=None):
    """vbhem_h3m_c_step_fc.m:1-449: EM loop; returns the output dict of
    form_outputH3M.m (labels 0-based).  ``estep(consts)`` -> per-pair dict
    (defaults to the C oracle)."""
    covmode = base["covmode"]
    K, S, d = post["m"].shape
    Kb = base["prior"].shape[0]
    T = opt["tau"]
    tildeN = opt["Nv"] * Kb * base["omega"]
    post = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in post.items()}
    lastL = -np.finfo(float).max
    it = 0
    LogLs = []
    syn = None
    stable = True
    while True:
        consts = prelude(post, covmode)
        pairs = estep(consts) if estep is not None else c_estep_pairs(base, consts, T)
        logOmega, hat_Z, Z, Nj = responsibilities(pairs["LL_elbo"], tildeN, post["alpha"])
        L = lower_bound(hat_Z, Z, Nj, pairs["LL_elbo"], logOmega, post, consts, opt)
        do_break = False
        if it > 1:
            if abs((L - lastL) / lastL) <= opt["minDiff"]:
                do_break = True
        if it == opt["max_iter"]:
            do_break = True
        if np.isnan(L):
            L = -np.inf
            stable = False
            break
        new = dict(eta=np.zeros((K, S)), epsilon=np.zeros((K, S, S)), lam=np.zeros((K, S)),
                   v=np.zeros((K, S)), m=np.zeros((K, S, d)), W=np.zeros_like(post["W"]))
        syn = []
        for j in range(K):
            pj = {k: pairs[k][:, j] for k in ("sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")}
            st = compute_statistics(Z[:, j], pj, S, d, covmode)
            syn.append(st)
            hj = mstep_component(st, opt, covmode)
            for k in new:
                new[k][j] = hj[k]
        new["alpha"] = opt["alpha0"] + Nj
        new["W0mode"] = post.get("W0mode", "iid")
        post = new
        it += 1
        LogLs.append(L)
        lastL = L
        if do_break:
            break
    out = dict(post=post, LogLs=np.array(LogLs), LL=L, hat_Z=hat_Z, L_elbo=pairs["LL_elbo"],
               Nj=Nj, stable=stable, iters=it)
    if stable:
        pt = convert_to_point(post, covmode)
        out.update(point=pt, label=hat_Z.argmax(1),
                   N1=np.array([s["Nj_rho1"] for s in syn]),
                   M=np.array([s["Nj_rho2rho"] for s in syn]),
                   Nrho=np.array([s["Nj_rho"] for s in syn]))
    return out


# ---------------------------------------------------------------------------
# VB-HMM forward-backward (src/hmm/vbhmm_fb.m, vbhmm_fb_mex.c)
# ---------------------------------------------------------------------------
def pack_sequences(data, dim: int):
    """data: list of [T_n x dim] arrays (vbhmm_fb.m `data{n}`, one row per
    observation) -> (offsets [N+1] int32, x [sum T][dim] fp64, maxT)."""
    lens = [int(np.asarray(a).reshape(-1, dim).shape[0]) for a in data]
    offsets = np.zeros(len(data) + 1, dtype=np.int32)
    offsets[1:] = np.cumsum(lens)
    x = (np.concatenate([np.asarray(a, dtype=np.float64).reshape(-1, dim) for a in data], axis=0)
         if offsets[-1] > 0 else np.zeros((0, dim)))
    return offsets, np.ascontiguousarray(x), max(lens) if lens else 0


def vbhmm_prelude(varpar: dict):
    """vbhmm_fb.m:54-93 (usegroups = 0) and :121-122: logLambdaTilde [K],
    logATilde [K][K] (row format), logPiTilde [K], const_denominator, and the
    MEX inputs t_pz1 = exp(logPiTilde), t_tpztzt1 = exp(logATilde).
    varpar: v [K], W [K][dim][dim], epsilon [K][K], alpha [K], m [K][dim], beta [K]."""
    from scipy.special import digamma
    v = np.asarray(varpar["v"], dtype=np.float64)
    W = np.asarray(varpar["W"], dtype=np.float64)
    K, dim = np.asarray(varpar["m"]).shape
    const = dim * np.log(2.0)
    lLT = np.zeros(K)
    for k in range(K):
        t1 = digamma(0.5 * (v[k] + 1.0) - 0.5 * np.arange(1, dim + 1))
        lLT[k] = t1.sum() + const + np.log(np.linalg.det(W[k]))
    eps = np.asarray(varpar["epsilon"], dtype=np.float64)
    logA = digamma(eps) - digamma(eps.sum(axis=1, keepdims=True))
    alpha = np.asarray(varpar["alpha"], dtype=np.float64)
    logPi = digamma(alpha) - digamma(alpha.sum())
    return dict(logLambdaTilde=lLT, logATilde=logA, logPiTilde=logPi,
                const_denominator=dim * np.log(2 * np.pi) / 2.0,
                pz1=np.exp(logPi), A=np.exp(logA))


def c_vbhmm_fb(data, varpar: dict, pre: dict = None):
    """vbhmm_fb_mex outputs from the C restatement: logrho [maxT][N][K],
    gamma [maxT][N][K], xi_sum [N][K][K] ([n][from][to]), phi_norm [N]."""
    lib = load_c_oracle()
    m = _c64(varpar["m"])
    K, dim = m.shape
    pre = vbhmm_prelude(varpar) if pre is None else pre
    offsets, x, maxT = pack_sequences(data, dim)
    N = len(data)
    out = dict(logrho=np.zeros((maxT, N, K)), gamma=np.zeros((maxT, N, K)),
               xi_sum=np.zeros((N, K, K)), phi_norm=np.zeros(N))
    rc = lib.oracle_vbhmm_fb(
        N, K, dim, maxT, offsets.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(x), _dp(m),
        _dp(_c64(varpar["W"])), _dp(_c64(varpar["v"])), _dp(_c64(varpar["beta"])),
        _dp(_c64(pre["logLambdaTilde"])), float(pre["const_denominator"]), _dp(_c64(pre["pz1"])),
        _dp(_c64(pre["A"])), _dp(out["logrho"]), _dp(out["gamma"]), _dp(out["xi_sum"]),
        _dp(out["phi_norm"]))
    if rc != 0:
        raise ValueError(f"oracle_vbhmm_fb failed rc={rc}")
    return out


def twin_vbhmm_fb(data, varpar: dict, pre: dict = None):
    """numpy restatement of the MATLAB path vbhmm_fb.m:227-379 (vectorised the way
    the .m file is, independent of the C restatement's loops); same outputs."""
    m = np.asarray(varpar["m"], dtype=np.float64)
    W = np.asarray(varpar["W"], dtype=np.float64)
    v = np.asarray(varpar["v"], dtype=np.float64)
    beta = np.asarray(varpar["beta"], dtype=np.float64)
    K, dim = m.shape
    pre = vbhmm_prelude(varpar) if pre is None else pre
    N = len(data)
    maxT = max([np.asarray(a).reshape(-1, dim).shape[0] for a in data] + [0])
    logrho_S = np.zeros((maxT, N, K))
    gamma_all = np.zeros((maxT, N, K))
    xi_sum = np.zeros((N, K, K))
    phi = np.zeros(N)
    pz1, A = pre["pz1"], pre["A"]
    for n in range(N):
        tdata = np.asarray(data[n], dtype=np.float64).reshape(-1, dim).T   # [dim x T]
        tT = tdata.shape[1]
        delta = np.zeros((K, tT))
        for k in range(K):
            diff = tdata - m[k][:, None]
            mterm = ((W[k] @ diff) * diff).sum(axis=0)
            delta[k] = dim / beta[k] + v[k] * mterm
        logrho = 0.5 * pre["logLambdaTilde"][:, None] - 0.5 * delta - pre["const_denominator"]
        logrho_S[:tT, n, :] = logrho.T
        fb = logrho.T                                   # [T x K]
        mx = fb.max(axis=1) if tT else np.zeros(0)
        px = np.exp(fb - mx[:, None])
        if tT >= 1:
            al = np.zeros((tT, K)); c = np.zeros(tT); be = np.zeros((tT, K)); g = np.zeros((K, tT))
            Dl = pz1 * px[0]
            c[0] = Dl.sum(); al[0] = Dl / c[0]
            for i in range(1, tT):
                Dl = (al[i - 1] @ A) * px[i]
                c[i] = Dl.sum(); al[i] = Dl / c[i]
            be[tT - 1] = 1.0
            g[:, tT - 1] = al[tT - 1] * be[tT - 1]
            sx = np.zeros((K, K))
            for i in range(tT - 2, -1, -1):
                bpi = be[i + 1] * px[i + 1]
                be[i] = (bpi @ A.T) / c[i + 1]
                g[:, i] = al[i] * be[i]
                sx += (A * np.outer(al[i], bpi)) / c[i + 1]
            gamma_all[:tT, n, :] = g.T
            xi_sum[n] = sx
            phi[n] = np.log(c).sum() + mx.sum()
    return dict(logrho=logrho_S, gamma=gamma_all, xi_sum=xi_sum, phi_norm=phi)

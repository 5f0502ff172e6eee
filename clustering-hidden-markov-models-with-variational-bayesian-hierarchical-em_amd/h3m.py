"""Packed H3M containers, input conversion and synthetic workloads.

* :class:`BaseSet` -- the N base HMMs ``h3m_b`` in the packed, zero-padded
  layout the device E-step consumes (include/vbhem_estep.h).
* :class:`Posterior` -- the K cluster HMMs' variational parameters ``h3m_r``
  (eta, epsilon, lambda, v, m, W per cluster; alpha over clusters).
* :func:`hmms_to_h3m_hem` -- src/vbhem/hmms_to_h3m_hem.m:1-144 (host), and
  :func:`hmms_to_h3m_hem_device` -- the same conversion as a HIP kernel.
* :func:`baseem_init` -- the 'baseem' initialisation of
  src/vbhem/vbhemhmm_init.m:58-100 with the random draws injected.
* :func:`synth_workload` -- the synthetic (N, K, S, d) grids of BASELINE.md.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional

import numpy as np
import torch

COV_DIAG, COV_FULL = 0, 1


@dataclasses.dataclass
class BaseSet:
    """h3m_b, packed: nstates [N], prior [N,SB], A [N,SB,SB] (A[i][from][to]),
    centres [N,SB,d], covars [N,SB,d,d] (full) | [N,SB,d] (diag), omega [N]."""
    nstates: torch.Tensor
    prior: torch.Tensor
    A: torch.Tensor
    centres: torch.Tensor
    covars: torch.Tensor
    omega: torch.Tensor
    covmode: int

    @property
    def N(self) -> int:
        return int(self.prior.shape[0])

    @property
    def SB(self) -> int:
        return int(self.prior.shape[1])

    @property
    def d(self) -> int:
        return int(self.centres.shape[2])

    def to(self, device) -> "BaseSet":
        f = lambda t: t.to(device).contiguous()
        return BaseSet(f(self.nstates), f(self.prior), f(self.A), f(self.centres), f(self.covars),
                       f(self.omega), self.covmode)

    def shard(self, lo: int, hi: int) -> "BaseSet":
        return BaseSet(self.nstates[lo:hi], self.prior[lo:hi], self.A[lo:hi], self.centres[lo:hi],
                       self.covars[lo:hi], self.omega[lo:hi], self.covmode)

    def numpy(self) -> dict:
        return dict(nstates=self.nstates.cpu().numpy().astype(np.int32),
                    prior=self.prior.cpu().numpy(), A=self.A.cpu().numpy(),
                    centres=self.centres.cpu().numpy(), covars=self.covars.cpu().numpy(),
                    omega=self.omega.cpu().numpy(), covmode=self.covmode)

    @staticmethod
    def from_numpy(d: dict) -> "BaseSet":
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64)
        return BaseSet(torch.as_tensor(np.asarray(d["nstates"], dtype=np.int32)), t(d["prior"]),
                       t(d["A"]), t(d["centres"]), t(d["covars"]), t(d["omega"]), int(d["covmode"]))


@dataclasses.dataclass
class Posterior:
    """h3m_r variational parameters (vbhemhmm_init.m:77-99, vbhem_mstep_component.m:42-69):
    alpha [K]; eta [K,S]; epsilon [K,S,S]; lam [K,S]; v [K,S]; m [K,S,d];
    W [K,S,d,d] (full) | [K,S,d] (diag)."""
    alpha: np.ndarray
    eta: np.ndarray
    epsilon: np.ndarray
    lam: np.ndarray
    v: np.ndarray
    m: np.ndarray
    W: np.ndarray
    W0mode: str = "iid"

    @property
    def K(self) -> int:
        return int(self.m.shape[0])

    @property
    def S(self) -> int:
        return int(self.m.shape[1])

    def copy(self) -> "Posterior":
        return Posterior(*(np.array(getattr(self, f.name)) if f.name != "W0mode" else self.W0mode
                           for f in dataclasses.fields(self)))

    def asdict(self) -> dict:
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)}


# ----------------------------------------------------------------------------
# input conversion (hmms_to_h3m_hem.m)
# ----------------------------------------------------------------------------
def hmms_to_h3m_hem(hmms: List[Optional[dict]], covmode: int = COV_FULL,
                    use_post: bool = True) -> BaseSet:
    """Convert a list of VB-HMMs (dicts with prior, trans, pdf[{mean,cov}],
    varpar{alpha,epsilon,beta}) into a packed :class:`BaseSet`.

    use_post=True (the vbhem_h3m_cluster default, :237): prior/A become
    exp(E[log]) -- sub-stochastic, never renormalised (:42-58) -- and each
    covariance is inflated by (beta+1)/beta (:82,88).  Empty entries (None)
    become a one-state dummy with weight 0 (:113-133)."""
    from scipy.special import digamma

    nin = next(len(h["pdf"][0]["mean"]) for h in hmms if h is not None)
    N = len(hmms)
    SB = max(len(h["prior"]) if h is not None else 1 for h in hmms)
    d = nin
    ns = np.ones(N, dtype=np.int32)
    prior = np.zeros((N, SB))
    A = np.zeros((N, SB, SB))
    cen = np.zeros((N, SB, d))
    cov = np.zeros((N, SB, d, d) if covmode == COV_FULL else (N, SB, d))
    omega = np.ones(N)
    for j, h in enumerate(hmms):
        if h is None:
            prior[j, 0] = 1.0
            A[j, 0, 0] = 1.0
            cov[j, 0] = np.eye(d) if covmode == COV_FULL else 1.0
            omega[j] = 0.0
            continue
        S = len(h["prior"])
        ns[j] = S
        if use_post:
            al = np.asarray(h["varpar"]["alpha"], float)
            ep = np.asarray(h["varpar"]["epsilon"], float)
            prior[j, :S] = np.exp(digamma(al) - digamma(al.sum()))
            A[j, :S, :S] = np.exp(digamma(ep) - digamma(ep.sum(1, keepdims=True)))
            infl = (np.asarray(h["varpar"]["beta"], float) + 1) / np.asarray(h["varpar"]["beta"], float)
        else:
            prior[j, :S] = h["prior"]
            A[j, :S, :S] = h["trans"]
            infl = np.ones(S)
        for s in range(S):
            cen[j, s] = h["pdf"][s]["mean"]
            c = np.asarray(h["pdf"][s]["cov"], float)
            cov[j, s] = infl[s] * (np.diag(c) if covmode == COV_DIAG else c)
    omega = omega / omega.sum()
    return BaseSet.from_numpy(dict(nstates=ns, prior=prior, A=A, centres=cen, covars=cov,
                                   omega=omega, covmode=covmode))


def hmms_to_h3m_hem_device(hmms: List[Optional[dict]], covmode: int = COV_FULL,
                           use_post: bool = True, device="cuda") -> BaseSet:
    """:func:`hmms_to_h3m_hem` with the conversion on the device
    (vbhem_hmms_to_h3m, csrc/vbhem_h3m.hip): the HMM list is packed into padded
    arrays of the raw variational counts, point estimates, means and covariances
    here, uploaded once, and the digamma / exp / inflation / weights run as a
    kernel; the BaseSet comes back on ``device``."""
    import ctypes

    from . import _capi
    nin = next(len(h["pdf"][0]["mean"]) for h in hmms if h is not None)
    N, d = len(hmms), nin
    SB = max(len(h["prior"]) if h is not None else 1 for h in hmms)
    ns = np.zeros(N, dtype=np.int32)
    al, be = np.ones((N, SB)), np.ones((N, SB))
    ep = np.ones((N, SB, SB))
    pr, tr = np.zeros((N, SB)), np.zeros((N, SB, SB))
    mu, cv = np.zeros((N, SB, d)), np.zeros((N, SB, d, d))
    for j, h in enumerate(hmms):
        if h is None:
            continue
        S = len(h["prior"])
        ns[j] = S
        if use_post:
            al[j, :S] = h["varpar"]["alpha"]
            ep[j, :S, :S] = h["varpar"]["epsilon"]
            be[j, :S] = h["varpar"]["beta"]
        else:
            pr[j, :S] = h["prior"]
            tr[j, :S, :S] = h["trans"]
        for st in range(S):
            mu[j, st] = h["pdf"][st]["mean"]
            cv[j, st] = h["pdf"][st]["cov"]
    dev = torch.device(device)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)
    ins = dict(ns=torch.as_tensor(ns, device=dev), al=t(al), ep=t(ep), be=t(be), pr=t(pr), tr=t(tr),
               mu=t(mu), cv=t(cv))
    out = dict(prior=torch.empty((N, SB), dtype=torch.float64, device=dev),
               A=torch.empty((N, SB, SB), dtype=torch.float64, device=dev),
               centres=torch.empty((N, SB, d), dtype=torch.float64, device=dev),
               covars=torch.empty((N, SB, d, d) if covmode == COV_FULL else (N, SB, d),
                                  dtype=torch.float64, device=dev),
               omega=torch.empty((N,), dtype=torch.float64, device=dev))
    ws = torch.zeros((1,), dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = _capi.ptr
    _capi.check(_capi.lib().vbhem_hmms_to_h3m(
        N, SB, d, int(covmode), 1 if use_post else 0, p(ins["ns"]), p(ins["al"]), p(ins["ep"]),
        p(ins["be"]), p(ins["pr"]), p(ins["tr"]), p(ins["mu"]), p(ins["cv"]), p(out["prior"]),
        p(out["A"]), p(out["centres"]), p(out["covars"]), p(out["omega"]), p(ws), st),
        "vbhem_hmms_to_h3m")
    nstates = torch.as_tensor(np.maximum(ns, 1), dtype=torch.int32, device=dev)
    return BaseSet(nstates, out["prior"], out["A"], out["centres"], out["covars"], out["omega"],
                   int(covmode))


# ----------------------------------------------------------------------------
# options (vbhem_h3m_cluster.m defaults consumed by the EM loop)
# ----------------------------------------------------------------------------
def default_options(K: int, S: int, d: int, **over) -> dict:
    """vbhem_h3m_cluster.m:150-229 (the subset the EM loop reads)."""
    m0 = {2: [256.0, 192.0], 3: [256.0, 192.0, 150.0]}.get(d, [0.0] * d)
    opt = dict(K=K, S=S, alpha0=1.0, eta0=1.0, epsilon0=1.0, m0=m0, W0=0.005, lambda0=1.0, v0=5.0,
               max_iter=200, minDiff=1e-5, Nv=100, tau=10, covmode=COV_FULL, verbose=0)
    opt["hyps_max"] = dict(alpha0=1.0686e13, eta0=1.0686e13, epsilon0=1.0686e13, v0=1e4,
                           lambda0=1.0686e13, W0=1.0686e13)
    opt["hyps_min"] = dict(alpha0=1.0686e-13, eta0=1.0686e-13, epsilon0=1.0686e-13,
                           v0=2.0612e-09 + d - 1, lambda0=1.0686e-13, W0=1.0686e-13)
    opt.update(over)
    opt["m0"] = np.asarray(opt["m0"], dtype=float).reshape(-1)
    if opt["v0"] <= d - 1:
        raise ValueError("v0 not large enough...should be > D-1")  # vbhem_h3m_cluster.m:233
    return opt


def clip_hyps(opt: dict, with_flags: bool = False):
    """vbhem_clip_hyps.m:20-85: clip each hyperparameter into [hyps_min, hyps_max].
    with_flags: also return the clipped flags (+1 at the max, -1 at the min), which
    vbhemh3m_lb.m:326-343 uses to zero derivatives pointing out of range."""
    out = dict(opt)
    flags = {}
    for name in ("alpha0", "eta0", "epsilon0", "v0", "lambda0", "W0"):
        val = np.array(opt[name], dtype=float, ndmin=1)
        fl = np.zeros(val.size)
        hi, lo = opt["hyps_max"][name], opt["hyps_min"][name]
        fl[val >= hi] = 1.0
        val = np.where(val >= hi, hi, val)
        fl[val <= lo] = -1.0
        val = np.where(val <= lo, lo, val)
        out[name] = val if np.ndim(opt[name]) else float(val[0])
        flags[name] = fl
    return (out, flags) if with_flags else out


def baseem_init(base: BaseSet, opt: dict, randomb: np.ndarray, randomg: np.ndarray,
                omega_rand: np.ndarray, n_total: Optional[int] = None) -> Posterior:
    """'baseem' initialisation (vbhemhmm_init.m:58-100, initopt.mode='u').

    randomb/randomg [K,S]: 0-based base-HMM / state draws (MATLAB randi);
    omega_rand [K]: uniform draws (MATLAB rand).  ``n_total`` = Kb when the
    draws come from a subset of a larger base set."""
    opt = clip_hyps(opt)
    K, S = opt["K"], opt["S"]
    Kb, d = (base.N if n_total is None else int(n_total)), base.d
    Nv = opt["Nv"] * Kb
    NLr = Nv / K
    lam = np.full((K, S), opt["lambda0"] + NLr / S)
    v = np.full((K, S), opt["v0"] + NLr / S + 1)
    rb = np.asarray(randomb, dtype=np.int64)
    rg = np.asarray(randomg, dtype=np.int64)
    ib = torch.as_tensor(rb.reshape(-1), device=base.centres.device)
    ig = torch.as_tensor(rg.reshape(-1), device=base.centres.device)
    cen = base.centres[ib, ig]
    cov = base.covars[ib, ig]
    m = cen.cpu().numpy().reshape(K, S, d)
    cov = cov.cpu().numpy()
    scale = (v.reshape(-1) - d - 1)
    if base.covmode == COV_DIAG:
        W = (1.0 / (scale[:, None] * cov)).reshape(K, S, d)
    else:
        W = np.linalg.inv(scale[:, None, None] * cov).reshape(K, S, d, d)
    eta = np.full((K, S), (1.0 / S) * NLr + opt["eta0"])
    epsilon = np.full((K, S, S), ((1.0 / S) * NLr) / S + opt["epsilon0"])
    omega = np.asarray(omega_rand, dtype=float)
    omega = omega / omega.sum()
    alpha = opt["alpha0"] + omega * Nv
    return Posterior(alpha=alpha, eta=eta, epsilon=epsilon, lam=lam, v=v, m=m, W=W,
                     W0mode="iid" if np.size(opt["W0"]) == 1 else "diag")


def baseem_draws(base: BaseSet, K: int, S: int, seed: int):
    """Seeded stand-in for MATLAB's randi/rand in baseem (numpy PCG64)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    rb = rng.integers(0, base.N, size=(K, S))
    ns = base.nstates.cpu().numpy()
    rg = np.floor(rng.random((K, S)) * ns[rb]).astype(np.int64)
    om = rng.random(K)
    return rb, rg, om


# ----------------------------------------------------------------------------
# 'wtkmeans' initialisation (vbhemhmm_init.m:294-425, my_weighted_kmeans.m)
# ----------------------------------------------------------------------------
def make_gmm_weights(p: np.ndarray, A: np.ndarray, mode: str) -> np.ndarray:
    """vbhemhmm_init.m makeGMMweights (:1109-1135): a base HMM's state weights."""
    p = np.asarray(p, dtype=float).reshape(-1)
    if "0" in mode:
        for _ in range(50):
            p = p @ A
        return p
    if "3" in mode:
        out = p.copy()
        for _ in range(2):
            p = p @ A
            out = out + p
        return out / 3.0
    if "x" in mode:
        return np.full(p.size, 1.0 / p.size)
    raise ValueError("unknown mode")


def make_a_prior(N: int, mode: str, rng: np.random.Generator):
    """vbhemhmm_init.m makeAprior (:1138-1150): uniform ('u') or random ('r') prior / A."""
    if "u" in mode:
        return np.full(N, 1.0 / N), np.full((N, N), 1.0 / N)
    if "r" in mode:
        prior = rng.random(N)
        prior = prior / prior.sum()
        A = rng.random((N, N))
        return prior, A / A.sum(1, keepdims=True)
    raise ValueError("unknown mode")


def _wk_centroids(point, cluster, weight, K):
    """my_weighted_kmeans.m gcentroids: weighted centres (zero for a weightless cluster)."""
    cen = np.zeros((K, point.shape[1]))
    cw = np.zeros(K)
    for j in range(K):
        mem = cluster == j
        cw[j] = weight[mem].sum()
        cen[j] = (point[mem] * weight[mem, None]).sum(0)
        if cw[j] > 0:
            cen[j] = cen[j] / cw[j]
    return cen, cw


def _wk_energy(point, weight, cen, cw, cluster):
    """my_weighted_kmeans.m genergy: member distances scaled by cw / (cw - w)."""
    f = np.zeros(point.shape[0])
    energy = np.zeros(cen.shape[0])
    with np.errstate(divide="ignore", invalid="ignore"):  # MATLAB: x/0 = Inf, 0/0 = NaN
        for j in range(cen.shape[0]):
            mem = cluster == j
            fm = ((point[mem] - cen[j]) ** 2).sum(1)
            energy[j] = (weight[mem] * fm).sum()
            f[mem] = fm * cw[j] / (cw[j] - weight[mem])
    return f, energy


def _nanargmin0(fmat: np.ndarray) -> np.ndarray:
    """MATLAB min(x, [], 1): NaN skipped, the first of equal minima; all-NaN -> 1st."""
    x = np.where(np.isnan(fmat), np.inf, fmat)
    return np.argmin(x, axis=0)


def weighted_kmeans(K: int, it_max: int, point: np.ndarray, weight: np.ndarray,
                    centres: np.ndarray):
    """my_weighted_kmeans.m: points [n][dim] with weights [n] from initial centres
    [K][dim]; returns (0-based cluster [n], centres [K][dim], energies)."""
    point = np.asarray(point, dtype=float)
    weight = np.asarray(weight, dtype=float).reshape(-1)
    cen = np.asarray(centres, dtype=float)
    d2 = ((point[None, :, :] - cen[:, None, :]) ** 2).sum(2)          # [K][n]
    cluster = _nanargmin0(d2)
    cen, cw = _wk_centroids(point, cluster, weight, K)
    f, energy = _wk_energy(point, weight, cen, cw, cluster)
    old = energy.sum()
    energies = [old]
    it = 0
    while it < it_max:
        fmat = np.zeros((K, point.shape[0]))
        with np.errstate(divide="ignore", invalid="ignore"):
            for j in range(K):
                mem = cluster == j
                fmat[j, mem] = f[mem]
                non = ~mem
                adj = cw[j] / (cw[j] + weight[non])
                fmat[j, non] = ((point[non] - cen[j]) ** 2).sum(1) * adj
        cluster = _nanargmin0(fmat)
        cen, cw = _wk_centroids(point, cluster, weight, K)
        f, energy = _wk_energy(point, weight, cen, cw, cluster)
        new = energy.sum()
        if abs(new - old) < 1e-6:
            break
        old = new
        it += 1
        energies.append(new)
    return cluster, cen, np.array(energies)


def kmeans_pp(X: np.ndarray, k: int, rng: np.random.Generator, max_iter: int = 100) -> np.ndarray:
    """Stand-in for MATLAB's kmeans(X, k, 'Replicates', 1) (Statistics Toolbox, absent):
    k-means++ seeding from ``rng``, then batch (Lloyd) updates, an emptied cluster
    re-seeded with the point farthest from its centre ('singleton').  Its draws are not
    MATLAB's twister stream, so the centres are not the reference's: parity unpinned."""
    X = np.asarray(X, dtype=float)
    n = X.shape[0]
    cen = np.empty((k, X.shape[1]))
    cen[0] = X[rng.integers(n)]
    d2 = ((X - cen[0]) ** 2).sum(1)
    for c in range(1, k):
        tot = d2.sum()
        i = rng.choice(n, p=d2 / tot) if tot > 0 else rng.integers(n)
        cen[c] = X[i]
        d2 = np.minimum(d2, ((X - cen[c]) ** 2).sum(1))
    lab = None
    for _ in range(max_iter):
        dist = ((X[None, :, :] - cen[:, None, :]) ** 2).sum(2)
        new = np.argmin(dist, axis=0)
        if lab is not None and np.array_equal(new, lab):
            break
        lab = new
        for c in range(k):
            mem = lab == c
            if mem.any():
                cen[c] = X[mem].mean(0)
            else:
                far = int(np.argmax(dist[lab, np.arange(n)]))
                cen[c] = X[far]
                lab[far] = c
    return cen


def wtkmeans_points(base: BaseSet, mode: str = "r0"):
    """vbhemhmm_init.m:296-323: every base state's mean [n][d] and its normalised
    weight [n] (makeGMMweights of its HMM), plus the first base state's covariance."""
    bn = base.numpy()
    ns = bn["nstates"]
    pts, w = [], []
    for i in range(base.N):
        m = int(ns[i])
        pts.append(bn["centres"][i, :m])
        w.append(make_gmm_weights(bn["prior"][i, :m], bn["A"][i, :m, :m], mode))
    wv = np.concatenate(w)
    return np.concatenate(pts, 0), wv / wv.sum(), bn["covars"][0, 0]


def wtkmeans_init(base: BaseSet, opt: dict, wtseed: int, points=None) -> Posterior:
    """'wtkmeans' initialisation (vbhemhmm_init.m:294-425, initopt.mode 'r0' by default,
    ``points`` = :func:`wtkmeans_points` computed once for all trials;
    vbhem_h3m_cluster.m:213-221): every base state's mean, weighted by its HMM's
    50-step state distribution (makeGMMweights), is clustered into K groups (k-means
    seed, then my_weighted_kmeans); each group's means into S state centres (k-means, or
    the means themselves padded with the first when there are at most S); random prior /
    A per cluster (makeAprior 'r'); counts NJ = (Nv Kb) Kb / K as the reference computes
    them (:386).  MATLAB's kmeans and twister draws are replaced by :func:`kmeans_pp` on
    numpy generators seeded with wtseed and wtseed + 1 (vbhem_h3m_c.m:53 sets wtseed =
    seed + trial): parity of the centres is unpinned, the construction around them
    follows the reference."""
    opt = clip_hyps(opt)
    mode = opt.get("initopt_mode", "r0")
    K, S = opt["K"], opt["S"]
    Kb, d = base.N, base.d
    mumtx, alpha_w, c11 = points if points is not None else wtkmeans_points(base, mode)
    g1 = np.random.Generator(np.random.PCG64(wtseed))
    init_c = kmeans_pp(mumtx, K, g1)
    cluster, _, _ = weighted_kmeans(K, 100, mumtx, alpha_w, init_c)
    centres = [None] * K
    g2 = g1
    for i in range(K):
        mi = mumtx[cluster == i]
        if mi.shape[0] == 0:
            continue
        if mi.shape[0] <= S:
            centres[i] = np.concatenate([mi, np.repeat(mi[:1], S - mi.shape[0], 0)], 0)
        else:
            g2 = np.random.Generator(np.random.PCG64(wtseed + 1))
            centres[i] = kmeans_pp(mi, S, g2)
    first = next(i for i in range(K) if centres[i] is not None)
    centres = [c if c is not None else centres[first] for c in centres]
    Nv = opt["Nv"] * Kb
    NJ = Nv * Kb / K
    nsj = NJ / S
    eta = np.empty((K, S))
    eps = np.empty((K, S, S))
    for j in range(K):
        prior, A = make_a_prior(S, mode, g2)
        eta[j] = prior * NJ + opt["eta0"]
        eps[j] = A * NJ + opt["epsilon0"]
    v = np.full((K, S), opt["v0"] + nsj + 1)
    lam = np.full((K, S), opt["lambda0"] + nsj)
    if base.covmode == COV_DIAG:
        W = np.broadcast_to(1.0 / ((opt["v0"] + nsj + 1 - d - 1) * c11), (K, S, d)).copy()
    else:
        W = np.broadcast_to(np.linalg.inv((opt["v0"] + nsj + 1 - d - 1) * c11), (K, S, d, d)).copy()
    alpha = opt["alpha0"] + NJ * np.ones(K)
    return Posterior(alpha=alpha, eta=eta, epsilon=eps, lam=lam, v=v, m=np.stack(centres), W=W,
                     W0mode="iid" if np.size(opt["W0"]) == 1 else "diag")


# ----------------------------------------------------------------------------
# 'gmmNew' initialisation (vbhemhmm_init.m:103-293, GMM_MixHierEM.m, naiveWordMix.m)
# ----------------------------------------------------------------------------
def gmm_mix_hier_em(centres: np.ndarray, covars: np.ndarray, full: bool, T: int,
                    virtual_samples: float, iterations: int, rng: np.random.Generator,
                    init_centres: Optional[np.ndarray] = None):
    """GMM_MixHierEM.m: the mixture of all base Gaussians (naiveWordMix: equal priors)
    reduced to T components by hierarchical EM with ``virtual_samples`` virtual samples;
    returns (priors [T], centres [T][d], covars [T][d][d] | [T][d], log-posteriors
    [T][n]).  The initial centres come from :func:`kmeans_pp` (the reference's arKmeans
    with its anchors start): parity of the result unpinned."""
    X = np.asarray(centres, dtype=float)
    C = np.asarray(covars, dtype=float)
    n, dim = X.shape
    prior = np.full(n, 1.0 / n)
    if T == 1:
        # (:60-73: second moments about the origin, as the reference computes them)
        cov = (prior[:, None, None] * (X[:, :, None] * X[:, None, :] + C)).sum(0) if full \
            else (prior[:, None] * (X ** 2 + C)).sum(0)
        return np.ones(1), (prior @ X)[None, :], cov[None], np.zeros((1, n))
    rng.random((T, n))                                   # (:91 post = rand(T, n): overwritten)
    cent = kmeans_pp(X, T, rng) if init_centres is None else np.array(init_centres, dtype=float)
    vr = np.repeat(C.mean(0)[None], T, 0) if full else np.repeat(C.max(0)[None], T, 0)
    mxwt = np.full(T, 1.0 / T)
    coef = -(dim / 2.0) * np.log(2 * np.pi)
    dpp = prior * virtual_samples
    last = -np.finfo(float).max
    logpost = np.zeros((T, n))
    for _ in range(int(iterations)):
        with np.errstate(divide="ignore", invalid="ignore"):
            if full:
                ivr = np.linalg.inv(vr)
                trc = np.einsum("tab,nab->tn", ivr, C)
                ld = np.log(np.linalg.det(vr))
                diff = cent[:, None, :] - X[None, :, :]
                quad = np.einsum("tna,tab,tnb->tn", diff, ivr, diff)
                xpt = np.log(mxwt)[:, None] + dpp[None, :] * (coef - 0.5 * (trc + quad + ld[:, None]))
            else:
                ivr = 1.0 / vr                                   # [T][d]
                trc = ivr @ C.T
                nrm = (cent * cent * ivr + np.log(vr)).sum(1)
                xpt = np.log(mxwt)[:, None] + dpp[None, :] * (
                    coef - 0.5 * (ivr @ (X * X).T - 2 * (cent * ivr) @ X.T + nrm[:, None] + trc))
            mv = xpt.max(0)
            lx = mv + np.log(np.exp(xpt - mv).sum(0))
            logpost = xpt - lx
            post = np.exp(logpost)
        logp = lx.mean()
        if not np.isfinite(logp) or logp - last < 1e-6:   # (:129-141: stop, keep the last update)
            break
        last = logp
        mxwt = post.mean(1)
        wts = post * prior[None, :]
        wts = wts / wts.sum(1, keepdims=True)
        cent = wts @ X
        for c in range(T):
            dx = X - cent[c]
            if full:
                vr[c] = np.einsum("n,nab->ab", wts[c], dx[:, :, None] * dx[:, None, :] + C)
            else:
                vr[c] = wts[c] @ (dx ** 2 + C)
    return mxwt, cent, vr, logpost


def gmmnew_init(base: BaseSet, opt: dict, seed: int, points=None) -> Posterior:
    """'gmmNew' initialisation (vbhemhmm_init.m:103-293, initopt.mode 'r0' by default):
    the base states' Gaussians reduced to S components (:func:`gmm_mix_hier_em`, Nv Kb
    virtual samples, initopt.iter = 30 iterations) shared by every cluster's states;
    random prior / A per cluster (makeAprior) and random cluster weights omega, counts
    Nsj = omega Nv Kb (:262-291).  ``points`` = (centres, covars) of all base states.
    Draws from one numpy generator seeded with ``seed`` (MATLAB's twister stream in the
    reference): parity unpinned."""
    opt = clip_hyps(opt)
    mode = opt.get("initopt_mode", "r0")
    if "m" in mode:
        raise ValueError("initopt.mode 'm' (priors from the base HMMs) is not supported for gmmNew")
    K, S = opt["K"], opt["S"]
    Kb, d = base.N, base.d
    full = base.covmode == COV_FULL
    if points is None:
        bn = base.numpy()
        ns = bn["nstates"]
        points = (np.concatenate([bn["centres"][i, :int(ns[i])] for i in range(Kb)]),
                  np.concatenate([bn["covars"][i, :int(ns[i])] for i in range(Kb)]))
    rng = np.random.Generator(np.random.PCG64(seed))
    Nv = opt["Nv"] * Kb
    _, cen, cov, _ = gmm_mix_hier_em(points[0], points[1], full, S, Nv,
                                     int(opt.get("initopt_iter", 30)), rng)
    rng.random((K, S))                                   # (:249-250 the emissions' priors)
    pa = [make_a_prior(S, mode, rng) for _ in range(K)]
    omega = rng.random(K)
    omega = omega / omega.sum()
    Nsj = omega * Nv
    eta = np.stack([pa[j][0] * Nsj[j] + opt["eta0"] for j in range(K)])
    eps = np.stack([pa[j][1] * Nsj[j] + opt["epsilon0"] for j in range(K)])
    v = opt["v0"] + Nsj[:, None] / S + 1 + np.zeros((K, S))
    lam = opt["lambda0"] + Nsj[:, None] / S + np.zeros((K, S))
    m = np.repeat(cen[None], K, 0)
    if full:
        W = np.linalg.inv((v - d - 1)[:, :, None, None] * cov[None])
    else:
        W = 1.0 / ((v - d - 1)[:, :, None] * cov[None])
    return Posterior(alpha=opt["alpha0"] + Nsj, eta=eta, epsilon=eps, lam=lam, v=v, m=m, W=W,
                     W0mode="iid" if np.size(opt["W0"]) == 1 else "diag")


# ----------------------------------------------------------------------------
# synthetic workloads
# ----------------------------------------------------------------------------
CONFIGS = {
    # name: (N, K, S, Sb, d, covmode, tau, Nv, option overrides)
    "C2": dict(N=100, K=4, S=3, Sb=2, d=2, covmode=COV_FULL, tau=50, Nv=100,
               opt=dict(alpha0=1e6, eta0=1.0, epsilon0=1.0, lambda0=1.0, v0=5.0, W0=1.0,
                        m0=[1.5, 1.5])),
    "C3": dict(N=10_000, K=8, S=5, Sb=5, d=2, covmode=COV_DIAG, tau=10, Nv=100, opt={}),
    # v0 must exceed d-1 (vbhem_h3m_cluster.m:233); the default 5 only suits d <= 5
    "C4": dict(N=100_000, K=16, S=8, Sb=8, d=8, covmode=COV_FULL, tau=10, Nv=100, opt=dict(v0=10.0)),
    "C5": dict(N=1_000_000, K=32, S=12, Sb=12, d=16, covmode=COV_FULL, tau=10, Nv=100,
               opt=dict(v0=18.0)),
}


def _digamma(x: torch.Tensor) -> torch.Tensor:
    return torch.special.digamma(x)


def synth_base_set(N: int, K: int, Sb: int, d: int, covmode: int, seed: int,
                   device="cpu", exprmt1: bool = False, ragged: bool = False,
                   n_total: Optional[int] = None, i_offset: int = 0,
                   face: bool = False) -> BaseSet:
    """Synthetic h3m_b built directly in packed form (use_post=1 semantics).

    Ground truth: K HMMs, base i is a noisy copy of GT g = i mod K: means
    U[0,5]^d + N(0,0.1^2) per base, covariance L L'/d + 0.5 I (full) or
    U[0.5,1.5] (diag), prior and A rows ~ Dirichlet(1); VB counts
    alpha = 1+25*pi, epsilon = 1+250*A, beta = 1+250/Sb, then the
    hmms_to_h3m_hem(use_post=1) transform.  exprmt1=True uses the two GT HMMs
    of Synthetic_experiment/exprmt1_sampledata.m:20-43 instead (Sb=d=2).
    face=True draws eye-fixation-scale emissions (demo/vbdemo_face.m: screen
    pixels): GT means [256, 192, 150, ...][:d] + U[-60, 60]^d, per-base mean
    noise N(0, 5^2), covariances 900 (L L'/d + 0.5 I) (about 30 px spread).
    ragged=True draws per-base state counts in [1, Sb] (zero-padded).
    Generated on ``device``; ``n_total``/``i_offset`` place this block of N
    bases inside a larger set (omega = 1/n_total, GT index (i_offset+i) mod K)."""
    device = torch.device(device)
    gcpu = torch.Generator(device="cpu").manual_seed(int(seed))
    g = torch.Generator(device=device).manual_seed(int(seed) + 1)
    dt = torch.float64
    n_total = N if n_total is None else int(n_total)
    if exprmt1:
        G = 2
        gt_prior = torch.tensor([[0.5, 0.5], [0.5, 0.5]], dtype=dt)
        gt_A = torch.tensor([[[0.6, 0.4], [0.4, 0.6]], [[0.4, 0.6], [0.6, 0.4]]], dtype=dt)
        gt_mu = torch.tensor([[[0.0, 0.0], [3.0, 3.0]]] * 2, dtype=dt)
        eye = torch.eye(2, dtype=dt)
        gt_cov = eye.expand(G, 2, 2, 2).clone() if covmode == COV_FULL else torch.ones(G, 2, 2, dtype=dt)
    else:
        G = K
        gt_prior = _dirichlet(gcpu, (G,), Sb)
        gt_A = _dirichlet(gcpu, (G, Sb), Sb)
        gt_mu = torch.rand((G, Sb, d), generator=gcpu, dtype=dt) * 5.0
        if covmode == COV_FULL:
            Lm = torch.randn((G, Sb, d, d), generator=gcpu, dtype=dt)
            gt_cov = Lm @ Lm.transpose(-1, -2) / d + 0.5 * torch.eye(d, dtype=dt)
        else:
            gt_cov = 0.5 + torch.rand((G, Sb, d), generator=gcpu, dtype=dt)
        if face:
            centre = torch.tensor(([256.0, 192.0, 150.0] + [128.0] * d)[:d], dtype=dt)
            gt_mu = centre + (gt_mu / 5.0 - 0.5) * 120.0
            gt_cov = 900.0 * gt_cov
    gt_prior, gt_A, gt_mu, gt_cov = (x.to(device) for x in (gt_prior, gt_A, gt_mu, gt_cov))
    gi = (torch.arange(N, device=device) + int(i_offset)) % G
    alpha = 1.0 + 25.0 * gt_prior[gi]
    eps = 1.0 + 250.0 * gt_A[gi]
    beta = 1.0 + 250.0 / Sb
    prior = torch.exp(_digamma(alpha) - _digamma(alpha.sum(-1, keepdim=True)))
    A = torch.exp(_digamma(eps) - _digamma(eps.sum(-1, keepdim=True)))
    noise = 5.0 if face else 0.1
    centres = gt_mu[gi] + noise * torch.randn((N, Sb, d), generator=g, dtype=dt, device=device)
    covars = ((beta + 1.0) / beta) * gt_cov[gi]
    nstates = torch.full((N,), Sb, dtype=torch.int32, device=device)
    if ragged and Sb > 1:
        nstates = torch.randint(1, Sb + 1, (N,), generator=g, dtype=torch.int32, device=device)
        mask = torch.arange(Sb, device=device)[None, :] < nstates[:, None].long()
        prior = prior * mask
        A = A * mask[:, :, None] * mask[:, None, :]
        centres = centres * mask[:, :, None]
        if covmode == COV_FULL:
            covars = torch.where(mask[:, :, None, None], covars,
                                 torch.eye(d, dtype=dt, device=device).expand_as(covars))
        else:
            covars = torch.where(mask[:, :, None], covars, torch.ones_like(covars))
    omega = torch.full((N,), 1.0 / n_total, dtype=dt, device=device)
    return BaseSet(nstates, prior.contiguous(), A.contiguous(), centres.contiguous(),
                   covars.contiguous(), omega, covmode)


def _dirichlet(g: torch.Generator, batch, n: int) -> torch.Tensor:
    # Dirichlet(1) = normalised Exp(1) draws
    e = -torch.log(torch.rand(tuple(batch) + (n,), generator=g, dtype=torch.float64).clamp_min(1e-300))
    return e / e.sum(-1, keepdim=True)


def synth_workload(name: str, seed: Optional[int] = None, device="cpu", N: Optional[int] = None,
                   shard: Optional[tuple] = None, ragged: bool = False):
    """(BaseSet, Posterior, options) for a named config; seed = 1001 + index
    (BASELINE.md).  ``N`` overrides the number of base HMMs (sub-sampling).
    ``shard=(lo, hi)`` generates only bases [lo, hi) of the N (seeded per
    shard); the Posterior is identical for every shard (baseem over the first
    min(N, 4096) bases of shard 0's seed)."""
    cfg = CONFIGS[name]
    idx = list(CONFIGS).index(name) + 1
    seed = 1001 + idx if seed is None else seed
    n = cfg["N"] if N is None else N
    lo, hi = (0, n) if shard is None else shard
    args = (cfg["K"], cfg["Sb"], cfg["d"], cfg["covmode"])
    ex = name == "C2"
    base = synth_base_set(hi - lo, *args, seed + 7919 * lo, device=device, exprmt1=ex,
                          ragged=ragged, n_total=n, i_offset=lo)
    opt = default_options(cfg["K"], cfg["S"], cfg["d"], tau=cfg["tau"], Nv=cfg["Nv"],
                          covmode=cfg["covmode"], **cfg["opt"])
    if shard is None and n <= 4096:
        init = base
    else:
        # every shard (and the unsharded large case) draws the initial clusters from the
        # same standalone first-4096-bases set, so all ranks hold identical posteriors
        init = synth_base_set(min(n, 4096), *args, seed, device=device, exprmt1=ex, ragged=ragged,
                              n_total=n)
    rb, rg, om = baseem_draws(init, cfg["K"], cfg["S"], seed)
    post = baseem_init(init, opt, rb, rg, om, n_total=n)
    return base, post, opt

"""VBHEM-H3M EM loop around the device E-step.

:func:`vbhem_h3m_c_step_fc` mirrors src/vbhem/vbhem_h3m_c_step_fc.m:1-449:
per iteration the psi prelude (:118-165), the E-step (:168-198) fused with the
responsibilities (:270-283) and the statistics reduction
(vbhem_compute_Statistics.m), the lower bound (:296, vbhemh3m_lb.m), the
convergence test (:311-354) and the M-step (:396-419); then
form_outputH3M.m.  With ``allreduce`` set, each rank runs the E-step on its
shard of base HMMs and the packed statistics are summed across ranks once per
iteration (the only collective); the host math is replicated on every rank.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional

import numpy as np
import torch

from . import host
from .estep import EStepEngine
from .h3m import Posterior


@dataclasses.dataclass
class EMResult:
    post: Posterior                 # h3m_r variational posteriors after the last M-step
    LogLs: List[float]              # h3m_r.LogLs (ELBO per iteration, before its M-step)
    LL: float                       # final lower bound (-inf if unstable)
    iters: int
    stable: bool
    hatZ: torch.Tensor              # [N_shard, K] responsibilities of the last E-step
    L_elbo: torch.Tensor            # [N_shard, K]
    Nj: np.ndarray                  # [K]
    syn: Optional[dict]             # Syn_STATS of the last M-step (Nj_rho1, Nj_rho2rho, Nj_rho, ...)
    point: Optional[dict] = None    # convert_h3mrtoh3mb point estimates
    label: Optional[torch.Tensor] = None  # argmax_j hat_Z (0-based), form_outputH3M.m:274-275
    dLL: Optional[dict] = None      # opt['calc_LLderiv']: bound derivatives at the last E-step
    iter_seconds: Optional[np.ndarray] = None  # native_em.run(timestamps=True): per-iteration clock


def tilde_n(engine: EStepEngine, Nv: float, total_N: int) -> torch.Tensor:
    """tilde_N_k = Nv * Kb * omega (step_fc.m:26-30) for the engine's shard;
    omega is the global normalised weight vector sliced to the shard."""
    return (float(Nv) * float(total_N)) * engine.base.omega.to(torch.float64)


def fused_stats_host(engine: EStepEngine, tN: torch.Tensor,
                     allreduce: Optional[Callable[[torch.Tensor], None]]) -> np.ndarray:
    """One fused E-step; its packed statistics on the host for the M-step.
    Single process: the statistics kernel writes them straight into a pinned
    host buffer (no copy after the E-step).  Sharded: device vector, all-reduce,
    then a copy."""
    if allreduce is None and isinstance(engine, EStepEngine):
        buf = getattr(engine, "_em_host_stats", None)
        if buf is None:
            buf = engine._em_host_stats = engine.host_stats_buffer()
        engine.fused(tN, out=buf)
        torch.cuda.current_stream(engine.device).synchronize()
        return buf.numpy().copy()
    stats = engine.fused(tN)
    if allreduce is not None:
        allreduce(stats)
    return stats.cpu().numpy()


def vbhem_h3m_c_step_fc(post: Posterior, engine: EStepEngine, opt: dict, *,
                        total_N: Optional[int] = None,
                        allreduce: Optional[Callable[[torch.Tensor], None]] = None,
                        max_iter: Optional[int] = None) -> EMResult:
    covmode = engine.base.covmode
    K, S, d = post.m.shape
    total_N = engine.N if total_N is None else int(total_N)
    tN = tilde_n(engine, opt["Nv"], total_N)
    maxIter = opt["max_iter"] if max_iter is None else max_iter
    minDiff = opt["minDiff"]
    post = post.copy()
    lastL = -np.finfo(float).max
    it = 0
    LogLs: List[float] = []
    syn = None
    stable = True
    L = -np.inf
    Nj = np.zeros(K)
    dLL = None
    do_deriv = bool(opt.get("calc_LLderiv", 0))
    while True:
        consts = host.cluster_constants(post, covmode)
        logOmega = host.log_omega_tilde(post.alpha)
        engine.set_clusters(consts)
        engine.set_log_omega(logOmega)
        st = host.unpack_stats(fused_stats_host(engine, tN, allreduce), K, S, d, covmode)
        Nj = st["Nj"] + 1e-50
        L = host.lower_bound(st["Lt1"], st["Lt7"], Nj, logOmega, post, consts, opt, covmode)
        do_break = False
        if it > 1 and abs((L - lastL) / lastL) <= minDiff:
            do_break = True
        if it == maxIter:
            do_break = True
        if np.isnan(L):
            # step_fc.m:338-374: unstable model -> L = -inf, stop before the M-step
            L = -np.inf
            stable = False
            if do_deriv:  # the gradient is invalidated (:362-368)
                dLL = {k: np.full_like(np.atleast_1d(v), np.nan)
                       for k, v in host.lower_bound_derivs(logOmega, post, consts, opt, covmode,
                                                           opt.get("hyp_clipped")).items()
                       if k != "raw"}
            break
        if do_break and do_deriv:
            # step_fc.m:356-360: derivatives before the last M-step (vbhemh3m_lb.m:202-356)
            dLL = host.lower_bound_derivs(logOmega, post, consts, opt, covmode,
                                          opt.get("hyp_clipped"))
        syn = host.finish_statistics(st, covmode)
        post = host.mstep(syn, Nj, opt, covmode, post.W0mode)
        it += 1
        LogLs.append(L)
        lastL = L
        if do_break:
            break
    res = EMResult(post=post, LogLs=LogLs, LL=L, iters=it, stable=stable, hatZ=engine.hatZ.clone(),
                   L_elbo=engine.LL.clone(), Nj=Nj, syn=syn, dLL=dLL)
    if stable:
        res.point = host.convert_to_point(post, covmode)
        res.label = torch.argmax(res.hatZ, dim=1)
    return res


def _stack_constants(all_consts: List[dict]) -> dict:
    """Trial-major concatenation of per-trial cluster constants (R x K -> R*K)."""
    return {k: np.concatenate([np.asarray(c[k]) for c in all_consts], axis=0)
            for k in ("logA", "logPi", "m", "P", "c")}


@dataclasses.dataclass
class TrialsResult:
    results: List[EMResult]         # one per trial (vbhem_h3m_c.m: h3m_news)
    LLall: np.ndarray               # [R] final lower bound per trial (LLall)
    best: int                       # argmax LLall (vbhem_h3m_c.m:167-170)


def vbhem_h3m_c_trials(posts: List[Posterior], engine: EStepEngine, opt: dict, *,
                       total_N: Optional[int] = None,
                       allreduce: Optional[Callable[[torch.Tensor], None]] = None,
                       max_iter: Optional[int] = None) -> TrialsResult:
    """R EM trials from their own initial posteriors (vbhem_h3m_c.m:28-67,
    `parfor it = 1:numits`), run in lockstep with one batched E-step launch per
    iteration (vbhem_estep_fused_trials).  Every trial follows
    :func:`vbhem_h3m_c_step_fc` exactly; a trial that has stopped keeps its
    final state (its clusters still ride along in the launch, their outputs
    unused).  The best trial is the one with the largest final bound."""
    R = len(posts)
    if engine.trials != R:
        raise ValueError("engine.trials must equal len(posts)")
    covmode = engine.base.covmode
    K, S, d = posts[0].m.shape
    total_N = engine.N if total_N is None else int(total_N)
    tN = tilde_n(engine, opt["Nv"], total_N)
    maxIter = opt["max_iter"] if max_iter is None else max_iter
    minDiff = opt["minDiff"]
    SL = host.stats_len(K, S, d, covmode)
    post = [p.copy() for p in posts]
    lastL = [-np.finfo(float).max] * R
    it = [0] * R
    LogLs: List[List[float]] = [[] for _ in range(R)]
    syn: List[Optional[dict]] = [None] * R
    stable = [True] * R
    L = [-np.inf] * R
    Nj = [np.zeros(K) for _ in range(R)]
    done = [False] * R
    hatZ: List[Optional[torch.Tensor]] = [None] * R
    Lel: List[Optional[torch.Tensor]] = [None] * R
    consts = [host.cluster_constants(p, covmode) for p in post]
    logOm = [host.log_omega_tilde(p.alpha) for p in post]
    while not all(done):
        engine.set_clusters(_stack_constants(consts))
        engine.set_log_omega(np.concatenate(logOm))
        vec = fused_stats_host(engine, tN, allreduce)
        for r in range(R):
            if done[r]:
                continue
            st = host.unpack_stats(vec[r * SL:(r + 1) * SL], K, S, d, covmode)
            Nj[r] = st["Nj"] + 1e-50
            Lr = host.lower_bound(st["Lt1"], st["Lt7"], Nj[r], logOm[r], post[r], consts[r], opt,
                                  covmode)
            stop = (it[r] > 1 and abs((Lr - lastL[r]) / lastL[r]) <= minDiff) or it[r] == maxIter
            if np.isnan(Lr):  # step_fc.m:338-374
                L[r] = -np.inf
                stable[r] = False
                stop = True
            else:
                L[r] = Lr
                syn[r] = host.finish_statistics(st, covmode)
                post[r] = host.mstep(syn[r], Nj[r], opt, covmode, post[r].W0mode)
                it[r] += 1
                LogLs[r].append(Lr)
                lastL[r] = Lr
            if stop:
                done[r] = True
                cols = slice(r * K, (r + 1) * K)
                hatZ[r] = engine.hatZ[:, cols].clone()
                Lel[r] = engine.LL[:, cols].clone()
            else:
                consts[r] = host.cluster_constants(post[r], covmode)
                logOm[r] = host.log_omega_tilde(post[r].alpha)
    results = []
    for r in range(R):
        res = EMResult(post=post[r], LogLs=LogLs[r], LL=L[r], iters=it[r], stable=stable[r],
                       hatZ=hatZ[r], L_elbo=Lel[r], Nj=Nj[r], syn=syn[r])
        if stable[r]:
            res.point = host.convert_to_point(post[r], covmode)
            res.label = torch.argmax(res.hatZ, dim=1)
        results.append(res)
    LLall = np.array([x.LL for x in results])
    return TrialsResult(results=results, LLall=LLall, best=int(np.argmax(LLall)))

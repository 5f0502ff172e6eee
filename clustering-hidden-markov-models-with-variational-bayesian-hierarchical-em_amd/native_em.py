"""The EM loop in C++ (include/vbhem_em.h).

:func:`run` drives ``vbhem_em_run``: the whole of vbhem_h3m_c_step_fc.m:1-449
(psi prelude, fused device E-step, lower bound, convergence test, M-step) runs
in the library; Python only allocates the device buffers and, with several
ranks, supplies the all-reduce of the packed statistics as a callback.  The
host steps are also exposed one by one (:func:`prelude`, :func:`mstep`,
:func:`lower_bound`) and as one call (:class:`HostIteration`), and are checked
against :mod:`vbhem_amd.host`.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import numpy as np
import torch

from . import _capi
from .em import EMResult
from .estep import EStepEngine
from .h3m import COV_FULL, Posterior


class _PostBuf:
    """Contiguous float64 host copies of a Posterior plus its vbhem_post_t view."""

    def __init__(self, post: Posterior, covmode: int):
        self.a = {k: np.ascontiguousarray(getattr(post, k), dtype=np.float64).copy()
                  for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W")}
        K, S, d = self.a["m"].shape
        self.W0mode = post.W0mode
        p = {k: self.a[k].ctypes.data for k in self.a}
        self.t = _capi.PostT(K, S, d, covmode, p["alpha"], p["eta"], p["epsilon"], p["lam"],
                             p["v"], p["m"], p["W"])

    def posterior(self) -> Posterior:
        return Posterior(W0mode=self.W0mode, **{k: v.copy() for k, v in self.a.items()})


class _OptBuf:
    def __init__(self, opt: dict):
        self.m0 = np.ascontiguousarray(opt["m0"], dtype=np.float64).reshape(-1)
        self.W0 = np.ascontiguousarray(np.array(opt["W0"], dtype=np.float64, ndmin=1))
        self.t = _capi.EmOptT(float(opt["alpha0"]), float(opt["eta0"]), float(opt["epsilon0"]),
                              float(opt["lambda0"]), float(opt["v0"]), self.m0.ctypes.data,
                              self.W0.ctypes.data, int(self.W0.size), float(opt["Nv"]),
                              int(opt["max_iter"]), float(opt["minDiff"]))


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def prelude(post: Posterior, covmode: int) -> dict:
    """vbhem_em_prelude: the E-step constants + logOmega (cf. host.cluster_constants)."""
    pb = _PostBuf(post, covmode)
    K, S, d = post.m.shape
    out = dict(logA=np.zeros((K, S, S)), logPi=np.zeros((K, S)), m=np.zeros((K, S, d)),
               P=np.zeros((K, S, d, d) if covmode == COV_FULL else (K, S, d)), c=np.zeros((K, S)),
               logLambdaTilde=np.zeros((K, S)), logOmega=np.zeros(K))
    _capi.check(_capi.lib().vbhem_em_prelude(ctypes.byref(pb.t), *(_p(out[k]) for k in (
        "logA", "logPi", "m", "P", "c", "logLambdaTilde", "logOmega"))), "vbhem_em_prelude")
    return out


def mstep(stats: np.ndarray, post: Posterior, opt: dict, covmode: int) -> Posterior:
    """vbhem_em_mstep on a packed statistics vector (cf. host.finish_statistics + mstep)."""
    pb, ob = _PostBuf(post, covmode), _OptBuf(opt)
    st = np.ascontiguousarray(stats, dtype=np.float64)
    _capi.check(_capi.lib().vbhem_em_mstep(ctypes.byref(ob.t), _p(st), ctypes.byref(pb.t)),
                "vbhem_em_mstep")
    return pb.posterior()


def lower_bound(stats: np.ndarray, post: Posterior, opt: dict, covmode: int, consts: dict) -> float:
    """vbhem_em_lower_bound (cf. host.lower_bound)."""
    pb, ob = _PostBuf(post, covmode), _OptBuf(opt)
    st = np.ascontiguousarray(stats, dtype=np.float64)
    c = {k: np.ascontiguousarray(consts[k], dtype=np.float64)
         for k in ("logLambdaTilde", "logA", "logPi", "logOmega")}
    L = ctypes.c_double()
    _capi.check(_capi.lib().vbhem_em_lower_bound(
        ctypes.byref(pb.t), ctypes.byref(ob.t), _p(st), _p(c["logLambdaTilde"]), _p(c["logA"]),
        _p(c["logPi"]), _p(c["logOmega"]), ctypes.byref(L)), "vbhem_em_lower_bound")
    return float(L.value)


class HostIteration:
    """The per-iteration host math of the C++ EM loop (vbhem_em_host_iteration:
    bound, M-step, next prelude) on fixed host buffers, callable repeatedly at
    the cost of one C call (what bench.py times as the EM iteration's host part)."""

    def __init__(self, post: Posterior, opt: dict, covmode: int):
        self.pb, self.ob = _PostBuf(post, covmode), _OptBuf(opt)
        self.pre = prelude(post, covmode)
        self.L = ctypes.c_double()
        self._args = None

    def __call__(self, stats: np.ndarray) -> float:
        st = np.ascontiguousarray(stats, dtype=np.float64)
        if self._args is None or self._args[0] is not st:
            self._args = (st, ctypes.byref(self.ob.t), _p(st), ctypes.byref(self.pb.t)) + tuple(
                _p(self.pre[k]) for k in ("logA", "logPi", "m", "P", "c", "logLambdaTilde",
                                           "logOmega")) + (ctypes.byref(self.L),)
        _capi.check(_capi.lib().vbhem_em_host_iteration(*self._args[1:]), "vbhem_em_host_iteration")
        return float(self.L.value)


def _workspace(engine: EStepEngine, nb: int) -> torch.Tensor:
    """The loop's device workspace, kept on the engine and reused by later runs
    (grown when a run needs more): no allocation on the per-run path."""
    ws = getattr(engine, "_em_ws", None)
    if ws is None or ws.numel() < nb:
        ws = engine._em_ws = torch.empty((nb,), dtype=torch.uint8, device=engine.device)
    return ws


def run(post: Posterior, engine: EStepEngine, opt: dict, *, total_N: Optional[int] = None,
        allreduce: Optional[Callable[[torch.Tensor], None]] = None,
        max_iter: Optional[int] = None, comm=None, timestamps: bool = False,
        calc_deriv: bool = False) -> EMResult:
    """The EM loop in C++ on the engine's base set; same result type as
    :func:`vbhem_amd.em.vbhem_h3m_c_step_fc`.

    comm:       a :class:`vbhem_amd.dist.RcclComm`: the loop all-reduces the packed
                statistics with RCCL on its own stream (no callback); exclusive
                with ``allreduce`` (a Python hook the loop calls once per E-step).
    timestamps: ``res.iter_seconds`` = the host clock at which each iteration's
                bound reached the host (the loop's own per-iteration timing).
    calc_deriv: ``res.dLL`` = the bound derivatives of the last accepted iteration
                (vbhemh3m_lb.m:202-356, before its M-step; computed by the C++
                loop), in the form of :func:`vbhem_amd.em.vbhem_h3m_c_step_fc`'s
                (``opt["hyp_clipped"]`` applied); NaN when the run is unstable."""
    from .em import tilde_n
    covmode = engine.base.covmode
    total_N = engine.N if total_N is None else int(total_N)
    opt = dict(opt)
    if max_iter is not None:
        opt["max_iter"] = int(max_iter)
    if comm is not None and allreduce is not None:
        raise ValueError("native_em.run: give comm or allreduce, not both")
    pb, ob = _PostBuf(post, covmode), _OptBuf(opt)
    K, S = pb.t.K, pb.t.S
    d = pb.a["m"].shape[2]
    tN = tilde_n(engine, opt["Nv"], total_N).contiguous()
    lib = _capi.lib()
    nb = int(lib.vbhem_em_workspace_bytes(ctypes.byref(engine._bt), K, S, engine.T))
    if nb == 0:
        raise _capi.VbhemError("vbhem_em_workspace_bytes: unsupported shape")
    ws = _workspace(engine, nb)
    LogLs = np.zeros(int(opt["max_iter"]) + 1)
    tsec = np.zeros(int(opt["max_iter"]) + 1) if timestamps else None
    nW = int(ob.W0.size)
    dLL = np.zeros(5 + nW + d) if calc_deriv else None
    iters, L, stable = ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
    stats = engine.stats

    def _ar(ptr, n, stream, ctx):  # the statistics buffer is engine.stats
        try:
            allreduce(stats)
            return 0
        except Exception:  # noqa: BLE001 -- reported as a status code to the C loop
            return 1

    cb = _capi.ALLREDUCE_FN(_ar) if allreduce is not None else _capi.ALLREDUCE_FN()
    ext = _capi.EmExtT(comm.handle if comm is not None else None,
                       _p(tsec) if tsec is not None else None, 1 if calc_deriv else 0,
                       _p(dLL) if dLL is not None else None)
    rc = lib.vbhem_em_run_ext(ctypes.byref(engine._bt), _capi.ptr(tN), engine.T, ctypes.byref(ob.t),
                              ctypes.byref(pb.t), _p(LogLs), ctypes.byref(iters), ctypes.byref(L),
                              ctypes.byref(stable), _capi.ptr(stats), _capi.ptr(engine.hatZ),
                              _capi.ptr(engine.LL), _capi.ptr(ws), ws.numel(), engine._stream(), cb,
                              None, ctypes.byref(ext))
    _capi.check(rc, "vbhem_em_run_ext")
    it = int(iters.value)
    res = EMResult(post=pb.posterior(), LogLs=[float(x) for x in LogLs[:it]], LL=float(L.value),
                   iters=it, stable=bool(stable.value), hatZ=engine.hatZ.clone(),
                   L_elbo=engine.LL.clone(), Nj=None, syn=None)
    if tsec is not None:
        res.iter_seconds = tsec[:max(it, 1) if not res.stable else it].copy()
    if dLL is not None:
        from . import host
        raw = _raw_dict(dLL, nW)
        # as em.vbhem_h3m_c_step_fc: clipped and transformed (step_fc.m:356-360), or
        # NaN when the run ended unstable (:362-368)
        tr = host.transform_derivs(raw, opt, opt.get("hyp_clipped"))
        res.dLL = tr if res.stable else {k: np.full_like(np.atleast_1d(v), np.nan)
                                         for k, v in tr.items() if k != "raw"}
    if res.stable:
        from . import host
        res.point = host.convert_to_point(res.post, covmode)
        res.label = torch.argmax(res.hatZ, dim=1)
    return res


def _raw_dict(g: np.ndarray, nW: int) -> dict:
    return {"alpha0": g[0:1].copy(), "eta0": g[1:2].copy(), "epsilon0": g[2:3].copy(),
            "v0": g[3:4].copy(), "lambda0": g[4:5].copy(), "W0": g[5:5 + nW].copy(),
            "m0": g[5 + nW:].copy()}


def lower_bound_derivs(post: Posterior, opt: dict, covmode: int) -> dict:
    """vbhem_em_lower_bound_derivs at a posterior (its prelude computed in C++):
    the raw derivatives, keyed as host.lower_bound_derivs(...)["raw"]."""
    pb, ob = _PostBuf(post, covmode), _OptBuf(opt)
    pre = prelude(post, covmode)
    d = pb.a["m"].shape[2]
    nW = int(ob.W0.size)
    g = np.zeros(5 + nW + d)
    _capi.check(_capi.lib().vbhem_em_lower_bound_derivs(
        ctypes.byref(pb.t), ctypes.byref(ob.t), _p(pre["logLambdaTilde"]), _p(pre["logA"]),
        _p(pre["logPi"]), _p(pre["logOmega"]), _p(g)), "vbhem_em_lower_bound_derivs")
    return _raw_dict(g, nW)

"""Hyperparameter learning for VBHEM.

* :func:`vbhem_h3m_c_hyp` -- src/vbhem/vbhem_h3m_c_hyp.m:1-63: maximise the
  lower bound over (transformed) hyperparameters with L-BFGS, where every
  function evaluation is a whole EM run (``vbh3m_grad``, :99-125) started from
  the trial's own posterior ('inith3m', vbhemhmm_init.m:428-455) with
  ``calc_LLderiv`` on, so the gradient is vbhemh3m_lb.m:202-356 at its last
  E-step (host.lower_bound_derivs); then one final EM run with the optimum.
* :func:`hypinfo` -- vbhem_get_hypinfo.m (names, transforms, derivative keys).
* :func:`minimize` -- src/util/minimize_new.m: the LBFGS / BFGS / CG direction
  methods with the Wolfe-Powell line search (cubic extrapolation and
  interpolation, MFEPLS function evaluations per line search, SIG 0.5, RHO
  SIG/2 ... as that file sets them).

The E-steps of every EM run go through the fused device E-step; nothing here
touches the per-pair arithmetic.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, List, Optional

import numpy as np

from . import em
from .estep import EStepEngine
from .h3m import BaseSet, Posterior, clip_hyps

ALL_HYPS = ("alpha0", "eta0", "epsilon0", "v0", "lambda0", "W0", "m0")


@dataclasses.dataclass
class HypInfo:
    optname: str
    derivname: str
    trans: Callable                  # optimiser space -> hyperparameter
    invtrans: Callable               # hyperparameter -> optimiser space
    dims: int


def hypinfo(learn_hyps, opt: dict) -> List[HypInfo]:
    """vbhem_get_hypinfo.m:12-96 ('W0' = the sqrt(W0inv) transform)."""
    dim = len(opt["m0"])
    names = ALL_HYPS if (learn_hyps is True or learn_hyps == 1) else tuple(learn_hyps)
    out = []
    for h in names:
        if h in ("alpha0", "eta0", "epsilon0", "lambda0"):
            out.append(HypInfo(h, "d_log" + h, np.exp, np.log, 1))
        elif h == "v0":
            out.append(HypInfo("v0", "d_logv0D1", lambda x: np.exp(x) + dim - 1,
                               lambda x: np.log(x - dim + 1), 1))
        elif h in ("W0", "W0isqrt"):
            out.append(HypInfo("W0", "d_sqrtW0inv", lambda x: x ** (-2.0),
                               lambda x: 1.0 / np.sqrt(x), int(np.size(opt["W0"]))))
        elif h == "W0log":
            out.append(HypInfo("W0", "d_logW0", np.exp, np.log, int(np.size(opt["W0"]))))
        elif h == "m0":
            out.append(HypInfo("m0", "d_m0", lambda x: x, lambda x: x, dim))
        else:
            raise ValueError("bad value of learn_hyp")
    return out


def init_x(opt: dict, info: List[HypInfo]) -> np.ndarray:
    """vbhem_h3m_c_hyp.m init_hyp."""
    return np.concatenate([np.atleast_1d(np.asarray(h.invtrans(np.asarray(opt[h.optname], float)),
                                                    dtype=float)).reshape(-1) for h in info])


def set_opt(X: np.ndarray, opt: dict, info: List[HypInfo]) -> dict:
    """vbhem_h3m_c_hyp.m set_vbopt: optimiser vector -> options."""
    o = dict(opt)
    i = 0
    for h in info:
        val = np.asarray(h.trans(X[i:i + h.dims]), dtype=float)
        o[h.optname] = float(val[0]) if (h.dims == 1 and np.ndim(opt[h.optname]) == 0) else val
        i += h.dims
    o["m0"] = np.asarray(o["m0"], dtype=float).reshape(-1)
    return o


# ----------------------------------------------------------------------------
# minimize_new.m
# ----------------------------------------------------------------------------
def _min_cubic(x, df, s0, s1, extr):
    """minimize_new.m minCubic: minimiser of the approximating cubic."""
    INT, EXT = 0.1, 5.0
    A = -6 * df + 3 * (s0 + s1) * x
    B = 3 * df - (2 * s0 + s1) * x
    with np.errstate(all="ignore"):
        if B < 0:
            z = s0 * x / (s0 - s1)
        else:
            disc = B * B - A * s0 * x
            z = -s0 * x * x / (B + np.sqrt(disc)) if disc >= 0 else np.nan
    if extr:
        if not np.isfinite(z) or z < x or z > x * EXT:
            z = EXT * x
        z = max(z, (1 + INT) * x)
    else:
        if not np.isfinite(z) or z < 0 or z > x:
            z = x / 2
        z = min(max(z, INT * x), (1 - INT) * x)
    return z


class _Wolfe:
    """minimize_new.m wp: Wolfe-Powell conditions set up at the line's start."""

    def __init__(self, p0, SIG, RHO):
        self.a, self.b, self.c = RHO * p0["s"], p0["f"], -SIG * p0["s"]

    def __call__(self, p):
        if p["f"] > self.a * p["x"] + self.b:
            return -1 if self.a > 0 else -2
        if p["s"] < -self.c:
            return 0
        if p["s"] > self.c:
            return 1
        return 2


def _line_search(f, x0, f0, df0, d, s, a, i, P):
    """minimize_new.m lineSearch (p.length > 0): extrapolate until the
    Wolfe-Powell conditions bracket a point, then interpolate; i counts line
    searches and comes back negative when the search failed."""
    LIMIT = P["MFEPLS"]
    p0 = dict(x=0.0, f=f0, df=df0, s=s)
    p1 = dict(p0)
    j = 0
    p3 = dict(p0, x=a)
    wp = _Wolfe(p0, P["SIG"], 0.0)                      # wp(p0, p.SIG, 0)
    while True:                                         # extrapolation
        ok = False
        while not ok and j < LIMIT:
            j += 1
            try:
                fv, dfv = f(x0 + p3["x"] * d)
                dfv = np.asarray(dfv, dtype=float).reshape(-1)
                sv = float(dfv @ d)
                p3.update(f=fv, df=dfv, s=sv)
                ok = True
                if not np.isfinite(fv + sv):
                    raise FloatingPointError("Objective function returned Inf or NaN")
            except Exception:  # noqa: BLE001 -- minimize_new.m:147-155: any error bisects
                p3["x"] = (p1["x"] + p3["x"]) / 2       # bisect and retry
                ok = False
                p3["f"] = np.nan
        if wp(p3) or j >= LIMIT:
            break
        p0, p1 = p1, dict(p3)
        p3 = dict(p3, x=p0["x"] + _min_cubic(p1["x"] - p0["x"], p1["f"] - p0["f"], p0["s"], p1["s"],
                                             True))
    while True:                                         # interpolation
        p2 = dict(p3) if p1["f"] > p3["f"] else dict(p1)
        if wp(p2) > 1 or j >= LIMIT:
            break
        p2["x"] = p1["x"] + _min_cubic(p3["x"] - p1["x"], p3["f"] - p1["f"], p1["s"], p3["s"], False)
        j += 1
        fv, dfv = f(x0 + p2["x"] * d)
        dfv = np.asarray(dfv, dtype=float).reshape(-1)
        p2.update(f=fv, df=dfv, s=float(dfv @ d))
        w = wp(p2)
        if (w > -1 and p2["s"] > 0) or w < -1:
            p3 = p2
        else:
            p1 = p2
    x = x0 + p2["x"] * d
    i = i + 1
    if wp(p2) < 2:
        i = -i
    return x, p2["x"], p2["f"], p2["df"], i


def minimize(X0: np.ndarray, F: Callable, length: int = 100, method: str = "LBFGS",
             MFEPLS: int = 10, MSR: float = 100.0, mem: Optional[int] = None):
    """minimize_new.m (p.length > 0: a budget of line searches).  F(x) -> (f, df).
    Returns (x, f history, line searches used)."""
    with np.errstate(all="ignore"):  # MATLAB arithmetic: 0/0 = NaN, x/0 = Inf, no exceptions
        return _minimize(X0, F, length, method, MFEPLS, np.float64(MSR), mem)


def _minimize(X0, F, length, method, MFEPLS, MSR, mem):
    x0 = np.asarray(X0, dtype=float).reshape(-1)
    fx0, dfx0 = F(x0)
    dfx0 = np.asarray(dfx0, dtype=float).reshape(-1)
    P = dict(MFEPLS=MFEPLS, SIG=0.1 if method in ("CG", "cg") else 0.5)
    fX = [fx0]
    i = 0
    x, dfx = x0, dfx0
    if method in ("LBFGS", "lbfgs"):
        n = x0.size
        m = min(100, n) if mem is None else mem
        k, ok = 0, False
        a = np.zeros(m)
        t = np.zeros((n, m))
        y = np.zeros((n, m))
        rho = np.zeros(m)
        bs = np.float64(-1.0) / MSR
        while i < abs(length):
            q = dfx0.copy()
            jl = None
            for jj in range(k - 1, max(0, k - m) - 1, -1):      # rem(k-1:-1:max(0,k-m), m)
                jl = jj % m
                a[jl] = t[:, jl] @ q / rho[jl]
                q = q - a[jl] * y[:, jl]
            if k == 0:
                r = -q / (q @ q)
            else:
                r = -(t[:, jl] @ y[:, jl]) / (y[:, jl] @ y[:, jl]) * q
            for jj in range(max(0, k - m), k):                  # rem(max(0,k-m):k-1, m)
                jn = jj % m
                r = r - t[:, jn] * (a[jn] + y[:, jn] @ r / rho[jn])
            s = float(r @ dfx0)
            if s >= 0:
                r = -dfx0
                s = float(r @ dfx0)
                k, ok = 0, False
            b = bs / np.fmin(bs, np.float64(s) / MSR) if np.isfinite(s) else np.float64(np.nan)
            if np.all(~np.isfinite(r)):                         # nonsense direction
                i = -i
            else:
                x, b, fx0, dfx, i = _line_search(F, x0, fx0, dfx0, r, s, b, i, P)
            if i < 0:                                           # line search failed
                i = -i
                if ok:
                    ok, k = False, 0
                else:
                    break
            else:
                jn = k % m
                t[:, jn] = x - x0
                y[:, jn] = dfx - dfx0
                rho[jn] = t[:, jn] @ y[:, jn]
                ok = True
                k += 1
                bs = b * s
            x0, dfx0 = x, dfx
            fX.append(fx0)
        return x0, np.array(fX), i
    if method in ("BFGS", "bfgs"):
        r = -dfx0
        s = float(-(r @ r))
        b = -1.0 / (s - 1)
        H = np.eye(x0.size)
        ok = False
        while i < abs(length):
            x, b, fx0, dfx, i = _line_search(F, x0, fx0, dfx0, r, s, b, i, P)
            if i < 0:
                i = -i
                if ok:
                    ok = False
                else:
                    break
            else:
                ok = True
                tt = x - x0
                yy = dfx - dfx0
                ty = tt @ yy
                Hy = H @ yy
                H = H + (ty + yy @ Hy) / ty ** 2 * np.outer(tt, tt) - np.outer(Hy, tt) / ty \
                    - np.outer(tt, Hy) / ty
            r = -H @ dfx
            s = float(r @ dfx)
            x0, dfx0 = x, dfx
            fX.append(fx0)
        return x0, np.array(fX), i
    if method in ("CG", "cg"):
        # minimize_new.m CG: Polack-Ribiere conjugate gradients, slope-ratio step
        ok = False
        r = -dfx0
        s = float(-(r @ r))
        b = -1.0 / (s - 1)
        bs = np.float64(-1.0)
        while i < abs(length):
            b = b * bs / np.fmin(b * s, bs / MSR)
            x, b, fx0, dfx, i = _line_search(F, x0, fx0, dfx0, r, s, b, i, P)
            if i < 0:
                i = -i
                if ok:
                    ok = False
                    r = -dfx
                else:
                    break
            else:
                ok = True
                bs = b * s
                r = float(dfx @ (dfx - dfx0)) / float(dfx0 @ dfx0) * r - dfx
            s = float(r @ dfx)
            if s >= 0:
                r = -dfx
                s = float(r @ dfx)
                ok = False
            x0, dfx0 = x, dfx
            fX.append(fx0)
        return x0, np.array(fX), i
    raise ValueError("method must be LBFGS, BFGS or CG")


# ----------------------------------------------------------------------------
# vbhem_h3m_c_hyp.m
# ----------------------------------------------------------------------------
def vbhem_h3m_c_hyp(base: BaseSet, opt: dict, init_post: Posterior, engine: EStepEngine,
                    length: Optional[int] = None, learn_hyps=None, loop: str = "python") -> dict:
    """Learn the hyperparameters for one trial (vbhem_h3m_c_hyp.m:1-63): L-BFGS
    on -LL over the transformed hyperparameters, each evaluation an EM run from
    ``init_post`` with its bound derivatives, then a final EM run.

    loop: "python" -- the EM runs on :func:`vbhem_amd.em.vbhem_h3m_c_step_fc`;
    "native" -- on the C++ loop (``native_em.run``, vbhem_em_run_ext), which
    computes the derivatives itself (vbhem_em_lower_bound_derivs)."""
    info = hypinfo(opt.get("learn_hyps", 1) if learn_hyps is None else learn_hyps, opt)
    n_eval = [0]
    if loop == "native":
        from . import native_em

        def em_run(post, eng, o):
            return native_em.run(post, eng, o, calc_deriv=bool(o.get("calc_LLderiv", 0)))
    elif loop == "python":
        em_run = em.vbhem_h3m_c_step_fc
    else:
        raise ValueError("loop must be 'python' or 'native'")

    def grad(X):
        o = set_opt(X, opt, info)
        o, flags = clip_hyps(o, with_flags=True)          # vbh3m_grad: vbhem_clip_hyps
        o["hyp_clipped"] = flags
        o["calc_LLderiv"] = 1
        res = em_run(init_post, engine, o)
        n_eval[0] += 1
        L = -res.LL
        dL = np.concatenate([-np.atleast_1d(res.dLL[h.derivname]).reshape(-1) for h in info])
        return L, dL

    X0 = init_x(opt, info)
    methods = {"minimize-lbfgs": "LBFGS", "minimize-bfgs": "BFGS", "minimize-cg": "CG"}
    name = opt.get("minimizer", "minimize-lbfgs")
    if name not in methods:                              # vbhem_h3m_c_hyp.m:51-52
        raise ValueError("bad minimizer specified")
    method = methods[name]
    Xopt, fX, nls = minimize(X0, grad, length=int(length or opt.get("hyp_length", 100)),
                             method=method)
    o2 = set_opt(Xopt, opt, info)
    o2 = clip_hyps(o2)
    final = em_run(init_post, engine, o2)
    return dict(result=final, opt_transhyp=Xopt, opt_L=-fX[-1], fX=fX, line_searches=nls,
                evaluations=n_eval[0], vbopt=o2, hypinfo=info)

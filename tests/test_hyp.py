"""Hyperparameter learning: vbhemh3m_lb.m:202-356
derivatives, the minimize_new.m optimiser, uniqueLL.m and the
form_outputH3M.m groups.

CPU: the analytic derivatives (host.lower_bound_derivs) against central finite
differences of the bound value (host.lower_bound, posterior held fixed) and
against the oracle's loop restatement; clipping; the L-BFGS / BFGS
minimisers on the Rosenbrock function; uniqueLL and groups on known inputs.
GPU: one hyperparameter-learning run (vbhem_h3m_c_hyp) whose every evaluation
is a fused-E-step EM run: the bound must not decrease, and the gradient the
EM run reports at convergence must match a finite difference of the
converged bound.
"""
import numpy as np
import pytest

from cases import make_case

HYPS = ("alpha0", "eta0", "epsilon0", "v0", "lambda0")


def _bound(vb, cs, opt, Lt1=-1234.5, Lt7=-3.25):
    """host.lower_bound with the case's posterior and constants held fixed."""
    P, consts = cs["P"], cs["consts"]
    logOm = vb.host.log_omega_tilde(P.alpha)
    Nj = P.alpha - cs["opt"]["alpha0"] + 1e-50
    return vb.host.lower_bound(Lt1, Lt7, Nj, logOm, P, consts, opt, opt["covmode"])


@pytest.mark.parametrize("cov,W0", [(1, 0.7), (1, [0.4, 0.9, 1.3]), (0, 0.25)],
                         ids=["full-iid", "full-diagW0", "diag-iid"])
def test_derivatives_match_finite_differences(vb, cov, W0):
    cs = make_case(7, 3, 4, 3, 3, cov, seed=17, tau=6, W0=W0, m0=[0.5, 1.0, 1.5])
    opt = dict(cs["opt"])
    P, consts = cs["P"], cs["consts"]
    logOm = vb.host.log_omega_tilde(P.alpha)
    g = vb.host.lower_bound_derivs(logOm, P, consts, opt, cov)["raw"]
    for h in HYPS:
        x = float(opt[h])
        e = 1e-6 * x
        fp = _bound(vb, cs, dict(opt, **{h: x + e}))
        fm = _bound(vb, cs, dict(opt, **{h: x - e}))
        fd = (fp - fm) / (2 * e)
        assert abs(fd - g[h][0]) <= 1e-6 * max(1.0, abs(fd)), (h, fd, g[h][0])
    W0v = np.atleast_1d(np.asarray(opt["W0"], float))
    for i in range(W0v.size):
        e = 1e-6 * W0v[i]
        wp, wm = W0v.copy(), W0v.copy()
        wp[i] += e
        wm[i] -= e
        cast = (lambda w: float(w[0])) if np.ndim(opt["W0"]) == 0 else (lambda w: w)
        fd = (_bound(vb, cs, dict(opt, W0=cast(wp))) - _bound(vb, cs, dict(opt, W0=cast(wm)))) / (2 * e)
        assert abs(fd - g["W0"][i]) <= 1e-6 * max(1.0, abs(fd)), ("W0", i, fd, g["W0"][i])
    m0 = np.asarray(opt["m0"], float)
    for a in range(m0.size):
        e = 1e-6 * max(1.0, abs(m0[a]))
        mp, mm = m0.copy(), m0.copy()
        mp[a] += e
        mm[a] -= e
        fd = (_bound(vb, cs, dict(opt, m0=mp)) - _bound(vb, cs, dict(opt, m0=mm))) / (2 * e)
        assert abs(fd - g["m0"][a]) <= 1e-6 * max(1.0, abs(fd)), ("m0", a, fd, g["m0"][a])


@pytest.mark.parametrize("cov,W0", [(1, 0.7), (1, [0.4, 0.9, 1.3]), (0, 0.25)])
def test_derivatives_match_oracle(vb, vo, cov, W0):
    cs = make_case(6, 4, 3, 3, 3, cov, seed=23, tau=5, W0=W0, m0=[0.2, 0.4, 0.8])
    opt = dict(cs["opt"])
    P, consts = cs["P"], cs["consts"]
    logOm = vb.host.log_omega_tilde(P.alpha)
    clipped = {h: np.zeros(np.size(opt[h])) for h in ("alpha0", "eta0", "epsilon0", "v0", "lambda0",
                                                         "W0")}
    clipped["alpha0"][0] = 1.0      # at the max: a positive derivative is zeroed
    clipped["v0"][0] = -1.0         # at the min: a negative derivative is zeroed
    got = vb.host.lower_bound_derivs(logOm, P, consts, opt, cov, clipped)
    ref = vo.lower_bound_derivs(logOm, cs["post"], consts, opt, clipped)
    for k, v in ref.items():
        np.testing.assert_allclose(np.atleast_1d(got[k]), np.atleast_1d(v), rtol=1e-12, atol=1e-12,
                                   err_msg=k)


def test_clip_flags(vb):
    opt = vb.default_options(2, 2, 2, alpha0=1e20, v0=5.0, W0=1e-20)
    o, fl = vb.clip_hyps(opt, with_flags=True)
    assert o["alpha0"] == opt["hyps_max"]["alpha0"] and fl["alpha0"][0] == 1
    assert o["W0"] == opt["hyps_min"]["W0"] and fl["W0"][0] == -1
    assert fl["v0"][0] == 0 and o["v0"] == 5.0


@pytest.mark.parametrize("method", ["LBFGS", "BFGS", "CG"])
def test_minimize_rosenbrock(vb, method):
    from vbhem_amd.hyp import minimize

    def F(x):
        a, b = x
        return ((1 - a) ** 2 + 100 * (b - a * a) ** 2,
                np.array([-2 * (1 - a) - 400 * a * (b - a * a), 200 * (b - a * a)]))

    x, fX, nls = minimize(np.array([-1.2, 1.0]), F, length=100, method=method)
    assert np.allclose(x, [1.0, 1.0], atol=1e-6) and fX[-1] < 1e-10
    assert np.all(np.diff(fX) <= 1e-12)          # every accepted line search descends
    assert nls <= 100


def test_minimize_bisects_on_any_error(vb):
    """minimize_new.m:147-155 catches ANY error of the objective during
    extrapolation and bisects: an exception other than a floating-point one
    (e.g. a C-ABI error on extreme hyperparameters) must not end the run."""
    from vbhem_amd.hyp import minimize
    calls = []

    def F(x):
        calls.append(float(x[0]))
        if len(calls) == 5:                      # the 4th extrapolation point fails once
            raise RuntimeError("vbhem_estep_fused: status -2")
        return (x[0] - 1.9) ** 2, np.array([2 * (x[0] - 1.9)])

    x, fX, _ = minimize(np.array([-10.0]), F, length=20, method="LBFGS")
    assert abs(x[0] - 1.9) < 1e-6 and len(calls) > 6


def test_minimizer_names(vb):
    """vbhem_h3m_c_hyp.m:34-52: lbfgs / bfgs / cg, anything else is an error."""
    from vbhem_amd import hyp
    opt = dict(minimizer="fminunc", m0=np.zeros(2), W0=1.0, alpha0=1.0, eta0=1.0,
               epsilon0=1.0, lambda0=1.0, v0=5.0)
    with pytest.raises(ValueError, match="bad minimizer"):
        hyp.vbhem_h3m_c_hyp(None, opt, None, None, length=1)


def test_minimize_quadratic_exact(vb):
    """A convex quadratic in 5 dimensions: L-BFGS reaches the minimiser."""
    from vbhem_amd.hyp import minimize
    rng = np.random.default_rng(3)
    Q = rng.normal(size=(5, 5))
    A = Q @ Q.T + 5 * np.eye(5)
    bvec = rng.normal(size=5)
    x, fX, _ = minimize(np.zeros(5), lambda x: (0.5 * x @ A @ x - bvec @ x, A @ x - bvec), length=50)
    np.testing.assert_allclose(x, np.linalg.solve(A, bvec), rtol=1e-7, atol=1e-9)


def test_unique_ll_and_groups(vb):
    from vbhem_amd.cluster import form_groups, unique_ll
    LL = [-100.0, -100.0001, -90.0, -100.5, -90.00001, -80.0]
    # thresh 2 * minDiff * 10 with minDiff 1e-5: 2e-4 relative
    assert unique_ll(LL, 2e-4) == [0, 2, 3, 5]
    assert unique_ll([-5.0], 1e-3) == [0]
    groups, size = form_groups(np.array([2, 0, 2, 1, 0, 2]), 4)
    assert [g.tolist() for g in groups] == [[1, 4], [3], [0, 2, 5], []]
    assert size.tolist() == [2, 1, 3, 0]


@pytest.mark.gpu
def test_hyp_learning_run(vb):
    """One vbhem_h3m_c_hyp run on a small C2-like problem: every objective
    evaluation is an EM run through the fused device E-step; the optimised bound
    is at least the starting one, and at the start the EM-reported gradient
    matches a central finite difference of the converged bound in log(alpha0)."""
    import torch
    from vbhem_amd import em, hyp
    from vbhem_amd.estep import EStepEngine
    cs = make_case(40, 3, 3, 2, 2, 1, seed=5, tau=10, W0=1.0, m0=[1.5, 1.5])
    opt = dict(cs["opt"], max_iter=200, minDiff=1e-10, learn_hyps=1)
    eng = EStepEngine(cs["bs"], 3, 3, 10, device="cuda:0")
    start = em.vbhem_h3m_c_step_fc(cs["P"], eng, opt)
    info = hyp.hypinfo(1, opt)
    X0 = hyp.init_x(opt, info)

    def f(X):
        o = vb.clip_hyps(hyp.set_opt(X, opt, info))
        o["calc_LLderiv"] = 1
        r = em.vbhem_h3m_c_step_fc(start.post, eng, o)
        return r.LL, r.dLL

    L0, d0 = f(X0)
    e = 1e-4
    Xp, Xm = X0.copy(), X0.copy()
    Xp[0] += e
    Xm[0] -= e
    fd = (f(Xp)[0] - f(Xm)[0]) / (2 * e)
    assert abs(fd - float(np.atleast_1d(d0["d_logalpha0"])[0])) <= 1e-3 * max(1.0, abs(fd))
    out = hyp.vbhem_h3m_c_hyp(cs["bs"], opt, start.post, eng, length=8)
    assert out["result"].stable and np.isfinite(out["result"].LL)
    assert out["result"].LL >= L0 - 1e-6 * abs(L0)
    assert out["evaluations"] >= 2
    del torch


@pytest.mark.parametrize("cov,W0", [(1, 0.7), (1, [0.4, 0.9, 1.3]), (0, 0.25), (0, [0.3, 0.5, 2.0])],
                         ids=["full-iid", "full-diagW0", "diag-iid", "diag-diagW0"])
def test_native_derivatives_match_host(vb, cov, W0):
    """vbhem_em_lower_bound_derivs (C++, the loop's calc_LLderiv) against
    host.lower_bound_derivs (itself checked against finite differences and the
    oracle above): raw derivatives at 1e-12."""
    from vbhem_amd import native_em
    cs = make_case(6, 4, 3, 3, 3, cov, seed=29, tau=5, W0=W0, m0=[0.2, -0.4, 0.8])
    opt = dict(cs["opt"])
    P, consts = cs["P"], cs["consts"]
    logOm = vb.host.log_omega_tilde(P.alpha)
    ref = vb.host.lower_bound_derivs(logOm, P, consts, opt, cov)["raw"]
    got = native_em.lower_bound_derivs(P, opt, cov)
    for k, v in ref.items():
        np.testing.assert_allclose(got[k], np.atleast_1d(v), rtol=1e-12, atol=1e-12, err_msg=k)
    # the clipping / change of variables is shared with the Python path
    tr = vb.host.transform_derivs(got, opt)
    full = vb.host.lower_bound_derivs(logOm, P, consts, opt, cov)
    for k in ("d_logalpha0", "d_logv0D1", "d_logW0", "d_m0"):
        np.testing.assert_allclose(tr[k], full[k], rtol=1e-12, atol=1e-12, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [1, 0])
def test_native_loop_derivatives_match_python_loop(vb, cov):
    """calc_LLderiv on the C++ loop (vbhem_em_run_ext: the posterior before the last
    M-step kept on the device, derivatives in C++) equals the Python loop's."""
    from vbhem_amd import em, native_em
    from vbhem_amd.estep import EStepEngine
    cs = make_case(60, 3, 3, 2, 2, cov, seed=41 + cov, tau=10, W0=1.0, m0=[1.5, 1.5])
    opt = dict(cs["opt"], max_iter=30, minDiff=1e-7, calc_LLderiv=1)
    eng = EStepEngine(cs["bs"], 3, 3, 10, device="cuda:0")
    ref = em.vbhem_h3m_c_step_fc(cs["P"], eng, opt)
    got = native_em.run(cs["P"], eng, opt, calc_deriv=True)
    assert got.iters == ref.iters and got.stable and ref.stable
    for k, v in ref.dLL.items():
        if k == "raw":
            continue
        np.testing.assert_allclose(np.atleast_1d(got.dLL[k]), np.atleast_1d(v), rtol=1e-10,
                                   atol=1e-9, err_msg=k)


@pytest.mark.gpu
def test_hyp_learning_native_loop_matches_python_loop(vb):
    """vbhem_h3m_c_hyp with every evaluation on the C++ loop (loop='native') follows
    the Python-loop run: same line searches, bounds and hyperparameters."""
    from vbhem_amd import em, hyp
    from vbhem_amd.estep import EStepEngine
    cs = make_case(40, 3, 3, 2, 2, 1, seed=5, tau=10, W0=1.0, m0=[1.5, 1.5])
    opt = dict(cs["opt"], max_iter=200, minDiff=1e-10, learn_hyps=1)
    eng = EStepEngine(cs["bs"], 3, 3, 10, device="cuda:0")
    start = em.vbhem_h3m_c_step_fc(cs["P"], eng, opt)
    a = hyp.vbhem_h3m_c_hyp(cs["bs"], opt, start.post, eng, length=6, loop="python")
    b = hyp.vbhem_h3m_c_hyp(cs["bs"], opt, start.post, eng, length=6, loop="native")
    assert a["evaluations"] == b["evaluations"] and a["line_searches"] == b["line_searches"]
    np.testing.assert_allclose(b["fX"], a["fX"], rtol=1e-10)
    np.testing.assert_allclose(b["opt_transhyp"], a["opt_transhyp"], rtol=1e-8, atol=1e-10)
    np.testing.assert_allclose(b["result"].LL, a["result"].LL, rtol=1e-10)

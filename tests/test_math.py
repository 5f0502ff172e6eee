"""Restricted-domain fp64 exp/log/reciprocal of csrc/vbhem_math.h (the
transcendentals of the recursions) against libm: <= 1 ulp on their domains.
Host build on the CPU; the gfx950 build (v_rcp_f64 seed) on the GPU."""
import ctypes

import numpy as np
import pytest

N = 400_000


def _samples():
    rng = np.random.default_rng(123)
    # exp(-x): x in [0, 700] (log-uniform and uniform); log/rcp: z in [1e-200, 1e3]
    x = np.concatenate([rng.uniform(0, 700, N // 4), 10 ** rng.uniform(-18, np.log10(700), N // 4),
                        10 ** rng.uniform(-200, 3, N // 4), rng.uniform(0.5, 2.0, N // 4)])
    x[:4] = [1e-300, 0.5, 1.0, 2.0]
    return np.ascontiguousarray(x)


def _run(fn, x):
    dp = ctypes.POINTER(ctypes.c_double)
    e, l, r = (np.zeros_like(x) for _ in range(3))
    rc = fn(len(x), x.ctypes.data_as(dp), e.ctypes.data_as(dp), l.ctypes.data_as(dp),
            r.ctypes.data_as(dp))
    return rc, e, l, r


def _ulps(a, b):
    return np.abs(a - b) / np.spacing(np.abs(b))


def _check(x, e, l, r):
    m = x <= 700
    assert _ulps(e[m], np.exp(-x[m])).max() <= 1.0
    pos = x >= 1e-200
    assert _ulps(l[pos], np.log(x[pos])).max() <= 1.0
    assert _ulps(r[pos], 1.0 / x[pos]).max() <= 1.0
    assert l[2] == 0.0 and e[2] == np.exp(-1.0)


def test_host_build(mathcheck):
    x = _samples()
    rc, e, l, r = _run(mathcheck.mathcheck_host, x)
    _check(x, e, l, r)


def test_exp_clamps_far_tail(mathcheck):
    x = np.array([745.0, 800.0, 1e4, 1e300])
    rc, e, l, r = _run(mathcheck.mathcheck_host, x)
    assert (e <= 5e-324).all() and (e >= 0).all()


@pytest.mark.gpu
def test_device_build(mathcheck):
    x = _samples()
    rc, e, l, r = _run(mathcheck.mathcheck_device, x)
    assert rc == 0
    _check(x, e, l, r)


def _check_logtab(fn):
    """log_tab at x and exp_tab at -x (the backward sweep's table-driven pair)."""
    x = _samples()
    x = np.concatenate([x, np.random.default_rng(7).uniform(0.99, 1.01, N // 4)])
    dp = ctypes.POINTER(ctypes.c_double)
    l, e = np.zeros_like(x), np.zeros_like(x)
    rc = fn(len(x), x.ctypes.data_as(dp), l.ctypes.data_as(dp), e.ctypes.data_as(dp))
    pos = x >= 1e-200
    assert _ulps(l[pos], np.log(x[pos])).max() <= 1.0
    assert l[2] == 0.0
    m = x <= 700
    assert _ulps(e[m], np.exp(-x[m])).max() <= 1.0
    return rc


def test_logtab_host_build(mathcheck):
    """Table-driven log of the backward sweep (log_tab_n), host build."""
    _check_logtab(mathcheck.logtab_host)


@pytest.mark.gpu
def test_logtab_device_build(mathcheck):
    assert _check_logtab(mathcheck.logtab_device) == 0


def _check_logtabf(fn):
    """Reduced-operation pair of the backward-only pass (log_tabf_n / exp_tabf_n):
    <= 2 ulp (log) and <= 2 ulp (exp) on the same samples."""
    x = _samples()
    x = np.concatenate([x, np.random.default_rng(7).uniform(0.99, 1.01, N // 4)])
    dp = ctypes.POINTER(ctypes.c_double)
    l, e = np.zeros_like(x), np.zeros_like(x)
    rc = fn(len(x), x.ctypes.data_as(dp), l.ctypes.data_as(dp), e.ctypes.data_as(dp))
    pos = x >= 1e-200
    assert _ulps(l[pos], np.log(x[pos])).max() <= 2.0
    assert l[2] == 0.0
    m = x <= 700
    assert _ulps(e[m], np.exp(-x[m])).max() <= 2.0
    return rc


def test_logtabf_host_build(mathcheck):
    _check_logtabf(mathcheck.logtabf_host)


@pytest.mark.gpu
def test_logtabf_device_build(mathcheck):
    assert _check_logtabf(mathcheck.logtabf_device) == 0


def _check_logtabc(fn):
    """Compact-table pair of fb_bwd2_kernel (log_tabc_n / exp_tabc_n): log within
    2 ulp + 4e-18 absolute (series cut after r^7), exp <= 2 ulp on [-700, 0] and
    exp(-700) below it (clamped so the exponent add stays normal)."""
    x = _samples()
    x = np.concatenate([x, np.random.default_rng(7).uniform(0.99, 1.01, N // 4),
                        [700.0, 745.0, 800.0, 1e4]])
    dp = ctypes.POINTER(ctypes.c_double)
    l, e = np.zeros_like(x), np.zeros_like(x)
    rc = fn(len(x), x.ctypes.data_as(dp), l.ctypes.data_as(dp), e.ctypes.data_as(dp))
    pos = x >= 1e-200
    ref = np.log(x[pos])
    assert (np.abs(l[pos] - ref) <= 2.0 * np.spacing(np.abs(ref)) + 4e-18).all()
    assert l[2] == 0.0
    m = x <= 700
    assert _ulps(e[m], np.exp(-x[m])).max() <= 2.0
    assert (e[x >= 700] == e[x == 700.0][0]).all() and e[x == 700.0][0] > 0
    return rc


def test_logtabc_host_build(mathcheck):
    _check_logtabc(mathcheck.logtabc_host)


@pytest.mark.gpu
def test_logtabc_device_build(mathcheck):
    assert _check_logtabc(mathcheck.logtabc_device) == 0


def _check_logtabe(fn):
    """Short-series pair of fb_bwd2_kernel (log_tabe_n / exp_tabe_n): log within
    2 ulp + 1e-17 absolute (1024 intervals, series cut after r^4), exp within
    2 ulp + 0.3 |x| ulp on [-700, 0] (one-constant reduction) and exp(-700) below."""
    x = _samples()
    x = np.concatenate([x, np.random.default_rng(9).uniform(0.99, 1.01, N // 4),
                        np.random.default_rng(10).uniform(0.0, 1.0, N // 4),
                        [700.0, 745.0, 800.0, 1e4]])
    dp = ctypes.POINTER(ctypes.c_double)
    l, e = np.zeros_like(x), np.zeros_like(x)
    rc = fn(len(x), x.ctypes.data_as(dp), l.ctypes.data_as(dp), e.ctypes.data_as(dp))
    pos = x >= 1e-200
    ref = np.log(x[pos])
    assert (np.abs(l[pos] - ref) <= 2.0 * np.spacing(np.abs(ref)) + 1e-17).all()
    assert abs(l[x == 1.0]).max() < 1e-17
    m = x <= 700
    assert (_ulps(e[m], np.exp(-x[m])) <= 2.0 + 0.3 * x[m]).all()
    assert _ulps(e[x <= 1.0], np.exp(-x[x <= 1.0])).max() <= 2.0
    assert (e[x >= 700] == e[x == 700.0][0]).all() and e[x == 700.0][0] > 0
    return rc


def test_logtabe_host_build(mathcheck):
    _check_logtabe(mathcheck.logtabe_host)


@pytest.mark.gpu
def test_logtabe_device_build(mathcheck):
    assert _check_logtabe(mathcheck.logtabe_device) == 0


@pytest.mark.gpu
def test_mfma_kernels_exp_log_device_build(mathcheck):
    """exp_m_n / log_m_n of fb_bwd4_kernel and fb_list4_kernel (vbhem_mfma4.h) at the
    column maximum m = 0: exp to second order (|r| <= ln2/4096: <= 8.1e-13 relative,
    plus the one-constant reduction's 3.3e-17 |x|) on [0, 700] and clamped at ~exp(-700)
    below; log1p to third order (<= 1.4e-14 absolute) over the positive normals."""
    dp = ctypes.POINTER(ctypes.c_double)
    fn = mathcheck.logtabm_device
    fn.argtypes = [ctypes.c_int, dp, dp, dp]
    x = _samples()
    x = np.concatenate([x, np.random.default_rng(11).uniform(0.99, 1.01, N // 4),
                        np.random.default_rng(12).uniform(0.0, 1.0, N // 4),
                        np.random.default_rng(13).uniform(0.0, 700.0, N // 4), [700.0, 745.0, 800.0, 1e4]])
    l, e = np.zeros_like(x), np.zeros_like(x)
    assert fn(len(x), x.ctypes.data_as(dp), l.ctypes.data_as(dp), e.ctypes.data_as(dp)) == 0
    pos = x >= 1e-200
    ref = np.log(x[pos])
    assert (np.abs(l[pos] - ref) <= 2.0 * np.spacing(np.abs(ref)) + 2e-14).all()
    m = x <= 700
    rel = np.abs(e[m] - np.exp(-x[m])) / np.exp(-x[m])
    assert (rel <= 1e-12 + 1e-16 * x[m]).all(), float(rel.max())
    assert (e[x > 710] > 0).all() and (e[x > 710] < 1e-300).all()


@pytest.mark.gpu
def test_scaled_log_table_device_build(mathcheck):
    """Round 6 (vbhem_mfma4.h): the log on the 2^1023-scaled 1/c table (log_x_n, the
    table's exponent lowered by Z's with one v_mad_i32_i24) gives the same bits as
    log_q_n on the plain table over the positive normals up to 1e300 (the scaled 1/c
    stays normal), for the decoupled (k ln 2) and the 2048-unit maxima, within the
    accuracy test_mfma_kernels_exp_log_device_build holds the old form to (the exp pair
    of the kernel is the unchanged exp_d_n, checked here beside it)."""
    dp = ctypes.POINTER(ctypes.c_double)
    fn = mathcheck.logtabx_device
    fn.argtypes = [ctypes.c_int, dp, dp]
    rng = np.random.default_rng(21)
    x = np.concatenate([np.exp(rng.uniform(np.log(1e-300), np.log(1e300), N // 2)),
                        rng.uniform(0.99, 1.01, N // 8), rng.uniform(0.0, 8.0, N // 8),
                        rng.uniform(0.0, 700.0, N // 8), rng.uniform(700.0, 7.0e5, N // 8),
                        [1e-300, 1.0, 2.0, 8.0, 700.0, 745.0, 6.99e5]])
    out = np.zeros(6 * len(x))
    assert fn(len(x), x.ctypes.data_as(dp), out.ctypes.data_as(dp)) == 0
    out = out.reshape(-1, 6)
    assert np.array_equal(out[:, 0], out[:, 1])
    assert np.array_equal(out[:, 2], out[:, 3])
    m = x < 7.0e5   # the exp's integer range (red_s)
    assert np.array_equal(out[m, 4], out[m, 5])
    ref = np.log(x)
    assert (np.abs(out[:, 0] - ref) <= 2.0 * np.spacing(np.abs(ref)) + 2e-13).all()
    e = x <= 700
    rel = np.abs(out[e, 4] - np.exp(-x[e])) / np.exp(-x[e])
    assert (rel <= 1e-12 + 1e-16 * x[e]).all(), float(rel.max())

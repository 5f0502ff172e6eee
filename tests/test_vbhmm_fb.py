"""VB-HMM forward-backward (src/hmm/vbhmm_fb_mex.c, vbhmm_fb.m).

CPU: the C restatement (oracle/vbhmm_fb_oracle.c, MEX loop order) against the
numpy restatement of the MATLAB path (vbhmm_fb.m:227-379) and closed forms:
gamma sums to 1 per step, xi_sum to T-1 per sequence, and phi_norm is the log
of the sum over all state paths of prod p(z_1) prod A prod exp(logrho) (brute
force on tiny cases) -- the scaled recursion's normaliser.
GPU: the HIP kernel through the C-ABI (device and host entry points) against
the C restatement; tolerance 1e-12 (normwise relative; same operation order,
libm vs device exp/log)."""
import ctypes
import itertools

import numpy as np
import pytest

import vbhem_oracle as vo
from conftest import rel_err


def make_fb_case(N=6, K=3, dim=2, maxT=9, seed=0, empty=True):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, maxT + 1, N)
    if empty and N > 2:
        lens[1] = 0
        lens[-1] = maxT
    # eye-fixation-like data: pixel coordinates around a few regions
    ctr = rng.uniform(50, 500, (K, dim))
    data = [ctr[rng.integers(0, K, int(T))] + rng.normal(0, 30, (int(T), dim)) for T in lens]
    L = rng.normal(size=(K, dim, dim))
    W = (L @ L.transpose(0, 2, 1)) / dim + 0.5 * np.eye(dim)
    W = W / 900.0  # precision scale of ~30 px spreads
    vp = dict(m=ctr + rng.normal(0, 10, (K, dim)), W=W, v=rng.uniform(dim + 1, dim + 8, K),
              beta=rng.uniform(0.5, 5, K), epsilon=rng.uniform(0.2, 5, (K, K)),
              alpha=rng.uniform(0.2, 5, K))
    return data, vp


FB_SHAPES = [  # (name, N, K, dim, maxT)
    ("eye", 12, 3, 2, 15), ("K1", 5, 1, 2, 6), ("T1", 6, 4, 2, 1), ("dim1", 7, 3, 1, 9),
    ("dim5", 5, 5, 5, 8), ("K8", 9, 8, 2, 20), ("K16", 4, 16, 3, 12), ("long", 3, 4, 2, 300),
]


@pytest.mark.parametrize("shape", FB_SHAPES, ids=[s[0] for s in FB_SHAPES])
def test_oracle_c_matches_matlab_twin(shape):
    name, N, K, dim, maxT = shape
    data, vp = make_fb_case(N, K, dim, maxT, seed=len(name))
    a, b = vo.c_vbhmm_fb(data, vp), vo.twin_vbhmm_fb(data, vp)
    for k in ("logrho", "gamma", "xi_sum", "phi_norm"):
        assert rel_err(a[k], b[k]) < 1e-12, (name, k, rel_err(a[k], b[k]))


def test_oracle_closed_forms():
    data, vp = make_fb_case(10, 4, 2, 12, seed=3)
    r = vo.c_vbhmm_fb(data, vp)
    for n, x in enumerate(data):
        T = len(x)
        if T == 0:
            assert r["phi_norm"][n] == 0 and not r["xi_sum"][n].any()
            continue
        assert np.allclose(r["gamma"][:T, n].sum(-1), 1.0, atol=1e-12)
        assert not r["gamma"][T:, n].any() and not r["logrho"][T:, n].any()
        assert abs(r["xi_sum"][n].sum() - (T - 1)) < 1e-11


def test_oracle_phi_norm_is_path_sum():
    data, vp = make_fb_case(4, 3, 2, 4, seed=9, empty=False)
    pre = vo.vbhmm_prelude(vp)
    r = vo.c_vbhmm_fb(data, vp, pre)
    for n, x in enumerate(data):
        T = len(x)
        lr = r["logrho"][:T, n]                       # [T][K]
        tot = []
        for path in itertools.product(range(3), repeat=T):
            s = np.log(pre["pz1"][path[0]]) + lr[0, path[0]]
            for t in range(1, T):
                s += np.log(pre["A"][path[t - 1], path[t]]) + lr[t, path[t]]
            tot.append(s)
        ref = np.log(np.sum(np.exp(np.array(tot) - max(tot)))) + max(tot)
        assert abs(r["phi_norm"][n] - ref) < 1e-10 * abs(ref)
        # and gamma is the path posterior marginal
        w = np.exp(np.array(tot) - ref)
        g = np.zeros((T, 3))
        for p, wi in zip(itertools.product(range(3), repeat=T), w):
            for t in range(T):
                g[t, p[t]] += wi
        assert np.allclose(g, r["gamma"][:T, n], atol=1e-12)


def test_fb_capi_argument_checks(capi_lib):
    from vbhem_amd import _capi
    p = 1 << 20
    s = _capi.SeqsT(4, 2, 5, p, p)
    q = _capi.HmmParamsT(3, 2, p, p, p, p, p, p, p, 1.0)
    assert capi_lib.vbhmm_fb_workspace_bytes(ctypes.byref(s), 3) >= 2 * 4 * 5 * 8
    q17 = _capi.HmmParamsT(17, 2, p, p, p, p, p, p, p, 1.0)
    v = ctypes.c_void_p(p)
    assert capi_lib.vbhmm_fb(ctypes.byref(s), ctypes.byref(q17), v, v, v, v, v,
                             ctypes.c_size_t(1 << 30), None) == -2
    qd = _capi.HmmParamsT(3, 3, p, p, p, p, p, p, p, 1.0)   # dim mismatch
    assert capi_lib.vbhmm_fb(ctypes.byref(s), ctypes.byref(qd), v, v, v, v, v,
                             ctypes.c_size_t(1 << 30), None) == -1
    assert capi_lib.vbhmm_fb(ctypes.byref(s), ctypes.byref(q), v, v, v, v, v,
                             ctypes.c_size_t(8), None) == -3


@pytest.mark.gpu
@pytest.mark.parametrize("shape", FB_SHAPES, ids=[s[0] for s in FB_SHAPES])
def test_fb_gpu_matches_oracle(vb, shape):
    from vbhem_amd import vbhmm
    name, N, K, dim, maxT = shape
    data, vp = make_fb_case(N, K, dim, maxT, seed=len(name) + 100)
    ref = vo.c_vbhmm_fb(data, vp)
    got = vbhmm.vbhmm_fb(data, vp, device="cuda:0")
    assert rel_err(got["logrho_Saved"], ref["logrho"].transpose(2, 1, 0)) < 1e-12
    assert rel_err(got["gamma_all"], ref["gamma"].transpose(2, 1, 0)) < 1e-12
    assert rel_err(got["xi_sum"], ref["xi_sum"].transpose(1, 2, 0)) < 1e-12
    assert rel_err(got["phi_norm"], ref["phi_norm"]) < 1e-12


@pytest.mark.gpu
def test_fb_gpu_host_entry_and_batch(vb, capi_lib):
    """The host-pointer entry point (the MEX gateway's call) on a larger ragged
    batch (4,000 sequences), checked on the full batch against the oracle."""
    from vbhem_amd import _capi
    data, vp = make_fb_case(4000, 5, 2, 40, seed=7)
    pre = vo.vbhmm_prelude(vp)
    off, x, maxT = vo.pack_sequences(data, 2)
    N, K = len(data), 5
    out = dict(logrho=np.zeros((maxT, N, K)), gamma=np.zeros((maxT, N, K)),
               xi_sum=np.zeros((N, K, K)), phi_norm=np.zeros(N))
    arrs = {k: np.ascontiguousarray(a, dtype=np.float64) for k, a in
            (("m", vp["m"]), ("W", vp["W"]), ("v", vp["v"]), ("beta", vp["beta"]),
             ("l", pre["logLambdaTilde"]), ("pz1", pre["pz1"]), ("A", pre["A"]))}
    s = _capi.SeqsT(N, 2, maxT, off.ctypes.data, x.ctypes.data)
    q = _capi.HmmParamsT(K, 2, *[arrs[k].ctypes.data for k in ("m", "W", "v", "beta", "l", "pz1", "A")],
                         float(pre["const_denominator"]))
    rc = capi_lib.vbhmm_fb_host(0, ctypes.byref(s), ctypes.byref(q), out["logrho"].ctypes.data,
                                out["gamma"].ctypes.data, out["xi_sum"].ctypes.data,
                                out["phi_norm"].ctypes.data)
    assert rc == 0, capi_lib.vbhem_last_error()
    ref = vo.c_vbhmm_fb(data, vp, pre)
    for k in out:
        assert rel_err(out[k], ref[k]) < 1e-12, k

"""The fused-E-step MEX gateway (integration/vbhem_estep_fused_mex.c) through
the mx API test double: argument checks (CPU), and on the GPU the outputs
[LL_elbo, hat_Z, stats] against the oracle, with the base set kept resident
across calls (same h3m_b: no re-upload; a different h3m_b: re-uploaded) and
released by the no-argument call / mexAtExit."""
import numpy as np
import pytest
from scipy.special import digamma

from cases import make_case
from conftest import RTOL_NORTH_STAR, RTOL_PAIRS, elem_err, hatz_err, stat_err
from mx import Mx, cluster_consts, matlab_h3m


@pytest.fixture(scope="module")
def mx(fused_gateway):
    gw, shim = fused_gateway
    shim.mxshim_clear.restype = None
    return Mx(shim, gw)


def _args(mx, cs, tscale=100.0, sizes=None, key=None):
    base, consts = cs["base"], cs["consts"]
    hb, hr, extra = matlab_h3m(mx, base, consts, sizes=sizes)
    N = base["prior"].shape[0]
    tN = tscale * N * base["omega"]
    alpha = cs["post"]["alpha"]
    logOm = digamma(alpha) - digamma(alpha.sum())          # step_fc.m:271-273
    S = consts["logPi"].shape[1]
    Sb = base["prior"].shape[1]
    args = [hb, hr, mx.double(cs["T"]), mx.double(Sb), mx.double(S)] + extra + \
        [mx.double(tN.reshape(-1, 1)), mx.double(logOm.reshape(1, -1))]
    if key is not None:
        args.append(mx.double(float(key)))
    return args, tN, logOm


def test_rejects_wrong_counts(mx):
    out, err = mx.call(3, [mx.cell([]), mx.cell([])])
    assert err[0] == "MyToolbox:arrayProduct:nrhs"
    cs = make_case(3, 2, 2, 2, 2, 0, seed=1, tau=4)
    args, _, _ = _args(mx, cs)
    out, err = mx.call(6, args)
    assert err == ("MyToolbox:arrayProduct:nlhs", "3 output required.")


def test_rejects_bad_weights(mx):
    cs = make_case(3, 2, 2, 2, 2, 0, seed=1, tau=4)
    args, _, _ = _args(mx, cs)
    args[-2] = mx.double(np.ones((2, 1)))          # tilde_N_k of the wrong length
    out, err = mx.call(3, args)
    assert err[0] == "vbhem_mex:invalidinput" and "tilde_N_k" in err[1]
    args, _, _ = _args(mx, cs)
    args[1] = mx.double(1.0)
    out, err = mx.call(3, args)
    assert err == ("vbhem_mex:invalidinput", "2nd arg must be cell")


def test_release_without_arguments(mx):
    out, err = mx.call(0, [])
    assert err is None
    mx.shim.mxshim_clear()


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [1, 0])
def test_fused_gateway_matches_oracle(mx, vo, vb, cov):
    N, K, S, Sb, d, T = 40, 4, 4, 3, 3, 6
    cs = make_case(N, K, S, Sb, d, cov, seed=70 + cov, ragged=True, tau=T)
    args, tN, logOm = _args(mx, cs)
    pairs = vo.c_estep_pairs(cs["base"], cs["consts"], T)
    hz, Z = vo.c_responsibilities(pairs["LL_elbo"], tN, logOm)
    st = vo.c_statistics(Z, pairs, cov)
    for call in range(2):  # the second call reuses the resident base set
        out, err = mx.call(3, args)
        assert err is None, err
        LL, hZ, vec = (mx.to_numpy(o) for o in out)
        assert LL.shape == (N, K) and hZ.shape == (N, K) and vec.shape[1] == 1
        assert elem_err(LL, pairs["LL_elbo"]) < RTOL_PAIRS
        assert hatz_err(hZ, hz) < RTOL_NORTH_STAR
        got = vb.host.unpack_stats(vec[:, 0], K, S, d, cov)
        for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
            assert stat_err(got[k], st[k]) < 1e-9, (call, k)
    # a different base set through the same gateway: re-uploaded, still right
    cs2 = make_case(N + 7, K, S, Sb, d, cov, seed=90 + cov, ragged=True, tau=T)
    args2, tN2, logOm2 = _args(mx, cs2)
    out, err = mx.call(3, args2)
    assert err is None, err
    p2 = vo.c_estep_pairs(cs2["base"], cs2["consts"], T)
    assert elem_err(mx.to_numpy(out[0]), p2["LL_elbo"]) < RTOL_PAIRS
    mx.shim.mxshim_clear()


def _overwrite(mx, hb_cell, N, field, values):
    """Edit h3m_b{i}.<field> IN PLACE (same mxArray, same data pointer), as MATLAB
    does for an unshared variable."""
    import ctypes
    for i in range(N):
        hb = mx.cell_item(hb_cell, i)
        f = mx.shim.mxGetField(hb, 0, field.encode())
        arr = np.asfortranarray(values[i]).ravel(order="F").astype(np.float64)
        ctypes.memmove(mx.shim.mxGetPr(f), arr.ctypes.data, arr.nbytes)


@pytest.mark.gpu
def test_fused_gateway_detects_in_place_edit(mx, vo):
    """A base set edited in place (same arrays, same pointers) is re-uploaded
    (content fingerprint); with a base_key the caller decides: the same key reuses
    the resident set, a new key re-uploads."""
    import ctypes
    mx.shim.mxGetField.restype = ctypes.c_void_p
    mx.shim.mxGetField.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p]
    N, K, S, Sb, d, T = 12, 3, 3, 3, 2, 5
    cs = make_case(N, K, S, Sb, d, 1, seed=81, tau=T)
    base = cs["base"]
    for key in (None, 7.0):
        args, tN, logOm = _args(mx, cs, key=key)
        out, err = mx.call(3, args)
        assert err is None, err
        p1 = vo.c_estep_pairs(base, cs["consts"], T)
        assert elem_err(mx.to_numpy(out[0]), p1["LL_elbo"]) < RTOL_PAIRS
        # the same arrays, new transition contents
        A2 = base["A"][:, ::-1, :].copy()
        _overwrite(mx, args[0], N, "A", [A2[i, :Sb, :Sb] for i in range(N)])
        b2 = dict(base, A=A2)
        p2 = vo.c_estep_pairs(b2, cs["consts"], T)
        out, err = mx.call(3, args)
        assert err is None, err
        if key is None:   # content fingerprint: re-uploaded
            assert elem_err(mx.to_numpy(out[0]), p2["LL_elbo"]) < RTOL_PAIRS
        else:             # same key: the caller said unchanged, the resident set is used
            assert elem_err(mx.to_numpy(out[0]), p1["LL_elbo"]) < RTOL_PAIRS
            args[-1] = mx.double(8.0)
            out, err = mx.call(3, args)
            assert elem_err(mx.to_numpy(out[0]), p2["LL_elbo"]) < RTOL_PAIRS
        mx.call(0, [])
    mx.shim.mxshim_clear()


@pytest.mark.gpu
def test_fused_gateway_mixed_cluster_sizes(mx, vo, vb):
    """Clusters of N2 = 4, 2, 3 states through the fused gateway (padded to 4):
    L_elbo, hat_Z (softmax over all clusters) and each cluster's statistics over its
    own N2 states equal the oracle run per cluster."""
    N, K, S, Sb, d, T, cov = 30, 3, 4, 3, 2, 6, 1
    sizes = [4, 2, 3]
    cs = make_case(N, K, S, Sb, d, cov, seed=83, ragged=True, tau=T)
    args, tN, logOm = _args(mx, cs, sizes=sizes)
    out, err = mx.call(3, args)
    assert err is None, err
    LL, hZ, vec = (mx.to_numpy(o) for o in out)
    pj = [vo.c_estep_pairs(cs["base"], cluster_consts(cs["consts"], j, n), T)
          for j, n in enumerate(sizes)]
    LLref = np.concatenate([p["LL_elbo"] for p in pj], axis=1)
    assert elem_err(LL, LLref) < RTOL_PAIRS
    hz, Z = vo.c_responsibilities(LLref, tN, logOm)
    assert hatz_err(hZ, hz) < RTOL_NORTH_STAR
    raw = vb.host.unpack_stats(vec[:, 0], K, S, d, cov)
    for j, n in enumerate(sizes):
        st = vo.c_statistics(np.ascontiguousarray(Z[:, j:j + 1]), pj[j], cov)
        assert stat_err(raw["Nj"][j], st["Nj"][0]) < 1e-9
        assert stat_err(raw["N1"][j, :n], st["N1"][0]) < 1e-9
        assert stat_err(raw["M"][j, :n, :n], st["M"][0]) < 1e-9
        for k in ("Nr", "Y", "SC"):
            assert stat_err(raw[k][j, :n], st[k][0]) < 1e-9, (j, k)
        # the padded states hold (numerically) nothing
        assert np.all(np.abs(raw["N1"][j, n:]) < 1e-250)
    mx.call(0, [])
    mx.shim.mxshim_clear()

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
from mx import Mx, matlab_h3m


@pytest.fixture(scope="module")
def mx(fused_gateway):
    gw, shim = fused_gateway
    shim.mxshim_clear.restype = None
    return Mx(shim, gw)


def _args(mx, cs, tscale=100.0):
    base, consts = cs["base"], cs["consts"]
    hb, hr, extra = matlab_h3m(mx, base, consts)
    N = base["prior"].shape[0]
    tN = tscale * N * base["omega"]
    alpha = cs["post"]["alpha"]
    logOm = digamma(alpha) - digamma(alpha.sum())          # step_fc.m:271-273
    S = consts["logPi"].shape[1]
    Sb = base["prior"].shape[1]
    args = [hb, hr, mx.double(cs["T"]), mx.double(Sb), mx.double(S)] + extra + \
        [mx.double(tN.reshape(-1, 1)), mx.double(logOm.reshape(1, -1))]
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

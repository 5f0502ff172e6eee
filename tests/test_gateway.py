"""The MATLAB MEX gateway (integration/vbhem_hmm_bwd_fwd_mex.c), driven through
the mx API test double.  Argument checks mirror the reference gateway
(src/vbhem/vbhem_hmm_bwd_fwd_mex.c:335-367) and run on the CPU; the full call
(GPU) is compared with the oracle."""
import numpy as np
import pytest

from cases import make_case
from conftest import RTOL_PAIRS, rel_err
from mx import Mx, cluster_consts, matlab_h3m


@pytest.fixture(scope="module")
def mx(gateway):
    gw, shim = gateway
    return Mx(shim, gw)


def test_rejects_wrong_input_count(mx):
    out, err = mx.call(6, [mx.cell([]), mx.cell([])])
    assert out is None and err[0] == "MyToolbox:arrayProduct:nrhs"


def test_rejects_wrong_output_count(mx):
    args = [mx.cell([]), mx.cell([]), mx.double(5), mx.double(2), mx.double(2)]
    out, err = mx.call(3, args)
    assert out is None and err == ("MyToolbox:arrayProduct:nlhs", "6 output required.")


def test_rejects_non_cell(mx):
    args = [mx.double(1), mx.cell([]), mx.double(5), mx.double(2), mx.double(2)]
    out, err = mx.call(6, args)
    assert err == ("vbhem_mex:invalidinput", "1st arg must be cell")
    args = [mx.cell([]), mx.double(1), mx.double(5), mx.double(2), mx.double(2)]
    out, err = mx.call(6, args)
    assert err == ("vbhem_mex:invalidinput", "2nd arg must be cell")


def test_rejects_non_scalar_T(mx):
    cs = make_case(2, 2, 2, 2, 2, 0, seed=1)
    hb, hr, extra = matlab_h3m(mx, cs["base"], cs["consts"])
    out, err = mx.call(6, [hb, hr, mx.double([1.0, 2.0]), mx.double(2), mx.double(2)])
    assert err == ("vbhmm_fb_mex:invalidinput", "arg must be scalar.")


def test_rejects_base_larger_than_maxN(mx):
    cs = make_case(2, 2, 2, 3, 2, 0, seed=1)
    hb, hr, extra = matlab_h3m(mx, cs["base"], cs["consts"])
    out, err = mx.call(6, [hb, hr, mx.double(5), mx.double(2), mx.double(2)])   # maxN=2 < 3
    assert err[0] == "vbhem_mex:invalidinput" and "maxN" in err[1]


def test_rejects_cluster_larger_than_maxN2(mx):
    cs = make_case(2, 2, 3, 2, 2, 0, seed=1)
    hb, hr, extra = matlab_h3m(mx, cs["base"], cs["consts"])
    out, err = mx.call(6, [hb, hr, mx.double(5), mx.double(2), mx.double(2)])   # maxN2=2 < 3
    assert err[0] == "vbhem_mex:invalidinput" and "maxN2" in err[1]


def test_empty_base_set_returns_empty_outputs(mx):
    cs = make_case(2, 2, 3, 2, 2, 0, seed=1)
    hb, hr, extra = matlab_h3m(mx, cs["base"], cs["consts"])
    out, err = mx.call(6, [mx.cell([]), hr, mx.double(5), mx.double(2), mx.double(3)])
    assert err is None
    assert mx.to_numpy(out[0]).shape == (0, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("cov,ragged", [(1, False), (0, False), (1, True), (0, True)])
def test_gateway_matches_oracle(mx, vo, cov, ragged):
    N, K, S, Sb, d, T = 5, 3, 4, 4, 3, 7
    cs = make_case(N, K, S, Sb, d, cov, seed=40 + cov, ragged=ragged, tau=T)
    base, consts = cs["base"], cs["consts"]
    hb, hr, extra = matlab_h3m(mx, base, consts)
    out, err = mx.call(6, [hb, hr, mx.double(T), mx.double(Sb), mx.double(S)] + extra)
    assert err is None, err
    ref = vo.c_estep_pairs(base, consts, T)
    LL = mx.to_numpy(out[0])
    assert LL.shape == (N, K)
    assert rel_err(LL, ref["LL_elbo"]) < RTOL_PAIRS
    for i in range(N):
        for j in range(K):
            cell = i + j * N
            nu = mx.to_numpy(mx.cell_item(out[1], cell))
            pr = mx.to_numpy(mx.cell_item(out[2], cell))
            mu = mx.to_numpy(mx.cell_item(out[3], cell))
            Mu = mx.to_numpy(mx.cell_item(out[4], cell))
            xi = mx.to_numpy(mx.cell_item(out[5], cell))
            assert nu.shape == (1, S) and pr.shape == (S, 1) and mu.shape == (S, d)
            assert xi.shape == (S, S)
            assert Mu.shape == ((S, d, d) if cov == 1 else (S, d))
            assert rel_err(nu[0], ref["sum_nu_1"][i, j]) < RTOL_PAIRS
            assert rel_err(pr[:, 0], ref["emit_pr"][i, j]) < RTOL_PAIRS
            assert rel_err(mu, ref["emit_mu"][i, j]) < RTOL_PAIRS
            assert rel_err(Mu, ref["emit_Mu"][i, j]) < RTOL_PAIRS
            assert rel_err(xi, ref["sum_xi"][i, j]) < RTOL_PAIRS


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [1, 0])
def test_gateway_mixed_cluster_sizes(mx, vo, cov):
    """Clusters of different sizes N2 <= maxN2 (mex.c:436-437, 506): every pair's
    outputs are N2[j]-shaped and equal the oracle run on cluster j alone."""
    N, K, S, Sb, d, T = 6, 4, 5, 4, 3, 6
    sizes = [5, 2, 3, 5]
    cs = make_case(N, K, S, Sb, d, cov, seed=44 + cov, ragged=True, tau=T)
    base, consts = cs["base"], cs["consts"]
    hb, hr, extra = matlab_h3m(mx, base, consts, sizes=sizes)
    out, err = mx.call(6, [hb, hr, mx.double(T), mx.double(Sb), mx.double(6)] + extra)
    assert err is None, err
    LL = mx.to_numpy(out[0])
    assert LL.shape == (N, K)
    for j, n in enumerate(sizes):
        ref = vo.c_estep_pairs(base, cluster_consts(consts, j, n), T)
        assert rel_err(LL[:, j], ref["LL_elbo"][:, 0]) < RTOL_PAIRS
        for i in range(N):
            cell = i + j * N
            nu = mx.to_numpy(mx.cell_item(out[1], cell))
            pr = mx.to_numpy(mx.cell_item(out[2], cell))
            mu = mx.to_numpy(mx.cell_item(out[3], cell))
            Mu = mx.to_numpy(mx.cell_item(out[4], cell))
            xi = mx.to_numpy(mx.cell_item(out[5], cell))
            assert nu.shape == (1, n) and pr.shape == (n, 1) and mu.shape == (n, d)
            assert xi.shape == (n, n) and Mu.shape == ((n, d, d) if cov == 1 else (n, d))
            assert rel_err(nu[0], ref["sum_nu_1"][i, 0]) < RTOL_PAIRS
            assert rel_err(pr[:, 0], ref["emit_pr"][i, 0]) < RTOL_PAIRS
            assert rel_err(mu, ref["emit_mu"][i, 0]) < RTOL_PAIRS
            assert rel_err(Mu, ref["emit_Mu"][i, 0]) < RTOL_PAIRS
            assert rel_err(xi, ref["sum_xi"][i, 0]) < RTOL_PAIRS

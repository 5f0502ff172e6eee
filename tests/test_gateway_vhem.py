"""The VHEM sibling MEX gateway (integration/hem_hmm_bwd_fwd_mex.c), driven
through the mx API test double.  Argument checks mirror the reference gateway
(src/compare_mtds/hem/vhem_h3m/hem_hmm_bwd_fwd_mex.c:334-367) and run on the
CPU; the full call (GPU) is compared with the VHEM oracle."""
import numpy as np
import pytest

from cases import make_case, make_reduced
from conftest import RTOL_PAIRS, rel_err
from mx import Mx


@pytest.fixture(scope="module")
def mx(hem_gateway):
    gw, shim = hem_gateway
    return Mx(shim, gw)


def matlab_vhem(mx: Mx, base: dict, red: dict, sizes=None):
    """(h3m_b.hmm, h3m_r.hmm as point-estimate HMMs, extra full-cov args) as MATLAB
    values; the extras are computed as hem_h3m_c_step.m:198-205 does.  ``sizes``:
    per-cluster state counts (the first N2[j] states of each reduced HMM)."""
    cov = base["covmode"]
    N = base["prior"].shape[0]
    K, S0 = red["prior"].shape
    sizes = [S0] * K if sizes is None else list(sizes)
    d = base["centres"].shape[2]
    hb = []
    for i in range(N):
        n = int(base["nstates"][i])
        emit = [mx.struct(centres=mx.double(base["centres"][i, k]),
                          covars=mx.double(base["covars"][i, k]), nin=mx.double(d))
                for k in range(n)]
        hb.append(mx.struct(prior=mx.double(base["prior"][i, :n].reshape(n, 1)),
                            A=mx.double(base["A"][i, :n, :n]), emit=mx.cell(emit)))
    hr = []
    for j in range(K):
        S = sizes[j]
        emit = [mx.struct(centres=mx.double(red["centres"][j, s]),
                          covars=mx.double(red["covars"][j, s]), nin=mx.double(d))
                for s in range(S)]
        hr.append(mx.struct(prior=mx.double(red["prior"][j, :S].reshape(S, 1)),
                            A=mx.double(red["A"][j, :S, :S]), emit=mx.cell(emit)))
    extra = []
    if cov == 1:
        cv = np.asarray(red["covars"])
        extra = [mx.cell([mx.double(np.log(np.linalg.det(cv[j, :sizes[j]]))) for j in range(K)]),
                 mx.cell([mx.double(np.transpose(np.linalg.inv(cv[j, :sizes[j]]), (1, 2, 0)))
                          for j in range(K)])]
    return mx.cell(hb), mx.cell(hr), extra


def test_rejects_wrong_input_count(mx):
    out, err = mx.call(6, [mx.cell([]), mx.cell([]), mx.double(5), mx.double(1), mx.double(2)])
    assert out is None and err == ("MyToolbox:arrayProduct:nrhs", "4 or 6 inputs required.")


def test_rejects_wrong_output_count(mx):
    args = [mx.cell([]), mx.cell([]), mx.double(5), mx.double(1), mx.double(2), mx.double(2)]
    out, err = mx.call(3, args)
    assert out is None and err == ("MyToolbox:arrayProduct:nlhs", "6 output required.")


def test_rejects_non_cell(mx):
    args = [mx.double(1), mx.cell([]), mx.double(5), mx.double(1), mx.double(2), mx.double(2)]
    assert mx.call(6, args)[1] == ("vbhmm_fb_mex:invalidinput", "1st arg must be cell")
    args = [mx.cell([]), mx.double(1), mx.double(5), mx.double(1), mx.double(2), mx.double(2)]
    assert mx.call(6, args)[1] == ("vbhmm_fb_mex:invalidinput", "2nd arg must be cell")


def test_rejects_non_scalar_smooth(mx):
    cs = make_case(2, 2, 2, 2, 2, 0, seed=1)
    hb, hr, extra = matlab_vhem(mx, cs["base"], make_reduced(2, 2, 2, 0, seed=1))
    out, err = mx.call(6, [hb, hr, mx.double(5), mx.double([1.0, 2.0]), mx.double(2), mx.double(2)])
    assert err == ("vbhmm_fb_mex:invalidinput", "arg must be scalar.")


def test_empty_base_set_returns_empty_outputs(mx):
    cs = make_case(2, 2, 3, 2, 2, 0, seed=1)
    hb, hr, extra = matlab_vhem(mx, cs["base"], make_reduced(2, 3, 2, 0, seed=1))
    out, err = mx.call(6, [mx.cell([]), hr, mx.double(5), mx.double(1), mx.double(2), mx.double(3)])
    assert err is None
    assert mx.to_numpy(out[0]).shape == (0, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("cov,ragged,smooth", [(1, False, 1.0), (0, False, 1.0), (1, True, 2.5),
                                               (0, True, 0.7)])
def test_vhem_gateway_matches_oracle(mx, vo, cov, ragged, smooth):
    N, K, S, Sb, d, T = 5, 3, 4, 4, 3, 7
    cs = make_case(N, K, S, Sb, d, cov, seed=60 + cov, ragged=ragged, tau=T)
    base = cs["base"]
    red = make_reduced(K, S, d, cov, seed=60 + cov)
    hb, hr, extra = matlab_vhem(mx, base, red)
    out, err = mx.call(6, [hb, hr, mx.double(T), mx.double(smooth), mx.double(Sb),
                           mx.double(S)] + extra)
    assert err is None, err
    ref = vo.c_vhem_estep_pairs(base, red, T, smooth)
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
            assert Mu.shape == ((S, d, d) if cov == 1 else (S, d))
            assert rel_err(nu[0], ref["sum_nu_1"][i, j]) < RTOL_PAIRS
            assert rel_err(pr[:, 0], ref["emit_pr"][i, j]) < RTOL_PAIRS
            assert rel_err(mu, ref["emit_mu"][i, j]) < RTOL_PAIRS
            assert rel_err(Mu, ref["emit_Mu"][i, j]) < RTOL_PAIRS
            assert rel_err(xi, ref["sum_xi"][i, j]) < RTOL_PAIRS


@pytest.mark.gpu
@pytest.mark.parametrize("cov", [1, 0])
def test_vhem_gateway_mixed_cluster_sizes(mx, vo, cov):
    """Reduced HMMs of different sizes: N2[j]-shaped outputs equal the VHEM oracle
    run on reduced HMM j alone (its first N2[j] states, as given)."""
    N, K, S, Sb, d, T, smooth = 5, 3, 4, 3, 2, 5, 1.5
    sizes = [2, 4, 3]
    cs = make_case(N, K, S, Sb, d, cov, seed=64 + cov, ragged=True, tau=T)
    base = cs["base"]
    red = make_reduced(K, S, d, cov, seed=64 + cov)
    hb, hr, extra = matlab_vhem(mx, base, red, sizes=sizes)
    out, err = mx.call(6, [hb, hr, mx.double(T), mx.double(smooth), mx.double(Sb),
                           mx.double(S)] + extra)
    assert err is None, err
    LL = mx.to_numpy(out[0])
    for j, n in enumerate(sizes):
        rj = {k: np.ascontiguousarray(v[j:j + 1, :n, :n] if k == "A" else v[j:j + 1, :n])
              for k, v in red.items()}
        ref = vo.c_vhem_estep_pairs(base, rj, T, smooth)
        assert rel_err(LL[:, j], ref["LL_elbo"][:, 0]) < RTOL_PAIRS
        for i in range(N):
            cell = i + j * N
            xi = mx.to_numpy(mx.cell_item(out[5], cell))
            Mu = mx.to_numpy(mx.cell_item(out[4], cell))
            assert xi.shape == (n, n)
            assert rel_err(xi, ref["sum_xi"][i, 0]) < RTOL_PAIRS
            assert rel_err(Mu, ref["emit_Mu"][i, 0]) < RTOL_PAIRS
            assert rel_err(mx.to_numpy(mx.cell_item(out[1], cell))[0],
                           ref["sum_nu_1"][i, 0]) < RTOL_PAIRS

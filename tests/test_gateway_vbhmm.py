"""The vbhmm_fb_mex MEX gateway (integration/vbhmm_fb_mex.c) driven through the
mx API test double: argument checks mirror the reference gateway
(src/hmm/vbhmm_fb_mex.c:223-270, CPU); the full call (GPU) returns the MEX's
outputs in MATLAB layout, compared with the oracle."""
import numpy as np
import pytest

import vbhem_oracle as vo
from conftest import rel_err
from mx import Mx
from test_vbhmm_fb import make_fb_case


@pytest.fixture(scope="module")
def mx(fb_gateway):
    gw, shim = fb_gateway
    return Mx(shim, gw)


def matlab_args(mx, data, vp, pre=None, maxT=None):
    """The 13 inputs of vbhmm_fb.m:144-145 as MATLAB values."""
    pre = vo.vbhmm_prelude(vp) if pre is None else pre
    K, dim = np.asarray(vp["m"]).shape
    maxT = max(len(x) for x in data) if maxT is None else maxT
    cells = mx.cell([mx.double(np.asarray(x).reshape(-1, dim)) for x in data], row=False)
    Wm = np.transpose(vp["W"], (1, 2, 0))
    if K == 1:
        Wm = Wm[:, :, 0]   # MATLAB drops the trailing singleton dimension
    return [cells, mx.double(K), mx.double(len(data)), mx.double(dim), mx.double(maxT),
            mx.double(np.asarray(vp["m"]).T), mx.double(Wm),
            mx.double(np.reshape(vp["v"], (K, 1))), mx.double(np.reshape(vp["beta"], (K, 1))),
            mx.double(np.reshape(pre["logLambdaTilde"], (1, K))), mx.double(pre["const_denominator"]),
            mx.double(np.reshape(pre["pz1"], (1, K))), mx.double(pre["A"])]


def test_rejects_wrong_counts(mx):
    data, vp = make_fb_case(3, 2, 2, 4, seed=1)
    args = matlab_args(mx, data, vp)
    out, err = mx.call(4, args[:12])
    assert err == ("MyToolbox:arrayProduct:nrhs", "13 inputs required.")
    out, err = mx.call(3, args)
    assert err == ("MyToolbox:arrayProduct:nlhs", "One output required.")


def test_rejects_bad_inputs(mx):
    data, vp = make_fb_case(3, 2, 2, 4, seed=1)
    args = matlab_args(mx, data, vp)
    bad = list(args)
    bad[0] = mx.double(1.0)
    assert mx.call(4, bad)[1] == ("vbhmm_fb_mex:invalidinput", "1st arg must be cell")
    bad = list(args)
    bad[5] = mx.double(np.zeros((3, 2)))   # m must be dim x K = 2 x 2
    assert mx.call(4, bad)[1] == ("vbhmm_fb_mex:invalidinput", "parseMatrix: invalid size.")
    bad = list(args)
    bad[6] = mx.double(np.zeros((2, 2)))   # W must be dim x dim x K (3-D for K > 1)
    assert mx.call(4, bad)[1] == ("vbhmm_fb_mex:invalidinput",
                                  "parseMatrix3: invalid num dimensions.")
    bad = list(args)
    bad[12] = mx.double(np.zeros((2, 3)))
    assert mx.call(4, bad)[1] == ("vbhmm_fb_mex:invalidinput", "parseMatrix: invalid size.")


@pytest.mark.gpu
@pytest.mark.parametrize("K,dim,N,maxT", [(3, 2, 9, 12), (1, 2, 4, 5), (6, 3, 20, 30)])
def test_gateway_matches_oracle(mx, K, dim, N, maxT):
    data, vp = make_fb_case(N, K, dim, maxT, seed=K * 10 + dim)
    pre = vo.vbhmm_prelude(vp)
    out, err = mx.call(4, matlab_args(mx, data, vp, pre))
    assert err is None, err
    lr, ga, xs, ph = (mx.to_numpy(o) for o in out)
    T = max(len(x) for x in data)
    assert lr.shape == (K, N, T) and ga.shape == (K, N, T) and xs.shape == (K, K, N)
    assert ph.shape == (1, N)
    ref = vo.c_vbhmm_fb(data, vp, pre)
    assert rel_err(lr, ref["logrho"].transpose(2, 1, 0)) < 1e-12
    assert rel_err(ga, ref["gamma"].transpose(2, 1, 0)) < 1e-12
    assert rel_err(xs, ref["xi_sum"].transpose(1, 2, 0)) < 1e-12
    assert rel_err(ph.ravel(), ref["phi_norm"]) < 1e-12

"""Python helpers around the mx API test double (tests/mxshim): build MATLAB
values (column-major doubles, cells, structs) and call a MEX gateway."""
from __future__ import annotations

import ctypes

import numpy as np

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


class Mx:
    def __init__(self, shim, gateway):
        self.shim = shim
        self.gw = gateway
        s = shim
        s.mxCreateNumericArray.restype = _vp
        s.mxCreateNumericArray.argtypes = [_sz, ctypes.POINTER(_sz), ctypes.c_int, ctypes.c_int]
        s.mxCreateCellMatrix.restype = _vp
        s.mxCreateCellMatrix.argtypes = [_sz, _sz]
        s.mxCreateStructMatrix.restype = _vp
        s.mxCreateStructMatrix.argtypes = [_sz, _sz, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        s.mxSetCell.argtypes = [_vp, _sz, _vp]
        s.mxGetCell.restype = _vp
        s.mxGetCell.argtypes = [_vp, _sz]
        s.mxSetField.argtypes = [_vp, _sz, ctypes.c_char_p, _vp]
        s.mxGetPr.restype = ctypes.POINTER(ctypes.c_double)
        s.mxGetPr.argtypes = [_vp]
        s.mxGetNumberOfDimensions.restype = _sz
        s.mxGetNumberOfDimensions.argtypes = [_vp]
        s.mxGetDimensions.restype = ctypes.POINTER(_sz)
        s.mxGetDimensions.argtypes = [_vp]
        s.mxGetNumberOfElements.restype = _sz
        s.mxGetNumberOfElements.argtypes = [_vp]
        s.mxDestroyArray.argtypes = [_vp]
        s.mxshim_call.restype = ctypes.c_int
        s.mxshim_call.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(_vp), ctypes.c_int,
                                  ctypes.POINTER(_vp)]
        s.mxshim_error_id.restype = ctypes.c_char_p
        s.mxshim_error_msg.restype = ctypes.c_char_p
        self.fn = ctypes.cast(gateway.mexFunction, _vp)

    # -- construction -------------------------------------------------------
    def double(self, a):
        a = np.asarray(a, dtype=np.float64)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        if a.ndim == 1:
            a = a.reshape(1, -1)
        dims = (_sz * a.ndim)(*a.shape)
        mx = self.shim.mxCreateNumericArray(a.ndim, dims, 3, 0)   # mxDOUBLE_CLASS
        flat = np.asfortranarray(a).ravel(order="F")
        pr = self.shim.mxGetPr(mx)
        ctypes.memmove(pr, flat.ctypes.data, flat.nbytes)
        return mx

    def cell(self, items, row=True):
        n = len(items)
        c = self.shim.mxCreateCellMatrix(1 if row else n, n if row else 1)
        for k, it in enumerate(items):
            self.shim.mxSetCell(c, k, it)
        return c

    def struct(self, **fields):
        names = list(fields)
        arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        s = self.shim.mxCreateStructMatrix(1, 1, len(names), arr)
        for n, v in fields.items():
            self.shim.mxSetField(s, 0, n.encode(), v)
        return s

    # -- reading -------------------------------------------------------------
    def to_numpy(self, mx):
        nd = self.shim.mxGetNumberOfDimensions(mx)
        dims = tuple(self.shim.mxGetDimensions(mx)[k] for k in range(nd))
        n = int(np.prod(dims))
        pr = self.shim.mxGetPr(mx)
        flat = np.ctypeslib.as_array(pr, shape=(n,)).copy() if n else np.zeros(0)
        return flat.reshape(dims, order="F")

    def cell_item(self, c, k):
        return self.shim.mxGetCell(c, k)

    # -- calls ---------------------------------------------------------------
    def call(self, nlhs, args):
        plhs = (_vp * max(nlhs, 1))()
        prhs = (_vp * max(len(args), 1))(*args)
        rc = self.shim.mxshim_call(self.fn, nlhs, plhs, len(args), prhs)
        if rc != 0:
            return None, (self.shim.mxshim_error_id().decode(), self.shim.mxshim_error_msg().decode())
        return [plhs[k] for k in range(nlhs)], None


def matlab_h3m(mx: Mx, base: dict, consts: dict, post: dict | None = None, sizes=None):
    """(h3m_b.hmm, h3m_r.hmm, extra full-cov args) as MATLAB values.  ``sizes``:
    per-cluster state counts N2[j] <= S (cluster j keeps its first N2[j] states)."""
    cov = base["covmode"]
    N = base["prior"].shape[0]
    K, S0 = consts["logPi"].shape
    sizes = [S0] * K if sizes is None else [int(x) for x in sizes]
    hb = []
    for i in range(N):
        n = int(base["nstates"][i])
        emit = [mx.struct(centres=mx.double(base["centres"][i, k]),
                          covars=mx.double(base["covars"][i, k]),
                          nin=mx.double(base["centres"].shape[2])) for k in range(n)]
        hb.append(mx.struct(prior=mx.double(base["prior"][i, :n].reshape(n, 1)),
                            A=mx.double(base["A"][i, :n, :n]), emit=mx.cell(emit)))
    hr = []
    for j in range(K):
        S = sizes[j]
        emit = []
        for s in range(S):
            f = dict(m=mx.double(consts["m"][j, s]))
            if cov == 0:
                # the kernel uses v*W; split as v = 1, W = P (any factorisation is equivalent)
                f.update(W=mx.double(consts["P"][j, s]), v=mx.double(1.0),
                         logLambdaTildePlusDdivlamda=mx.double(consts["c"][j, s]))
            emit.append(mx.struct(**f))
        hr.append(mx.struct(logATilde=mx.double(consts["logA"][j, :S, :S]),
                            logPiTilde=mx.double(consts["logPi"][j, :S].reshape(S, 1)),
                            emit=mx.cell(emit)))
    extra = []
    if cov == 1:
        extra = [mx.cell([mx.double(consts["c"][j, :sizes[j]]) for j in range(K)]),
                 mx.cell([mx.double(np.transpose(consts["P"][j, :sizes[j]], (1, 2, 0)))
                          for j in range(K)])]
    return mx.cell(hb), mx.cell(hr), extra


def cluster_consts(consts: dict, j: int, n: int) -> dict:
    """The E-step constants of cluster j alone, its first n states (K = 1)."""
    return {k: np.ascontiguousarray(v[j:j + 1, :n, :n] if k == "logA" else v[j:j + 1, :n])
            for k, v in consts.items() if k in ("logA", "logPi", "m", "P", "c")}

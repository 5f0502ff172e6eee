"""VB-HMM forward-backward on the GPU.

:func:`vbhmm_fb` mirrors src/hmm/vbhmm_fb.m (the ``useMEX`` path, :96-145):
the psi prelude of :54-93 on the host, then the per-sequence scaled
forward-backward of vbhmm_fb_mex.c on the device through the C-ABI
``vbhmm_fb`` (include/vbhmm_fb.h).  It returns the ``fbstats`` fields of
:383-389 with the reference's index order: logrho_Saved / gamma_all as
[K, N, maxT], xi_sum as [K, K, N] (xi_sum[:, :, n][i, j] = from i to j, as
t_sumxi in vbhmm_fb.m:347-355), phi_norm as [N].  There is no CPU path: the
HIP library must load.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np
import torch
from scipy.special import digamma

from . import _capi

F64 = torch.float64


def prelude(varpar: dict) -> dict:
    """vbhmm_fb.m:54-93 (usegroups = 0), :121-122: logLambdaTilde, logATilde,
    logPiTilde, const_denominator and the MEX inputs t_pz1, t_tpztzt1."""
    v = np.asarray(varpar["v"], dtype=np.float64).reshape(-1)
    W = np.asarray(varpar["W"], dtype=np.float64)
    m = np.asarray(varpar["m"], dtype=np.float64)
    K, dim = m.shape
    lLT = np.array([digamma(0.5 * (v[k] + 1.0) - 0.5 * np.arange(1, dim + 1)).sum()
                    + dim * np.log(2.0) + np.log(np.linalg.det(W[k])) for k in range(K)])
    eps = np.asarray(varpar["epsilon"], dtype=np.float64)
    logA = digamma(eps) - digamma(eps.sum(axis=1, keepdims=True))
    alpha = np.asarray(varpar["alpha"], dtype=np.float64).reshape(-1)
    logPi = digamma(alpha) - digamma(alpha.sum())
    return dict(logLambdaTilde=lLT, logATilde=logA, logPiTilde=logPi,
                const_denominator=dim * np.log(2 * np.pi) / 2.0, pz1=np.exp(logPi), A=np.exp(logA))


class SequenceBatch:
    """A ragged batch of observation sequences resident on the GPU:
    offsets [N+1] (int32) and x [sum T][dim] (fp64), as include/vbhmm_fb.h."""

    def __init__(self, data: List[np.ndarray], dim: int, device="cuda"):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("SequenceBatch lives on a GPU (HIP); there is no CPU path")
        lens = [int(np.asarray(a).reshape(-1, dim).shape[0]) for a in data]
        off = np.zeros(len(data) + 1, dtype=np.int32)
        off[1:] = np.cumsum(lens)
        x = (np.concatenate([np.asarray(a, dtype=np.float64).reshape(-1, dim) for a in data])
             if off[-1] > 0 else np.zeros((1, dim)))
        self.N, self.dim, self.maxT = len(data), int(dim), max(lens) if lens else 0
        self.offsets = torch.from_numpy(off).to(self.device)
        self.x = torch.from_numpy(np.ascontiguousarray(x)).to(self.device)

    def desc(self) -> "_capi.SeqsT":
        return _capi.SeqsT(self.N, self.dim, self.maxT, _capi.ptr(self.offsets), _capi.ptr(self.x))


def vbhmm_fb(data, varpar: dict, device="cuda", pre: Optional[dict] = None,
             batch: Optional[SequenceBatch] = None) -> dict:
    """fbstats of vbhmm_fb.m for the sequences ``data`` (list of [T_n x dim]
    arrays) under the variational posterior ``varpar`` (v [K], W [K][dim][dim],
    epsilon [K][K], alpha [K], m [K][dim], beta [K]); K <= 16, dim <= 8."""
    lib = _capi.lib()
    m = np.ascontiguousarray(varpar["m"], dtype=np.float64)
    K, dim = m.shape
    pre = prelude(varpar) if pre is None else pre
    sb = batch if batch is not None else SequenceBatch(data, dim, device)
    dev = sb.device
    t = {k: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)
         for k, a in (("m", m), ("W", varpar["W"]), ("v", np.reshape(varpar["v"], -1)),
                      ("beta", np.reshape(varpar["beta"], -1)),
                      ("lLT", pre["logLambdaTilde"]), ("pz1", pre["pz1"]), ("A", pre["A"]))}
    par = _capi.HmmParamsT(K, dim, *[_capi.ptr(t[k]) for k in ("m", "W", "v", "beta", "lLT",
                                                                 "pz1", "A")],
                           float(pre["const_denominator"]))
    N, T = sb.N, sb.maxT
    logrho = torch.empty((max(T, 1), max(N, 1), K), dtype=F64, device=dev)
    gamma = torch.empty_like(logrho)
    xi = torch.empty((max(N, 1), K, K), dtype=F64, device=dev)
    phi = torch.empty((max(N, 1),), dtype=F64, device=dev)
    sd = sb.desc()
    nb = int(lib.vbhmm_fb_workspace_bytes(ctypes.byref(sd), K))
    ws = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rc = lib.vbhmm_fb(ctypes.byref(sd), ctypes.byref(par), _capi.ptr(logrho), _capi.ptr(gamma),
                      _capi.ptr(xi), _capi.ptr(phi), _capi.ptr(ws), ws.numel(), stream)
    _capi.check(rc, "vbhmm_fb")
    lr = logrho[:T, :N].permute(2, 1, 0).cpu().numpy()     # [K, N, maxT]
    ga = gamma[:T, :N].permute(2, 1, 0).cpu().numpy()
    xs = xi[:N].permute(1, 2, 0).cpu().numpy()             # [K, K, N]
    return dict(logrho_Saved=lr, gamma_all=ga, xi_sum=xs, phi_norm=phi[:N].cpu().numpy(),
                logLambdaTilde=pre["logLambdaTilde"], logPiTilde=pre["logPiTilde"],
                logATilde=pre["logATilde"])

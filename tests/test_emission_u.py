"""The emission GEMM on the prepared base-set operand (vbhem_prepare_base +
emission_u_kernel, csrc/vbhem_emission.hip) against the oracle and against the
previous kernels (raw / generic, which build the operand per column tile from
the covariances): every per-pair output and the fused E-step.

Shapes cover the three register buckets of the kernel (k-steps <= 4, <= 12, <= 40),
one and several W' row chunks (K*S <= 128 and > 128), ragged bases, face-scale
means (the fixed base-mean shift of the prepared operand), and the per-call operand
(prepare=False: built for each call's bases, shifted by the cluster means).
"""
import os

import numpy as np
import pytest
import torch

from cases import make_case
from conftest import RTOL_PAIRS, elem_err, stat_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")

# name: (N, K, S, Sb, d, covmode, extra make_case args)
SHAPES = {
    "diag_d2": (40, 4, 3, 3, 2, 0, {}),            # k-steps 1
    "full_d2_face": (40, 4, 3, 3, 2, 1, dict(face=True, ragged=True, tau=5, Nv=10)),
    "full_d8": (24, 16, 8, 8, 8, 1, {}),           # k-steps 11 (C4 shape)
    "full_d8_rows": (12, 20, 8, 6, 8, 1, {}),      # K*S = 160 > 128: two W' chunks
    "full_d16": (6, 8, 12, 12, 16, 1, dict(tau=6)),  # k-steps 38 (C5 shape), 12 row chunks
    "diag_d12": (10, 6, 5, 4, 12, 0, {}),          # k-steps 6
    # statistics only: > 64 gated pairs per cluster (one block per cluster walks them)
    "full_d4_long": (300, 3, 4, 4, 4, 1, {}),
}


def _pairs(vb, cs, prepare, old=False):
    from vbhem_amd.estep import EStepEngine
    if old:
        os.environ["VBHEM_NO_UGEMM"] = "1"
    try:
        K, S = cs["consts"]["logPi"].shape
        eng = EStepEngine(cs["bs"], K, S, cs["T"], device=DEV, prepare=prepare)
        eng.set_clusters(cs["consts"])
        out = eng.pairs(want_tnu=True)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in out.items()}, eng
    finally:
        os.environ.pop("VBHEM_NO_UGEMM", None)


@pytest.mark.parametrize("name", list(SHAPES))
def test_prepared_operand_pairs(vb, vo, name):
    N, K, S, Sb, d, cov, extra = SHAPES[name]
    cs = make_case(N, K, S, Sb, d, cov, seed=sum(map(ord, name)) % 1000, **extra)
    ref = vo.c_estep_pairs(cs["base"], cs["consts"], cs["T"], nthreads=4, want_tnu=True)
    got, eng = _pairs(vb, cs, prepare=True)
    assert eng._U is not None  # the prepared path ran
    per_call, _ = _pairs(vb, cs, prepare=False)
    old, _ = _pairs(vb, cs, prepare=True, old=True)
    # L_elbo entry by entry; the posterior sums and moments with stat_err's floor
    # (moments of means near the origin cancel: tests/conftest.py)
    for k in KEYS + ("sum_t_nu",):
        err = elem_err if k == "LL_elbo" else stat_err
        assert err(got[k], ref[k]) < RTOL_PAIRS, (name, k, err(got[k], ref[k]))
        assert err(per_call[k], ref[k]) < RTOL_PAIRS, (name, k, err(per_call[k], ref[k]))
        # the three GEMM variants differ only by the shift and summation order
        assert stat_err(got[k], old[k]) < 1e-10, (name, k, stat_err(got[k], old[k]))


@pytest.mark.parametrize("name", ["full_d8", "full_d16", "diag_d2"])
def test_prepared_operand_fused(vb, name):
    """Fused E-step (gated schedule) with the prepared operand vs the per-call one."""
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    N, K, S, Sb, d, cov, extra = SHAPES[name]
    cs = make_case(N, K, S, Sb, d, cov, seed=7 + len(name), **extra)
    outs = []
    for prepare in (True, False):
        eng = EStepEngine(cs["bs"], K, S, cs["T"], device=DEV, prepare=prepare)
        eng.set_clusters(cs["consts"])
        eng.set_log_omega(host.log_omega_tilde(cs["P"].alpha))
        tN = (100.0 * N) * eng.base.omega
        st = eng.fused(tN).cpu().numpy()
        outs.append((st, eng.hatZ.cpu().numpy(), eng.LL.cpu().numpy()))
    for a, b in zip(outs[0], outs[1]):
        assert stat_err(a, b) < 1e-9


def test_prepared_operand_layout(vb):
    """The operand buffer: shift = mean of the valid base means (ragged bases), zero
    padding past the last column, size as vbhem_prepare_base_bytes says."""
    import ctypes
    from vbhem_amd import _capi
    from vbhem_amd.estep import EStepEngine
    cs = make_case(7, 3, 3, 3, 4, 1, seed=5, ragged=True)
    eng = EStepEngine(cs["bs"], 3, 3, cs["T"], device=DEV)
    U = eng._U.cpu().numpy()
    b = cs["base"]
    ns = b["nstates"]
    valid = np.concatenate([b["centres"][i, :ns[i]] for i in range(len(ns))])
    np.testing.assert_allclose(U[:4], valid.mean(axis=0), rtol=1e-13)
    assert np.all(U[4:64] == 0.0)
    kq = (4 * 5 // 2 + 4 + 3) // 4
    ncols = 7 * 3
    ntile = (ncols + 15) // 16
    nu = 1 + 4 + 4 * 5 // 2        # statistic features: 1 | mu' | packed Sigma + mu'mu'
    sbp, nup = 4, 16               # Us block per base: [SB -> 4][NU -> 16]
    nt = 64 + ntile * kq * 64
    assert U.size == nt + 7 * sbp * nup
    assert int(eng.lib.vbhem_prepare_base_bytes(ctypes.byref(eng._bt))) == U.size * 8
    # columns past the end of the base set are zero in every k-step
    tiles = U[64:nt].reshape(ntile, kq, 4, 16)
    last = ncols - 16 * (ntile - 1)
    assert np.all(tiles[-1, :, :, last:] == 0.0)
    # the statistics copy: per base state the ones column, mu' = mu - z, and the packed
    # second moments as in U's k-steps; zero rows / columns past SB and NU
    Us = U[nt:].reshape(7, sbp, nup)
    z = U[:4]
    assert np.all(Us[:, 3:, :] == 0.0) and np.all(Us[:, :, nu:] == 0.0)
    assert np.all(Us[:, :3, 0] == 1.0)
    mu = b["centres"] - z                       # [N][SB][d]
    np.testing.assert_allclose(Us[:, :3, 1:5], mu, rtol=0, atol=1e-12)
    ut = tiles.transpose(0, 3, 1, 2).reshape(ntile * 16, kq * 4)[:ncols]   # [col][e]
    npf = 10
    np.testing.assert_array_equal(Us[:, :3, 5:nu].reshape(ncols, npf), ut[:, :npf])
    np.testing.assert_array_equal(Us[:, :3, 1:5].reshape(ncols, 4), ut[:, npf:npf + 4])
    del _capi


@pytest.mark.parametrize("name", ["full_d8", "full_d16", "diag_d12", "full_d2_face", "full_d4_long"])
@pytest.mark.parametrize("prepare", [True, False])
def test_stats_on_prepared_operand(vb, name, prepare, monkeypatch):
    """Gated statistics from the prepared operand (stats_list_u_kernel, and
    stats_list_g_kernel for small NU: moments read from U and shifted back by z) vs the
    covariance gather (stats_list_kernel), with several
    base groups (the second group adds into the slabs) and fewer blocks than chunks (the
    first group zero-fills the slabs past its grid)."""
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    N, K, S, Sb, d, cov, extra = SHAPES[name]
    N = max(N, 40)
    cs = make_case(N, K, S, Sb, d, cov, seed=11 + len(name), **extra)
    monkeypatch.setenv("VBHEM_GROUP_BASES", str(N // 2 + 1))
    outs = []
    # VBHEM_STATS_U=1: the prepared-operand kernel also where the default picks the
    # covariance path (NU > 64)
    # VBHEM_NO_STATS_G=1: the one-pair-per-wave kernel where the grouped one (small NU)
    # is the default
    # default (prepared): the MFMA kernel on the statistics copy Us, also with one block
    # per cluster (> 64 pairs per wave: the list-base refetch); VBHEM_NO_STATS_M=1: the
    # older prepared-operand kernels
    no_m = {"VBHEM_NO_STATS_M": "1"}
    for env in ({"VBHEM_NO_STATS_U": "1"}, {"VBHEM_STATS_U": "1", **no_m},
                {"VBHEM_STATS_U": "1", "VBHEM_SU_BLOCKS": str(K), **no_m},
                {"VBHEM_STATS_U": "1", "VBHEM_NO_STATS_G": "1", **no_m},
                {}, {"VBHEM_SU_BLOCKS": str(K + 1)}):
        for k in ("VBHEM_NO_STATS_U", "VBHEM_SU_BLOCKS", "VBHEM_STATS_U", "VBHEM_NO_STATS_G",
                  "VBHEM_NO_STATS_M"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        eng = EStepEngine(cs["bs"], K, S, cs["T"], device=DEV, prepare=prepare)
        eng.set_clusters(cs["consts"])
        eng.set_log_omega(host.log_omega_tilde(cs["P"].alpha))
        st = eng.fused((100.0 * N) * eng.base.omega).cpu().numpy()
        outs.append(st)
    assert np.isfinite(outs[0]).all()
    for st in outs[1:]:
        assert stat_err(st, outs[0]) < 1e-10, (name, prepare, stat_err(st, outs[0]))


@pytest.mark.parametrize("N", [37, 2001, 12500])
def test_row_split_bit_identical(vb, monkeypatch, N):
    """The one-chunk GEMM in half-tiles (small base counts, e.g. a 12,500-base shard:
    each wave takes 4 of a tile's 8 row tiles) computes every E entry with the same MFMA
    chain as the whole-tile kernel: the fused E-step's outputs are bit-identical with the
    split forced on and off (VBHEM_EM_SPLIT), at C4's shape."""
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload("C4", N=N, device=DEV)
    consts = host.cluster_constants(P, base.covmode)
    outs = []
    for split in ("0", "1"):
        monkeypatch.setenv("VBHEM_EM_SPLIT", split)
        eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
        eng.set_clusters(consts)
        eng.set_log_omega(host.log_omega_tilde(P.alpha))
        tN = (100.0 * N) * eng.base.omega
        outs.append((eng.fused(tN).clone(), eng.LL.clone(), eng.hatZ.clone()))
        del eng
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,N", [("C4", 12500), ("C3", 4000)])
@pytest.mark.parametrize("switch", ["VBHEM_EM_NOBST", "VBHEM_RESP_GENERIC"])
def test_store_paths_bit_identical(vb, monkeypatch, cfg, N, switch):
    """The one-chunk emission GEMM's buffer stores (lanes outside the tile dropped by an
    out-of-range offset) and resp_kernel's K-templated path (unrolled group reductions,
    buffer stores of hat_Z / Z) write exactly what the branched paths write: the fused
    E-step's outputs are bit-identical with VBHEM_EM_NOBST / VBHEM_RESP_GENERIC set and
    unset (both read at launch), C4's shape (K = 16) and C3's (K = 8)."""
    from vbhem_amd import host
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload(cfg, N=N, device=DEV)
    consts = host.cluster_constants(P, base.covmode)
    outs = []
    for on in (False, True):
        if on:
            monkeypatch.setenv(switch, "1")
        else:
            monkeypatch.delenv(switch, raising=False)
        eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
        eng.set_clusters(consts)
        eng.set_log_omega(host.log_omega_tilde(P.alpha))
        tN = (100.0 * N) * eng.base.omega
        outs.append((eng.fused(tN).clone(), eng.LL.clone(), eng.hatZ.clone()))
        del eng
    for a, b in zip(*outs):
        assert torch.equal(a, b)

"""GPU parity of the HIP E-step (through the C-ABI) against the oracle.

* per-pair MEX outputs (vbhem_estep_pairs) over every shape in cases.SHAPES;
* fused statistics / hat_Z / L_elbo (vbhem_estep_fused) over the same shapes;
* the exact fallback (forced by an adversarial cluster whose factorised
  log-sum-exp normaliser underflows);
* the host-pointer entry point the MEX gateway uses;
* full-size (C4, N = 100,000) size-independent properties: determinism, shard
  additivity, normalisation and mass rules, and a sampled oracle comparison.

Tolerances (elementwise unless noted; conftest.elem_err / hatz_err / post_err):
per-pair outputs RTOL_PAIRS = 1e-10 (normwise, and elementwise with a 1e-8
relative floor); statistics 1e-9; hat_Z / posteriors / ELBO the north-star
1e-5 (hat_Z entries below 1e-8 absolutely).
"""
import ctypes
import zlib

import numpy as np
import pytest
import torch

from cases import SHAPES, make_case
from conftest import RTOL_NORTH_STAR, RTOL_PAIRS, elem_err, hatz_err, post_err, rel_err, stat_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
PAIR_KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")


def engine(vb, base_np, consts, T, K=None, S=None):
    from vbhem_amd.estep import EStepEngine
    K0, S0 = consts["logPi"].shape
    eng = EStepEngine(vb.BaseSet.from_numpy(base_np), K0, S0, T, device=DEV)
    eng.set_clusters(consts)
    return eng


def seed_of(name):
    return zlib.crc32(name.encode()) % 1000


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_pairs_match_oracle(vb, vo, shape):
    name, N, K, S, Sb, d, cov, T, ragged = shape
    cs = make_case(N, K, S, Sb, d, cov, seed=seed_of(name), ragged=ragged, tau=T)
    ref = vo.c_estep_pairs(cs["base"], cs["consts"], T, nthreads=4, want_tnu=True)
    eng = engine(vb, cs["base"], cs["consts"], T)
    got = eng.pairs(want_tnu=True)
    torch.cuda.synchronize()
    for k in PAIR_KEYS + ("sum_t_nu",):
        g = got[k].cpu().numpy()
        e = rel_err(g, ref[k])
        assert e < RTOL_PAIRS, (name, k, e)
        e = stat_err(g, ref[k])
        assert e < 1e-8, (name, k, e)


@pytest.fixture(params=["gated", "dense"])
def fused_mode(request):
    """Run a fused test under both schedules (VBHEM_FUSED_GATED / _DENSE)."""
    from vbhem_amd import _capi
    prev = _capi.set_fused_mode(_capi.FUSED_GATED if request.param == "gated" else _capi.FUSED_DENSE)
    yield request.param
    _capi.set_fused_mode(prev)


@pytest.fixture(params=[("gated", 100.0), ("dense", 100.0), ("gated", 1e-9)],
                ids=["gated-Nv100", "dense-Nv100", "gated-allgated"])
def mode_tscale(request):
    """(schedule, tscale): the all-gated edge case targets the gated schedule only."""
    from vbhem_amd import _capi
    mode, tscale = request.param
    prev = _capi.set_fused_mode(_capi.FUSED_GATED if mode == "gated" else _capi.FUSED_DENSE)
    yield tscale
    _capi.set_fused_mode(prev)


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_fused_matches_oracle(vb, vo, shape, mode_tscale):
    """tscale = Nv: 100 (the configs' virtual samples: Z mostly one-hot, the gate
    drops most pairs) and 1e-9 (every Z < 1e-8: no pair passes the gate)."""
    name, N, K, S, Sb, d, cov, T, ragged = shape
    tscale = mode_tscale
    cs = make_case(N, K, S, Sb, d, cov, seed=seed_of(name) + 1, ragged=ragged, tau=T)
    base, consts = cs["base"], cs["consts"]
    pairs = vo.c_estep_pairs(base, consts, T, nthreads=4)
    tN = tscale * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, cov)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    vec = eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy()
    got = vb.host.unpack_stats(vec, K, S, d, cov)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, (name, k, stat_err(got[k], st[k]))
    Lt1 = float((Z * pairs["LL_elbo"]).sum())
    Lt7 = float((hz * np.log(hz)).sum())
    assert abs(got["Lt1"] - Lt1) <= 1e-10 * abs(Lt1)
    assert abs(got["Lt7"] - Lt7) <= 1e-9 * abs(Lt7) + 1e-9
    assert hatz_err(eng.hatZ.cpu().numpy(), hz) < RTOL_NORTH_STAR
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


def test_fused_multigroup(vb, vo, fused_mode, monkeypatch):
    """The fused call split into several base groups (VBHEM_GROUP_BASES: E, the
    per-pair scratch and the gate lists are per group; the slabs accumulate)."""
    name, N, K, S, Sb, d, cov, T = "multigroup", 300, 6, 5, 4, 3, 1, 7
    monkeypatch.setenv("VBHEM_GROUP_BASES", "64")
    monkeypatch.setenv("VBHEM_NSLAB", "7")
    cs = make_case(N, K, S, Sb, d, cov, seed=seed_of(name), ragged=True, tau=T)
    base, consts = cs["base"], cs["consts"]
    pairs = vo.c_estep_pairs(base, consts, T, nthreads=4)
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, cov)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, cov)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k
    assert hatz_err(eng.hatZ.cpu().numpy(), hz) < RTOL_NORTH_STAR
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.parametrize("S,Sb,d,cov", [(5, 5, 2, 0), (3, 3, 2, 1), (6, 4, 4, 0)])
def test_k1_in_recursion_kernels(vb, vo, S, Sb, d, cov, monkeypatch):
    """Gated schedule with a short K1 (kdp <= 8: d = 2 full, d <= 4 diag -- C2, C3):
    fb_bwd2_kernel and fb_split_kernel's list mode evaluate E from the prepared
    operand, with no emission GEMM and no E buffer.  Statistics, hat_Z and L_elbo
    against the oracle, and against the same call through the emission GEMM
    (VBHEM_NO_K1_IN_KERNEL=1): the same sums blocked differently, equal to rounding."""
    from vbhem_amd import _capi
    prev = _capi.set_fused_mode(_capi.FUSED_GATED)
    try:
        N, K, T = 777, 5, 10
        cs = make_case(N, K, S, Sb, d, cov, seed=17 + S, ragged=True, tau=T)
        base, consts = cs["base"], cs["consts"]
        pairs = vo.c_estep_pairs(base, consts, T, nthreads=8)
        tN = 100.0 * N * base["omega"]
        logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
        st = vo.c_statistics(Z, pairs, cov)
        out = {}
        for label in ("in_kernel", "gemm"):
            if label == "gemm":
                monkeypatch.setenv("VBHEM_NO_K1_IN_KERNEL", "1")
            eng = engine(vb, base, consts, T)
            eng.set_log_omega(logOmega)
            raw = eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy()
            out[label] = (vb.host.unpack_stats(raw, K, S, d, cov), eng.LL.cpu().numpy(),
                          eng.hatZ.cpu().numpy())
            del eng
        got, LL, hzg = out["in_kernel"]
        for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
            assert stat_err(got[k], st[k]) < 1e-9, k
            assert stat_err(got[k], out["gemm"][0][k]) < 1e-12, k
        assert elem_err(LL, pairs["LL_elbo"]) < RTOL_PAIRS
        assert elem_err(LL, out["gemm"][1]) < 1e-13
        assert hatz_err(hzg, hz) < RTOL_NORTH_STAR
    finally:
        _capi.set_fused_mode(prev)


@pytest.mark.parametrize("S,Sb,d,cov,adv,N,group", [
    (5, 5, 2, 0, False, 333, None), (3, 3, 2, 1, False, 333, None), (4, 4, 1, 1, False, 333, None),
    (6, 4, 4, 0, False, 333, None), (4, 4, 2, 1, True, 333, None), (5, 3, 2, 0, True, 333, None),
    (5, 5, 2, 0, False, 40000, None), (5, 5, 2, 0, True, 5000, None), (5, 5, 2, 0, False, 5000, 1200)])
def test_bwd2_in_kernel_prep(vb, vo, S, Sb, d, cov, adv, N, group, monkeypatch):
    """emission_prep_kernel's work inside fb_bwd2_kernel (SplitArgs::prep: the short-K1
    gated schedule on a prepared operand, C2 / C3): W', bias', A' computed per block with
    the same arithmetic, the fallback counters zeroed in the kernel unless the previous
    call left them closed (vbhem_internal.h kFlagPre); 6 to 512 statistics chunks,
    several base groups with `group`.  Bit for bit the launch path's outputs
    (VBHEM_NO_BWD2_PREP=1) over repeated calls, after a call on the other path (its
    zeroed head), after garbage in the counters with the tag cleared and after garbage
    in the whole workspace; the fallback count with them.  adv: cluster 0 underflows
    for every base (both passes flag it; the exact fallback runs inside the steps)."""
    from vbhem_amd import _capi
    if group:
        monkeypatch.setenv("VBHEM_GROUP_BASES", str(group))
    prev = _capi.set_fused_mode(_capi.FUSED_GATED)
    try:
        K, T = 4, 6 if adv else 10
        if adv:
            cs, consts = adversarial_case(cov, S=S, Sb=Sb, d=d, N=N, K=K, T=T)
            consts["c"][1:] = 1.0e4  # cluster 0 wins (gated) for every base
        else:
            cs = make_case(N, K, S, Sb, d, cov, seed=5 + S + d, ragged=True, tau=T)
            consts = cs["consts"]
        base = cs["base"]
        tN = torch.as_tensor(100.0 * N * base["omega"], device=DEV)
        logOmega = np.log(np.full(K, 1.0 / K))

        def run(eng):
            eng.fused(tN)
            torch.cuda.synchronize()
            return (eng.stats.cpu().numpy().copy(), eng.LL.cpu().numpy().copy(),
                    eng.hatZ.cpu().numpy().copy(), eng.fallback_count())

        monkeypatch.setenv("VBHEM_NO_BWD2_PREP", "1")
        e0 = engine(vb, base, consts, T)
        e0.set_log_omega(logOmega)
        ref = run(e0)
        del e0
        monkeypatch.delenv("VBHEM_NO_BWD2_PREP")
        eng = engine(vb, base, consts, T)
        eng.set_log_omega(logOmega)
        outs = [run(eng), run(eng)]
        monkeypatch.setenv("VBHEM_NO_BWD2_PREP", "1")
        outs.append(run(eng))  # the launch path: its head zeroed, tag included
        monkeypatch.delenv("VBHEM_NO_BWD2_PREP")
        outs.append(run(eng))
        head = eng._ws_fused.view(torch.int32)
        head[:2] = 0               # the tag cleared ...
        head[4:8] = 987654         # ... and garbage in the counters
        outs.append(run(eng))
        eng._ws_fused.fill_(1)     # garbage everywhere: tag, counters, chunk flags, buffers
        outs.append(run(eng))
        outs.append(run(eng))
        for o in outs:
            for a, b in zip(o[:3], ref[:3]):
                assert np.array_equal(a, b, equal_nan=True)
            assert o[3] == ref[3]
        if adv:
            assert ref[3] >= N
        else:
            assert ref[3] == 0
    finally:
        _capi.set_fused_mode(prev)


def adversarial_case(cov=1, S=4, Sb=4, d=3, N=4, K=3, T=6):
    """Cluster 0's transitions put all mass on sigma+1 while its emissions put
    all mass on state 0: the factorised normaliser Z ~ e^-600 underflows the
    safe range (kZMin = 1e-200), so those pairs take the exact fallback."""
    cs = make_case(N, K, S, Sb, d, cov, seed=99, tau=T)
    c = {k: np.array(v, copy=True) for k, v in cs["consts"].items()}
    lA = np.full((S, S), -600.0)
    for r in range(S):
        lA[r, (r + 1) % S] = 0.0
    c["logA"][0] = lA
    c["c"][0] = 1200.0
    c["c"][0, 0] = 0.0
    return cs, c


@pytest.mark.parametrize("cov", [0, 1])
def test_exact_fallback_pairs(vb, vo, cov):
    cs, consts = adversarial_case(cov)
    T = cs["T"]
    ref = vo.c_estep_pairs(cs["base"], consts, T, want_tnu=True)
    eng = engine(vb, cs["base"], consts, T)
    got = eng.pairs(want_tnu=True)
    nfb = eng.fallback_count()
    assert nfb > 0
    for k in PAIR_KEYS + ("sum_t_nu",):
        assert rel_err(got[k].cpu().numpy(), ref[k]) < RTOL_PAIRS, k


@pytest.mark.parametrize("env", [{}, {"VBHEM_NO_FOLD_EXACT": "1"}])
def test_exact_fallback_large_states(vb, vo, env, monkeypatch):
    """S = 20, Sb = 18: a flagged pair's small arrays (6 S Sb + S^2 + Sb doubles) no
    longer fit the wavefront's LDS region, so exact_pair_wave keeps them in the tail of
    its global scratch slot (agent-scope fences between its exchange steps)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cs, consts = adversarial_case(1, S=20, Sb=18, d=3, N=6, K=2, T=5)
    consts["c"][1:] = 1.0e4
    base, T = cs["base"], cs["T"]
    N, K, S, d = 6, 2, 20, 3
    ref = vo.c_estep_pairs(base, consts, T, want_tnu=True)
    eng = engine(vb, base, consts, T)
    got = eng.pairs(want_tnu=True)
    assert eng.fallback_count() > 0
    for k in PAIR_KEYS + ("sum_t_nu",):
        assert rel_err(got[k].cpu().numpy(), ref[k]) < RTOL_PAIRS, k
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(ref["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, ref, 1)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k


def test_exact_fallback_fused(vb, vo, fused_mode):
    cs, consts = adversarial_case(1)
    base, T = cs["base"], cs["T"]
    N, K = base["prior"].shape[0], consts["logPi"].shape[0]
    S, d = consts["logPi"].shape[1], base["centres"].shape[2]
    pairs = vo.c_estep_pairs(base, consts, T)
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, 1)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    assert eng.fallback_count() > 0
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k


@pytest.mark.parametrize("N,K", [(4, 1), (300, 2), (3000, 2)])
@pytest.mark.parametrize("env", [{}, {"VBHEM_NO_FOLD_EXACT": "1"}, {"VBHEM_NO_STATS_M": "1"},
                                 {"VBHEM_NO_LIST_INLINE": "1"}])
def test_exact_fallback_gated_pairs(vb, vo, N, K, env, monkeypatch):
    """The adversarial cluster wins every base (the other cluster's emissions are far
    worse), so its pairs are flagged by the backward pass AND are gated: the gate-list
    pass flags them again.  Default: the backward pass's fallback folded into resp_kernel
    (several chunks at N = 300), the list pass's recomputed by the list kernel itself
    (fb_split_kernel, S = 4: SplitArgs::xinline); VBHEM_NO_LIST_INLINE: an fb_exact_kernel
    launch for the list pass's instead; VBHEM_NO_FOLD_EXACT: a launch after each pass;
    VBHEM_NO_STATS_M: the other statistics kernels."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cs, consts = adversarial_case(1, N=N, K=K)
    if K > 1:
        consts["c"][1:] = 1.0e4
    base, T = cs["base"], cs["T"]
    S, d = consts["logPi"].shape[1], base["centres"].shape[2]
    pairs = vo.c_estep_pairs(base, consts, T)
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    assert (Z[:, 0] > 1e-8).all()  # the flagged cluster is gated for every base
    st = vo.c_statistics(Z, pairs, 1)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    assert eng.fallback_count() >= 2 * N  # both passes flagged cluster 0 of every base
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.parametrize("env", [{}, {"VBHEM_NO_FOLD_EXACT": "1"}, {"VBHEM_NO_LIST_INLINE": "1"}])
@pytest.mark.parametrize("S,N", [(8, 41), (8, 5000), (12, 41)])
def test_exact_fallback_mfma_kernels(vb, vo, env, monkeypatch, S, N):
    """The adversarial cluster at S = Sb = 8 (12), T = 10: its pairs underflow in the
    MFMA backward pass (fb_bwd4_kernel / fb_bwd12_kernel) and, being gated, again in
    the gate-list pass (fb_list4_kernel / fb_list12_kernel); both passes' flags reach
    the exact fallback (folded into the consumers -- fb_list4_kernel's from its per-wave
    queue; at N = 5000 waves hold two items, 8 queued pairs -- or fb_exact_kernel
    launches)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    K = 2
    cs, consts = adversarial_case(1, S=S, Sb=S, d=3, N=N, K=K, T=10)
    consts["c"][1:] = 1.0e4
    base, T = cs["base"], cs["T"]
    d = 3
    pairs = vo.c_estep_pairs(base, consts, T)
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    assert (Z[:, 0] > 1e-8).all()
    st = vo.c_statistics(Z, pairs, 1)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    assert eng.fallback_count() >= 2 * N
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.parametrize("shift", [8.0e5, -8.0e5])
@pytest.mark.parametrize("S", [8, 12])
def test_range_check_mfma_kernels(vb, vo, S, shift):
    """Cluster 0's emission constants shifted by |shift| > the kernels' |V| limit (7e5):
    no underflow, only the per-tile range check (|E|, |Ef| >= vlim as ordered compare
    masks, VBHEM_RANGE_CMP) flags its pairs in the MFMA kernels (fb_bwd4_kernel /
    fb_bwd12_kernel, and the list kernels when the cluster is gated), and the exact
    fallback must give the oracle's numbers."""
    N, K, d = 41, 2, 3
    cs = make_case(N, K, S, S, d, 1, seed=7, tau=10)
    consts = {k: np.array(v, copy=True) for k, v in cs["consts"].items()}
    consts["c"][0] += shift
    base, T = cs["base"], cs["T"]
    pairs = vo.c_estep_pairs(base, consts, T)
    assert np.isfinite(pairs["LL_elbo"]).all()
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, 1)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    assert eng.fallback_count() >= N  # every pair of cluster 0 failed the range check
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


def _emission(base, consts):
    """E[i, j, sigma, beta] of mex.c:715-865 (full covariance), numpy."""
    mu, Sg = base["centres"], base["covars"]
    m, P, c = consts["m"], consts["P"], consts["c"]
    d = mu.shape[-1]
    diff = mu[:, None, None, :, :] - m[None, :, :, None, :]          # [N][K][S][SB][d]
    quad = np.einsum("nksbx,ksxy,nksby->nksb", diff, P, diff)
    tr = np.einsum("ksxy,nbyx->nksb", P, Sg)
    return -0.5 * (d * np.log(2 * np.pi) + c[None, :, :, None] + tr + quad)


@pytest.mark.parametrize("env", [{}, {"VBHEM_NO_FOLD_EXACT": "1"}])
@pytest.mark.parametrize("case", ["near", "far", "rowsum", "far+rowsum"])
@pytest.mark.parametrize("S", [8, 12])
def test_range_check_exact_flags(vb, vo, S, case, env, monkeypatch):
    """The per-tile range check of the MFMA kernels flags exactly the pairs it must
    (ADVICE r05): one base state of one base pushed towards or out of range -- its E
    column made very negative through that state's covariance (every cluster shares one
    precision, so every E entry of the column lands in a chosen window) -- and / or one
    base row of A summing to 1.5.  Windows: "near" |E| in [1.1e4, 5e4], large but
    inside the integer maxima's limit (7e5 / T - 3): nothing flagged; "far" |E| >= 8e4,
    past it, so the backward pass flags the base's K pairs and the gate-list pass its
    gated ones again; "rowsum" flags the row's base in both passes.  The fallback count
    must equal that exactly, and every output must be the oracle's."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    N, K, d, T = 41, 3, 3, 10
    cs = make_case(N, K, S, S, d, 1, seed=9, tau=T)
    base = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in cs["base"].items()}
    consts = {k: np.array(v, copy=True) for k, v in cs["consts"].items()}
    consts["P"][:] = consts["P"][0, 0]          # one precision: E columns move together
    i0, b0, i1 = 17, 3, 29
    if "near" in case or "far" in case:
        trP = float(np.trace(consts["P"][0, 0]))
        E0 = _emission(base, consts)[i0, :, :, b0]
        target = 3.0e4 if "near" in case else 1.6e5
        lam = 2.0 * (target + E0.mean()) / trP
        base["covars"][i0, b0] += lam * np.eye(d)
        E1 = _emission(base, consts)[i0, :, :, b0]
        lo, hi = (1.1e4, 5.0e4) if "near" in case else (8.0e4, 1e9)
        assert (-E1 >= lo).all() and (-E1 <= hi).all(), (E1.min(), E1.max())
    if "rowsum" in case:
        base["A"][i1, 2] *= 1.5 / base["A"][i1, 2].sum()
    pairs = vo.c_estep_pairs(base, consts, T)
    assert np.isfinite(pairs["LL_elbo"]).all()
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, 1)
    eng = engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    got = vb.host.unpack_stats(eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy(), K, S, d, 1)
    gated = (Z > 1e-8)
    expect = 0
    if "far" in case:
        expect += K + int(gated[i0].sum())
    if "rowsum" in case:
        expect += K + int(gated[i1].sum())
    assert eng.fallback_count() == expect
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, k
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


def test_host_pointer_entry_point(vb, vo, capi_lib):
    """vbhem_estep_pairs_host (what the MEX gateway calls): host arrays in/out."""
    from vbhem_amd import _capi
    cs = make_case(5, 3, 4, 3, 3, 1, seed=12, ragged=True, tau=7)
    base, consts, T = cs["base"], cs["consts"], 7
    N, K, S, SB, d = 5, 3, 4, 3, 3
    keep = {k: np.ascontiguousarray(base[k], dtype=np.float64)
            for k in ("prior", "A", "centres", "covars")}
    ns = np.ascontiguousarray(base["nstates"], dtype=np.int32)
    ck = {k: np.ascontiguousarray(consts[k], dtype=np.float64) for k in ("logA", "logPi", "m", "P", "c")}
    b = _capi.BaseT(N, SB, d, 1, ns.ctypes.data, keep["prior"].ctypes.data, keep["A"].ctypes.data,
                    keep["centres"].ctypes.data, keep["covars"].ctypes.data)
    c = _capi.ClusterT(K, S, *[ck[k].ctypes.data for k in ("logA", "logPi", "m", "P", "c")])
    out = dict(LL_elbo=np.zeros((N, K)), sum_nu_1=np.zeros((N, K, S)), emit_pr=np.zeros((N, K, S)),
               emit_mu=np.zeros((N, K, S, d)), emit_Mu=np.zeros((N, K, S, d, d)),
               sum_xi=np.zeros((N, K, S, S)))
    rc = capi_lib.vbhem_estep_pairs_host(0, ctypes.byref(b), ctypes.byref(c), T,
                                         *[out[k].ctypes.data for k in ("LL_elbo", "sum_nu_1", "emit_pr",
                                                                        "emit_mu", "emit_Mu", "sum_xi")])
    assert rc == 0, capi_lib.vbhem_last_error()
    ref = vo.c_estep_pairs(base, consts, T)
    for k in PAIR_KEYS:
        assert rel_err(out[k], ref[k]) < RTOL_PAIRS, k


def test_side_stream_and_timing(vb, vo):
    from vbhem_amd import _capi
    cs = make_case(64, 4, 3, 3, 2, 1, seed=13, tau=10)
    eng = engine(vb, cs["base"], cs["consts"], 10)
    ref = vo.c_estep_pairs(cs["base"], cs["consts"], 10)
    _capi.timing_enable(True)
    try:
        s = torch.cuda.Stream(device=DEV)
        with torch.cuda.stream(s):
            got = eng.pairs()
        s.synchronize()
        t = _capi.timing_read()
    finally:
        _capi.timing_enable(False)
    assert t["fb_launches"] >= 1 and t["fb_pairs"] == 64 * 4 and t["fb_ms"] > 0
    assert rel_err(got["LL_elbo"].cpu().numpy(), ref["LL_elbo"]) < RTOL_PAIRS


def test_empty_shard(vb):
    cs = make_case(3, 2, 3, 3, 2, 1, seed=1)
    base = {k: (v[:0] if isinstance(v, np.ndarray) else v) for k, v in cs["base"].items()}
    eng = engine(vb, base, cs["consts"], 5)
    eng.set_log_omega(np.zeros(2))
    eng.stats.fill_(7.0)                 # the output must be overwritten with zeros
    vec = eng.fused(torch.zeros(0, dtype=torch.float64, device=DEV)).cpu().numpy()
    assert np.all(vec == 0)
    out = eng.pairs()
    assert out["LL_elbo"].shape == (0, 2)


# ----------------------------------------------------------------------------
# full size: C4 (N = 100,000, K = 16, S = Sb = d = 8, full covariances, tau = 10)
# ----------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c4_full(vb):
    from vbhem_amd.em import tilde_n
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload("C4", device=DEV)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    consts = vb.host.cluster_constants(P, 1)
    eng.set_clusters(consts)
    eng.set_log_omega(vb.host.log_omega_tilde(P.alpha))
    tN = tilde_n(eng, opt["Nv"], base.N)
    return dict(base=base, P=P, opt=opt, eng=eng, consts=consts, tN=tN)


def test_c4_deterministic(c4_full):
    eng, tN = c4_full["eng"], c4_full["tN"]
    a = eng.fused(tN).clone()
    hz_a = eng.hatZ.clone()
    b = eng.fused(tN).clone()
    assert torch.equal(a, b)
    assert torch.equal(hz_a, eng.hatZ)
    assert eng.fallback_count() == 0


def test_c4_gated_matches_dense(c4_full):
    """Both fused schedules at full size: same statistics, hat_Z and L_elbo up to
    rounding (sums in a different order; the gated backward pass uses the
    table-driven log, <= 1 ulp like log_pos)."""
    from vbhem_amd import _capi
    eng, tN = c4_full["eng"], c4_full["tN"]
    prev = _capi.set_fused_mode(_capi.FUSED_GATED)
    try:
        g = eng.fused(tN).clone()
        hz, LL = eng.hatZ.clone(), eng.LL.clone()
        _capi.set_fused_mode(_capi.FUSED_DENSE)
        d = eng.fused(tN).clone()
    finally:
        _capi.set_fused_mode(prev)
    assert rel_err(g.cpu().numpy(), d.cpu().numpy()) < 1e-10
    assert rel_err(LL.cpu().numpy(), eng.LL.cpu().numpy()) < 1e-13
    assert rel_err(hz.cpu().numpy(), eng.hatZ.cpu().numpy()) < 1e-9


def test_c4_shard_additivity(vb, c4_full):
    """Shards combine by summation (the multi-GPU all-reduce contract)."""
    from vbhem_amd.estep import EStepEngine
    base, P, opt, tN = c4_full["base"], c4_full["P"], c4_full["opt"], c4_full["tN"]
    full = c4_full["eng"].fused(tN).clone()
    acc = torch.zeros_like(full)
    N = base.N
    for lo, hi in ((0, 37_123), (37_123, N)):
        e = EStepEngine(base.shard(lo, hi), P.K, P.S, opt["tau"], device=DEV)
        e.set_clusters(c4_full["consts"])
        e.set_log_omega(vb.host.log_omega_tilde(P.alpha))
        acc += e.fused(tN[lo:hi])
        del e
    assert rel_err(acc.cpu().numpy(), full.cpu().numpy()) < 1e-12


def test_c4_normalisation_and_mass(vb, c4_full):
    eng, tN, P = c4_full["eng"], c4_full["tN"], c4_full["P"]
    vec = eng.fused(tN).cpu().numpy()
    st = vb.host.unpack_stats(vec, P.K, P.S, 8, 1)
    hz = eng.hatZ.cpu().numpy()
    # log_Z = tilde_N (logOmega + L_elbo) ~ 1e5..1e6 carries ~1e-11 absolute rounding,
    # so rows sum to 1 within ~1e-12 (the oracle behaves the same)
    np.testing.assert_allclose(hz.sum(1), 1.0, rtol=1e-10)
    assert abs(st["Nj"].sum() - tN.sum().item()) <= 1e-10 * tN.sum().item()
    assert np.isfinite(vec).all()
    # symmetric second moments, positive occupancies
    assert (st["Nr"] >= 0).all()
    LL = eng.LL.cpu().numpy()
    assert np.isfinite(LL).all() and (LL < 0).all()


def test_c4_sampled_oracle(vb, vo, c4_full):
    eng, base, consts = c4_full["eng"], c4_full["base"], c4_full["consts"]
    eng.fused(c4_full["tN"])
    LL = eng.LL.cpu().numpy()
    idx = np.random.default_rng(0).choice(base.N, 48, replace=False)
    sub = {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim and v.shape[0] == base.N else v)
           for k, v in base.shard(0, base.N).numpy().items()}
    ref = vo.c_estep_pairs(sub, consts, c4_full["opt"]["tau"], nthreads=8)
    assert elem_err(LL[idx], ref["LL_elbo"]) < RTOL_PAIRS


def test_c4_em_iterations_vs_oracle_sample(vb, vo):
    """Three EM iterations on a 2,000-base C4 slice: GPU EM vs oracle EM."""
    from vbhem_amd.em import vbhem_h3m_c_step_fc
    from vbhem_amd.estep import EStepEngine
    from cases import post_dict
    base, P, opt = vb.synth_workload("C4", N=2000)
    opt = dict(opt, max_iter=3)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    res = vbhem_h3m_c_step_fc(P, eng, opt)
    ref = vo.em_step_fc(post_dict(P), base.numpy(), opt)
    np.testing.assert_allclose(res.LogLs, ref["LogLs"], rtol=RTOL_NORTH_STAR)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert post_err(getattr(res.post, k), ref["post"][k]) < RTOL_NORTH_STAR, k
    assert hatz_err(res.hatZ.cpu().numpy(), ref["hat_Z"]) < RTOL_NORTH_STAR


# ----------------------------------------------------------------------------
# VHEM sibling (vhem_estep_pairs, hem_hmm_bwd_fwd_mex.c) against its oracle
# ----------------------------------------------------------------------------
from test_oracle import VHEM_SHAPES  # noqa: E402


@pytest.mark.parametrize("shape", VHEM_SHAPES, ids=[s[0] for s in VHEM_SHAPES])
def test_vhem_pairs_match_oracle(vb, vo, shape):
    from cases import make_reduced
    name, N, K, S, Sb, d, cov, T, ragged, smooth, zt = shape
    seed = seed_of(name)
    cs = make_case(N, K, S, Sb, d, cov, seed=seed, ragged=ragged, tau=T)
    red = make_reduced(K, S, d, cov, seed=seed, zero_transition=zt)
    ref = vo.c_vhem_estep_pairs(cs["base"], red, T, smooth, nthreads=4, want_tnu=True)
    eng = engine(vb, cs["base"], vb.host.vhem_cluster_constants(red, cov), T)
    got = eng.pairs(want_tnu=True, smooth=smooth)
    torch.cuda.synchronize()
    for k in PAIR_KEYS + ("sum_t_nu",):
        e = rel_err(got[k].cpu().numpy(), ref[k])
        assert e < RTOL_PAIRS, (name, k, e)


def test_vhem_rejects_bad_smooth(vb):
    from vbhem_amd import _capi
    from cases import make_reduced
    cs = make_case(3, 2, 2, 2, 2, 1, seed=5, tau=4)
    eng = engine(vb, cs["base"], vb.host.vhem_cluster_constants(make_reduced(2, 2, 2, 1), 1), 4)
    for bad in (0.0, -1.0, float("nan")):
        with pytest.raises(_capi.VbhemError):
            eng.pairs(smooth=bad)

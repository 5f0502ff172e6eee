"""Parity at the scales the synthetic grids and the demo actually run at.

* face scale (demo/vbdemo_face.m:49-61): means around [256, 192] px with ~30 px
  spread, W0 = 0.001, v0 = 10, Nv = 10, tau = 5, d = 2 full, S in {1, 2, 3},
  ragged base HMMs.  This pins the shifted, expanded quadratic form of the
  emission GEMM where |mu| is large next to the spread
  (hard part 3): per-pair outputs, the fused E-step and an EM
  run against the oracle;
* C3 at its full size (N = 10,000, K = 8, S = 5, d = 2 diag): every pair's
  L_elbo, hat_Z and the statistics against the oracle;
* a C5 slice (N = 1,000 of the 10^6 bases, K = 32, S = 12, d = 16 full): the
  MFMA emission path for d > 8 at more than one MFMA tile, against the oracle.

Tolerances are elementwise (conftest.elem_err / hatz_err / stat_err / post_err).
"""
import numpy as np
import pytest
import torch

from cases import make_case, post_dict
from conftest import RTOL_NORTH_STAR, RTOL_PAIRS, elem_err, hatz_err, post_err, stat_err

DEV = "cuda:0"
PAIR_KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")


def face_case(S, seed, N=80, K=4):
    return make_case(N, K, S, 3, 2, 1, seed=seed, ragged=True, tau=5, face=True, Nv=10)


def _engine(vb, base, consts, T, K=None, S=None):
    from vbhem_amd.estep import EStepEngine
    K0, S0 = consts["logPi"].shape
    eng = EStepEngine(vb.BaseSet.from_numpy(base) if isinstance(base, dict) else base, K0, S0, T,
                      device=DEV)
    eng.set_clusters(consts)
    return eng


def test_face_scale_oracle_twin(vo):
    """CPU: the two oracle restatements agree at face scale as well."""
    for S in (1, 2, 3):
        cs = face_case(S, seed=70 + S, N=12)
        c = vo.c_estep_pairs(cs["base"], cs["consts"], cs["T"], want_tnu=True)
        t = vo.twin_estep_pairs(cs["base"], cs["post"], cs["consts"], cs["T"])
        for k in PAIR_KEYS:
            assert stat_err(c[k], t[k]) < 1e-10, (S, k, stat_err(c[k], t[k]))
        # the quadratic form is large: |E| reaches hundreds of nats here
        assert np.abs(c["LL_elbo"]).max() > 10.0


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 2, 3])
def test_face_scale_pairs(vb, vo, S):
    cs = face_case(S, seed=60 + S)
    ref = vo.c_estep_pairs(cs["base"], cs["consts"], cs["T"], nthreads=4, want_tnu=True)
    got = _engine(vb, cs["base"], cs["consts"], cs["T"]).pairs(want_tnu=True)
    torch.cuda.synchronize()
    for k in PAIR_KEYS + ("sum_t_nu",):
        g = got[k].cpu().numpy()
        assert stat_err(g, ref[k]) < 1e-8, (S, k, stat_err(g, ref[k]))
    assert elem_err(got["LL_elbo"].cpu().numpy(), ref["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 2, 3])
def test_face_scale_fused(vb, vo, S):
    cs = face_case(S, seed=80 + S, N=120)
    base, consts, T = cs["base"], cs["consts"], cs["T"]
    N = base["prior"].shape[0]
    pairs = vo.c_estep_pairs(base, consts, T, nthreads=4)
    tN = 10.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, cs["post"]["alpha"])
    st = vo.c_statistics(Z, pairs, 1)
    eng = _engine(vb, base, consts, T)
    eng.set_log_omega(logOmega)
    vec = eng.fused(torch.as_tensor(tN, device=DEV)).cpu().numpy()
    K = consts["logPi"].shape[0]
    got = vb.host.unpack_stats(vec, K, S, 2, 1)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, (S, k, stat_err(got[k], st[k]))
    assert hatz_err(eng.hatZ.cpu().numpy(), hz) < RTOL_NORTH_STAR
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 2, 3])
def test_face_scale_em_vs_oracle(vb, vo, S):
    """EM from the same initial posterior (6 iterations) on the GPU and in the oracle."""
    from vbhem_amd.em import vbhem_h3m_c_step_fc
    from vbhem_amd.estep import EStepEngine
    cs = face_case(S, seed=90 + S, N=60, K=3)
    opt = dict(cs["opt"], max_iter=6)
    eng = EStepEngine(cs["bs"], 3, S, cs["T"], device=DEV)
    res = vbhem_h3m_c_step_fc(cs["P"], eng, opt)
    ref = vo.em_step_fc(post_dict(cs["P"]), cs["base"], opt)
    assert res.iters == ref["iters"]
    np.testing.assert_allclose(res.LogLs, ref["LogLs"], rtol=RTOL_NORTH_STAR)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert post_err(getattr(res.post, k), ref["post"][k]) < RTOL_NORTH_STAR, (S, k)
    assert hatz_err(res.hatZ.cpu().numpy(), ref["hat_Z"]) < RTOL_NORTH_STAR


def _fused_vs_oracle(vb, vo, name, N=None, nthreads=8):
    from vbhem_amd.em import tilde_n
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload(name, N=N)
    cov = base.covmode
    consts = vb.host.cluster_constants(P, cov)
    logOm = vb.host.log_omega_tilde(P.alpha)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    eng.set_clusters(consts)
    eng.set_log_omega(logOm)
    tN = tilde_n(eng, opt["Nv"], base.N)
    vec = eng.fused(tN).cpu().numpy()
    bnp = base.numpy()
    pairs = vo.c_estep_pairs(bnp, consts, opt["tau"], nthreads=nthreads)
    tNn = tN.cpu().numpy()
    hz, Z = vo.c_responsibilities(pairs["LL_elbo"], tNn, logOm)
    st = vo.c_statistics(Z, pairs, cov)
    got = vb.host.unpack_stats(vec, P.K, P.S, base.d, cov)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], st[k]) < 1e-9, (name, k, stat_err(got[k], st[k]))
    assert hatz_err(eng.hatZ.cpu().numpy(), hz) < RTOL_NORTH_STAR
    assert elem_err(eng.LL.cpu().numpy(), pairs["LL_elbo"]) < RTOL_PAIRS
    assert eng.fallback_count() == 0
    return hz


@pytest.mark.gpu
def test_c3_full_size_vs_oracle(vb, vo):
    """C3 at N = 10,000 (80,000 pairs), every pair checked."""
    hz = _fused_vs_oracle(vb, vo, "C3")
    assert hz.shape == (10_000, 8)


@pytest.mark.gpu
def test_c5_slice_vs_oracle(vb, vo):
    """C5 shapes (K = 32, S = Sb = 12, d = 16 full) on 1,000 bases = 32,000 pairs."""
    hz = _fused_vs_oracle(vb, vo, "C5", N=1000, nthreads=16)
    assert hz.shape == (1000, 32)


def test_chunked_oracle_matches_whole(vb, vo):
    """CPU: the chunked fused oracle (vbhem_oracle.c_fused) equals the unchunked
    pipeline (pairs -> responsibilities -> statistics) up to summation order."""
    cs = make_case(23, 3, 3, 3, 2, 1, seed=90, tau=5)
    base, consts = cs["base"], cs["consts"]
    tN = 100.0 * 23 * base["omega"]
    logOm, _, _, _ = vo.responsibilities(np.zeros((23, 3)), tN, cs["post"]["alpha"])
    whole = vo.c_estep_pairs(base, consts, 5)
    hz, Z = vo.c_responsibilities(whole["LL_elbo"], tN, logOm)
    st = vo.c_statistics(Z, whole, 1)
    ch = vo.c_fused(base, consts, 5, tN, logOm, chunk=4)
    assert np.array_equal(ch["LL_elbo"], whole["LL_elbo"]) and np.array_equal(ch["hat_Z"], hz)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(ch[k], st[k]) < 1e-13, k
    assert abs(ch["Lt1"] - float((Z * whole["LL_elbo"]).sum())) < 1e-12 * abs(ch["Lt1"])


def _full_size_vs_oracle(vb, vo, name, N=None, chunk=4096, nthreads=16):
    """The fused device E-step against the chunked oracle on EVERY pair: L_elbo
    (elementwise 1e-10), hat_Z (1e-5), the statistics (1e-9) and the ELBO
    partials Lt1 / Lt7."""
    from vbhem_amd.em import tilde_n
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload(name, N=N)
    cov = base.covmode
    consts = vb.host.cluster_constants(P, cov)
    logOm = vb.host.log_omega_tilde(P.alpha)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    eng.set_clusters(consts)
    eng.set_log_omega(logOm)
    tN = tilde_n(eng, opt["Nv"], base.N)
    vec = eng.fused(tN).cpu().numpy()
    LL, hZ = eng.LL.cpu().numpy(), eng.hatZ.cpu().numpy()
    assert eng.fallback_count() == 0
    del eng
    ref = vo.c_fused(base.numpy(), consts, opt["tau"], tN.cpu().numpy(), logOm,
                     nthreads=nthreads, chunk=chunk)
    assert elem_err(LL, ref["LL_elbo"]) < RTOL_PAIRS
    assert hatz_err(hZ, ref["hat_Z"]) < RTOL_NORTH_STAR
    got = vb.host.unpack_stats(vec, P.K, P.S, base.d, cov)
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], ref[k]) < 1e-9, (name, k, stat_err(got[k], ref[k]))
    for k in ("Lt1", "Lt7"):
        assert abs(got[k] - ref[k]) <= 1e-9 * abs(ref[k]), (k, got[k], ref[k])
    return base.N


@pytest.mark.gpu
def test_c4_full_size_vs_oracle(vb, vo):
    """C4 at its full size (N = 100,000, K = 16: 1.6 M pairs), every pair, every
    hat_Z entry and every statistic against the oracle (16 host threads)."""
    assert _full_size_vs_oracle(vb, vo, "C4", chunk=10_000) == 100_000


@pytest.mark.gpu
def test_c5_multigroup_vs_oracle(vb, vo, monkeypatch):
    """C5 shapes (K = 32, S = Sb = 12, d = 16 full) on 20,000 bases (640,000 pairs)
    through the multi-group path of the full-size run: VBHEM_GROUP_BASES = 6,000
    splits the call into 4 base groups (C5 at N = 10^6 runs as 14 groups of
    <= 74 k), each with its own emission GEMM, backward pass, gate lists and list
    statistics accumulated into the same slabs."""
    monkeypatch.setenv("VBHEM_GROUP_BASES", "6000")
    assert _full_size_vs_oracle(vb, vo, "C5", N=20_000, chunk=1000) == 20_000


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 6, 7, 9, 15, 16, 17, 31, 33, 125, 250, 333, 500, 501])
def test_c4_shard_sizes_vs_oracle(vb, vo, N):
    """C4 shapes (S = Sb = 8, T = 10: fb_bwd4_kernel and fb_list4_kernel, the MFMA
    kernels) at base counts of every residue class that matters to them -- a quad
    is 4 bases, a block's tile 16 -- up to the 500 / 501-base shards of a two-rank
    run: every pair, hat_Z entry and statistic against the oracle.  (Regression
    for the mid-round-3 two-rank C4 failure)"""
    assert _full_size_vs_oracle(vb, vo, "C4", N=N, chunk=512, nthreads=8) == N


@pytest.mark.gpu
def test_c5_full_size_sampled_vs_oracle(vb, vo):
    """C5 at its full size (N = 10^6, K = 32, S = Sb = 12, d = 16 full: 14 base groups of
    <= 74 k bases, 32 M pairs) in one fused call, checked three ways:
    * L_elbo (elementwise 1e-10) and hat_Z (1e-5) against the oracle on 4,000 bases
      spread evenly over all N, so every base group is sampled (hat_Z of a base depends
      on its own L_elbo row only, vbhem_h3m_c_step_fc.m:275-276);
    * determinism: a second call gives bit-identical statistics, L_elbo and hat_Z;
    * the gated schedule equals the dense one (every pair's forward sweep,
      vbhem_compute_Statistics.m:33-55) on the whole statistics vector (1e-9)."""
    from vbhem_amd import _capi
    from vbhem_amd.em import tilde_n
    from vbhem_amd.estep import EStepEngine
    BaseSet = vb.BaseSet
    base, P, opt = vb.synth_workload("C5", device=DEV)
    assert base.N == 1_000_000
    cov = base.covmode
    consts = vb.host.cluster_constants(P, cov)
    logOm = vb.host.log_omega_tilde(P.alpha)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    eng.set_clusters(consts)
    eng.set_log_omega(logOm)
    tN = tilde_n(eng, opt["Nv"], base.N)
    vec = eng.fused(tN).clone()
    LL, hZ = eng.LL.clone(), eng.hatZ.clone()
    assert eng.fallback_count() == 0
    vec2 = eng.fused(tN).clone()
    assert torch.equal(vec, vec2) and torch.equal(eng.LL, LL) and torch.equal(eng.hatZ, hZ)
    prev = _capi.set_fused_mode(_capi.FUSED_DENSE)
    try:
        dvec = eng.fused(tN).clone()
    finally:
        _capi.set_fused_mode(prev)
    K, S, d = P.K, P.S, base.d
    got, dense = (vb.host.unpack_stats(v.cpu().numpy(), K, S, d, cov) for v in (vec, dvec))
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(got[k], dense[k]) < 1e-9, (k, stat_err(got[k], dense[k]))
    idx = torch.linspace(0, base.N - 1, 4000, device=DEV).round().long().unique()
    sub = BaseSet(*(t[idx] for t in (base.nstates, base.prior, base.A, base.centres,
                                     base.covars, base.omega)), cov).numpy()
    del eng
    ref = vo.c_estep_pairs(sub, consts, opt["tau"], nthreads=16)
    ii = idx.cpu().numpy()
    hz_ref, _ = vo.c_responsibilities(ref["LL_elbo"], tN.cpu().numpy()[ii], logOm)
    assert elem_err(LL.cpu().numpy()[ii], ref["LL_elbo"]) < RTOL_PAIRS
    assert hatz_err(hZ.cpu().numpy()[ii], hz_ref) < RTOL_NORTH_STAR

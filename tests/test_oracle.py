"""The oracle itself (CPU): the C restatement of the reference MEX against the
independent numpy restatement of the MATLAB twin, and both against closed-form
known answers.  The reference ships no fixtures, so these
cross-checks are what pins the oracle ("Oracle").
"""
import zlib

import numpy as np
import pytest
from scipy.special import logsumexp

from cases import SHAPES, make_case
from conftest import rel_err

PAIR_KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")


def emission_E(base, consts, i, j):
    """E[beta, sigma] = -1/2 (d ln 2pi + c + <P, Sigma_beta> + (mu-m)' P (mu-m)),
    mex.c:718-830 / fast.m:66-140 (independent restatement for the KATs)."""
    cen = base["centres"][i]
    cov = base["covars"][i]
    m, P, c = consts["m"][j], consts["P"][j], consts["c"][j]
    d = cen.shape[1]
    diff = cen[:, None, :] - m[None, :, :]                         # [Sb, S, d]
    if base["covmode"] == 1:
        tr = np.einsum("sab,kab->ks", P, cov)
        mah = np.einsum("ksa,sab,ksb->ks", diff, P, diff)
    else:
        tr = np.einsum("sa,ka->ks", P, cov)
        mah = np.einsum("ksa,sa->ks", diff * diff, P)
    return -0.5 * (d * np.log(2 * np.pi) + c[None, :] + tr + mah)


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_c_oracle_matches_numpy_twin(vo, shape):
    name, N, K, S, Sb, d, cov, T, ragged = shape
    cs = make_case(N, K, S, Sb, d, cov, seed=zlib.crc32(name.encode()) % 1000, ragged=ragged, tau=T)
    c = vo.c_estep_pairs(cs["base"], cs["consts"], T, nthreads=4)
    tw = vo.twin_estep_pairs(cs["base"], cs["post"], cs["consts"], T)
    for k in PAIR_KEYS:
        assert rel_err(c[k], tw[k]) < 1e-12, (k, rel_err(c[k], tw[k]))


def test_c_oracle_thread_count_invariant(vo):
    cs = make_case(7, 4, 3, 3, 2, 1, seed=3, tau=8)
    a = vo.c_estep_pairs(cs["base"], cs["consts"], 8, nthreads=1, want_tnu=True)
    b = vo.c_estep_pairs(cs["base"], cs["consts"], 8, nthreads=5, want_tnu=True)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


@pytest.mark.parametrize("cov", [0, 1])
def test_kat_T1(vo, cov):
    """T = 1: no transitions; LL = sum_b pi_b LSE_s(logPi_s + E[b,s])."""
    cs = make_case(4, 3, 4, 3, 3, cov, seed=11, tau=1)
    base, consts = cs["base"], cs["consts"]
    o = vo.c_estep_pairs(base, consts, 1, want_tnu=True)
    for i in range(4):
        for j in range(3):
            E = emission_E(base, consts, i, j)
            lt = consts["logPi"][j][None, :] + E                   # [Sb, S]
            ls = logsumexp(lt, axis=1)
            th = np.exp(lt - ls[:, None])
            pi = base["prior"][i]
            assert abs(o["LL_elbo"][i, j] - pi @ ls) <= 1e-12 * abs(pi @ ls)
            nu1 = (pi[:, None] * th).sum(0)
            np.testing.assert_allclose(o["sum_nu_1"][i, j], nu1, rtol=1e-12, atol=1e-300)
            np.testing.assert_allclose(o["emit_pr"][i, j], nu1, rtol=1e-12, atol=1e-300)
            np.testing.assert_array_equal(o["sum_xi"][i, j], 0.0)
            np.testing.assert_allclose(o["emit_mu"][i, j], (pi[:, None] * th).T @ base["centres"][i],
                                       rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("cov", [0, 1])
def test_kat_single_cluster_state(vo, cov):
    """S = 1: logA = logPi = 0, so LL = pi . sum_k A^k E and the occupancies are
    the base chain's marginals pi A^t."""
    T = 7
    cs = make_case(4, 2, 1, 4, 2, cov, seed=5, tau=T)
    base, consts = cs["base"], cs["consts"]
    np.testing.assert_array_equal(consts["logA"], 0.0)
    np.testing.assert_array_equal(consts["logPi"], 0.0)
    o = vo.c_estep_pairs(base, consts, T, want_tnu=True)
    for i in range(4):
        A, pi = base["A"][i], base["prior"][i]
        for j in range(2):
            E = emission_E(base, consts, i, j)[:, 0]
            acc, v = np.zeros_like(E), E.copy()
            for _ in range(T):
                acc += v
                v = A @ v
            LL = pi @ acc
            assert abs(o["LL_elbo"][i, j] - LL) <= 1e-12 * abs(LL)
            marg, tnu, xi = pi.copy(), np.zeros_like(pi), 0.0
            for t in range(T):
                tnu += marg
                if t > 0:
                    xi += marg.sum()
                marg = marg @ A
            np.testing.assert_allclose(o["sum_t_nu"][i, j, 0], tnu, rtol=1e-12)
            assert abs(o["sum_xi"][i, j, 0, 0] - xi) <= 1e-12 * xi
            assert abs(o["sum_nu_1"][i, j, 0] - pi.sum()) <= 1e-14


@pytest.mark.parametrize("shape", SHAPES[:12], ids=[s[0] for s in SHAPES[:12]])
def test_occupancy_mass_rules(vo, shape):
    """Column masses of the forward occupancies follow the base chain:
    sum_s nu_t(s, .) = pi A^(t-1), for any cluster parameters."""
    name, N, K, S, Sb, d, cov, T, ragged = shape
    cs = make_case(N, K, S, Sb, d, cov, seed=21, ragged=ragged, tau=T)
    base = cs["base"]
    o = vo.c_estep_pairs(base, cs["consts"], T, want_tnu=True)
    for i in range(N):
        A, pi = base["A"][i], base["prior"][i]
        marg, tot, xi = pi.copy(), np.zeros_like(pi), 0.0
        for t in range(T):
            tot += marg
            if t > 0:
                xi += marg.sum()
            marg = marg @ A
        for j in range(K):
            np.testing.assert_allclose(o["sum_t_nu"][i, j].sum(0), tot, rtol=1e-11, atol=1e-14)
            assert abs(o["sum_nu_1"][i, j].sum() - pi.sum()) <= 1e-12
            assert abs(o["emit_pr"][i, j].sum() - tot.sum()) <= 1e-11 * tot.sum()
            assert abs(o["sum_xi"][i, j].sum() - xi) <= 1e-11 * max(xi, 1e-300)


def test_base_state_permutation_invariance(vo):
    cs = make_case(3, 3, 3, 4, 2, 1, seed=8, tau=6)
    base = cs["base"]
    perm = np.array([2, 0, 3, 1])
    pb = dict(base)
    pb["prior"] = base["prior"][:, perm]
    pb["A"] = base["A"][:, perm][:, :, perm]
    pb["centres"] = base["centres"][:, perm]
    pb["covars"] = base["covars"][:, perm]
    a = vo.c_estep_pairs(base, cs["consts"], 6, want_tnu=True)
    b = vo.c_estep_pairs(pb, cs["consts"], 6, want_tnu=True)
    for k in PAIR_KEYS:
        assert rel_err(b[k], a[k]) < 1e-13, k
    np.testing.assert_allclose(b["sum_t_nu"], a["sum_t_nu"][..., perm], rtol=1e-12, atol=1e-300)


def test_zero_padding_is_exact(vo):
    """Padding base HMMs with zero-prior, zero-transition states changes nothing
    (include/vbhem_estep.h conventions)."""
    cs = make_case(3, 2, 3, 3, 2, 1, seed=9, tau=5)
    base = cs["base"]
    pad = 2
    SB = base["prior"].shape[1] + pad
    pb = dict(base)
    pb["prior"] = np.pad(base["prior"], ((0, 0), (0, pad)))
    pb["A"] = np.pad(base["A"], ((0, 0), (0, pad), (0, pad)))
    pb["centres"] = np.pad(base["centres"], ((0, 0), (0, pad), (0, 0)))
    cv = np.zeros((3, SB, 2, 2))
    cv[:, :3] = base["covars"]
    cv[:, 3:] = np.eye(2)
    pb["covars"] = cv
    a = vo.c_estep_pairs(base, cs["consts"], 5, want_tnu=True)
    b = vo.c_estep_pairs(pb, cs["consts"], 5, want_tnu=True)
    for k in PAIR_KEYS:
        np.testing.assert_array_equal(b[k], a[k])
    np.testing.assert_array_equal(b["sum_t_nu"][..., :3], a["sum_t_nu"])
    np.testing.assert_array_equal(b["sum_t_nu"][..., 3:], 0.0)


def test_responsibilities_c_vs_numpy(vo):
    rng = np.random.default_rng(3)
    N, K = 50, 6
    LL = rng.normal(-40, 15, (N, K))
    tN = rng.uniform(5, 200, N)
    alpha = rng.uniform(1, 300, K)
    logOmega, hz, Z, Nj = vo.responsibilities(LL, tN, alpha)
    hz_c, Z_c = vo.c_responsibilities(LL, tN, logOmega)
    assert rel_err(hz_c, hz) < 1e-14
    assert rel_err(Z_c, Z) < 1e-14
    # direct definition (step_fc.m:275-283)
    lz = tN[:, None] * (logOmega[None, :] + LL)
    ref = np.exp(lz - logsumexp(lz, axis=1, keepdims=True)) + 1e-50
    assert rel_err(hz, ref) < 1e-14
    np.testing.assert_allclose(hz.sum(1), 1.0, rtol=1e-12)


@pytest.mark.parametrize("cov", [0, 1])
def test_statistics_c_vs_numpy(vo, cov):
    cs = make_case(12, 4, 3, 3, 3, cov, seed=31, tau=6)
    o = vo.c_estep_pairs(cs["base"], cs["consts"], 6)
    rng = np.random.default_rng(2)
    Z = rng.uniform(0, 3, (12, 4))
    Z[rng.random((12, 4)) < 0.3] = 1e-9      # below the 1e-8 gate
    st = vo.c_statistics(Z, o, cov)
    for j in range(4):
        pj = {k: o[k][:, j] for k in ("sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")}
        ref = vo.compute_statistics(Z[:, j], pj, 3, 3, cov)
        np.testing.assert_allclose(st["N1"][j], ref["Nj_rho1"], rtol=1e-13)
        np.testing.assert_allclose(st["M"][j], ref["Nj_rho2rho"], rtol=1e-13)
        # ref Nr carries +1e-50 and y/SC are normalised; compare raw sums
        g = Z[:, j] > 1e-8
        np.testing.assert_allclose(st["Nr"][j], (Z[g, j, None] * o["emit_pr"][g, j]).sum(0),
                                   rtol=1e-13)
        np.testing.assert_allclose(st["Nj"][j], Z[:, j].sum(), rtol=1e-14)


# ----------------------------------------------------------------------------
# VHEM sibling (hem_hmm_bwd_fwd_mex.c): C restatement vs the numpy twin of
# hem_hmm_bwd_fwd.m, and vs the VBHEM oracle fed the equivalent constants
# ----------------------------------------------------------------------------
VHEM_SHAPES = [  # (name, N, K, S, Sb, d, cov, T, ragged, smooth, zero_transition)
    ("vhem_full", 5, 3, 3, 3, 2, 1, 6, False, 1.0, False),
    ("vhem_diag", 5, 3, 3, 3, 2, 0, 6, False, 1.0, False),
    ("vhem_full_smooth", 6, 3, 4, 3, 3, 1, 7, True, 2.5, False),
    ("vhem_diag_smooth", 6, 3, 4, 3, 3, 0, 7, True, 0.4, False),
    ("vhem_zero_transition", 5, 2, 3, 3, 2, 1, 5, False, 1.0, True),
]


def vhem_twin_pairs(vo, base, red, T, smooth):
    N = base["prior"].shape[0]
    K = red["prior"].shape[0]
    res = None
    for i in range(N):
        Sb = int(base["nstates"][i])
        for j in range(K):
            o = vo.twin_vhem_pair_estep(base["prior"][i, :Sb], base["A"][i, :Sb, :Sb],
                                        base["centres"][i, :Sb], base["covars"][i, :Sb],
                                        base["covmode"], T, smooth, red["A"][j], red["prior"][j],
                                        red["centres"][j], red["covars"][j])
            if res is None:
                res = {k: np.zeros((N, K) + np.shape(v)) for k, v in o.items() if k != "sum_t_nu"}
            for k, v in o.items():
                if k != "sum_t_nu":
                    res[k][i, j] = v
    return res


@pytest.mark.parametrize("shape", VHEM_SHAPES, ids=[s[0] for s in VHEM_SHAPES])
def test_vhem_oracle_matches_twin(vo, shape):
    from cases import make_reduced
    name, N, K, S, Sb, d, cov, T, ragged, smooth, zt = shape
    seed = zlib.crc32(name.encode()) % 1000
    cs = make_case(N, K, S, Sb, d, cov, seed=seed, ragged=ragged, tau=T)
    red = make_reduced(K, S, d, cov, seed=seed, zero_transition=zt)
    c = vo.c_vhem_estep_pairs(cs["base"], red, T, smooth, nthreads=4)
    tw = vhem_twin_pairs(vo, cs["base"], red, T, smooth)
    for k in PAIR_KEYS:
        assert np.isfinite(c[k]).all(), k
        assert rel_err(c[k], tw[k]) < 1e-12, (k, rel_err(c[k], tw[k]))


def test_vhem_full_equals_vbhem_with_point_constants(vo, vb):
    """Full covariances at smooth = 1: the VHEM recursion is the VBHEM one fed
    logA = log A_r, logPi = log prior_r, P = inv(Sigma_r), c = log det(Sigma_r)
    (the product's vhem_cluster_constants) -- identical code path in the oracle."""
    from cases import make_reduced
    cs = make_case(5, 3, 3, 3, 2, 1, seed=17, tau=6)
    red = make_reduced(3, 3, 2, 1, seed=17)
    consts = vb.host.vhem_cluster_constants(red, 1)
    a = vo.c_vhem_estep_pairs(cs["base"], red, 6, 1.0)
    b = vo.c_estep_pairs(cs["base"], consts, 6)
    for k in PAIR_KEYS:
        assert rel_err(a[k], b[k]) < 1e-13, k

"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from
the oracle; parity unpinned by the reference itself -- see that script).

CPU: the oracle and the product EM loop reproduce the fixtures.
GPU: the HIP E-step (pairs and fused entry points) and the GPU EM loop
reproduce them within the stated tolerances."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN_DIR, RTOL_NORTH_STAR, RTOL_PAIRS, elem_err, hatz_err, post_err, rel_err, stat_err

PAIR_KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")
PAIR_FILES = sorted(glob.glob(os.path.join(GOLDEN_DIR, "pairs_*.npz")))
PAIR_IDS = [os.path.basename(p)[:-4] for p in PAIR_FILES]


def load(path):
    z = np.load(path)
    base = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    base["covmode"] = int(z["covmode"])
    consts = {k[2:]: z[k] for k in z.files if k.startswith("c_")}
    out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    fz = {k[3:]: z[k] for k in z.files if k.startswith("fz_")}
    return base, consts, out, fz, int(z["T"])


def test_fixtures_present():
    assert len(PAIR_FILES) >= 4
    assert os.path.exists(os.path.join(GOLDEN_DIR, "em_c2.npz"))


@pytest.mark.parametrize("path", PAIR_FILES, ids=PAIR_IDS)
def test_oracle_reproduces_fixture(vo, path):
    base, consts, out, fz, T = load(path)
    got = vo.c_estep_pairs(base, consts, T, nthreads=2, want_tnu="sum_t_nu" in out)
    for k, v in out.items():
        assert rel_err(got[k], v) < 1e-13, k


def test_product_em_reproduces_em_fixture(vb):
    from oracle_engine import OracleEngine
    from vbhem_amd.em import vbhem_h3m_c_step_fc

    z = np.load(os.path.join(GOLDEN_DIR, "em_c2.npz"))
    base = vb.BaseSet.from_numpy({**{k[3:]: z[k] for k in z.files if k.startswith("in_")},
                                  "covmode": 1})
    P = vb.Posterior(**{k[5:]: z[k] for k in z.files if k.startswith("init_")})
    opt = vb.synth_workload("C2", N=4)[2]
    res = vbhem_h3m_c_step_fc(P, OracleEngine(base, P.K, P.S, int(z["T"])), opt)
    assert res.iters == int(z["iters"])
    np.testing.assert_allclose(res.LogLs, z["LogLs"], rtol=1e-10)
    np.testing.assert_array_equal(res.label.numpy(), z["label"])


# ----------------------------------------------------------------------------
# GPU
# ----------------------------------------------------------------------------
def _engine(vb, base, consts, T):
    from vbhem_amd.estep import EStepEngine
    K, S = consts["logPi"].shape
    eng = EStepEngine(vb.BaseSet.from_numpy(base), K, S, T, device="cuda:0")
    eng.set_clusters(consts)
    return eng


@pytest.mark.gpu
@pytest.mark.parametrize("path", PAIR_FILES, ids=PAIR_IDS)
def test_hip_pairs_reproduce_fixture(vb, path):
    base, consts, out, fz, T = load(path)
    eng = _engine(vb, base, consts, T)
    got = eng.pairs(want_tnu="sum_t_nu" in out)
    torch.cuda.synchronize()
    for k, v in out.items():
        assert rel_err(got[k].cpu().numpy(), v) < RTOL_PAIRS, (k, rel_err(got[k].cpu().numpy(), v))
    assert eng.fallback_count() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("path", PAIR_FILES, ids=PAIR_IDS)
def test_hip_fused_reproduces_fixture(vb, path):
    base, consts, out, fz, T = load(path)
    eng = _engine(vb, base, consts, T)
    eng.set_log_omega(fz["logOmega"])
    tN = torch.as_tensor(fz["tildeN"], dtype=torch.float64, device="cuda:0")
    stats = eng.fused(tN).cpu().numpy()
    K, S = consts["logPi"].shape
    d = base["centres"].shape[2]
    st = vb.host.unpack_stats(stats, K, S, d, base["covmode"])
    for k in ("Nj", "N1", "M", "Nr", "Y", "SC"):
        assert stat_err(st[k], fz[k]) < 1e-9, (k, stat_err(st[k], fz[k]))
    assert abs(st["Lt1"] - fz["Lt1"]) <= 1e-9 * abs(fz["Lt1"])
    # Lt7 = sum hatZ log hatZ can be ~0 (one-hot rows): absolute floor, tiny next to the ELBO
    assert abs(st["Lt7"] - fz["Lt7"]) <= 1e-9 * abs(fz["Lt7"]) + 1e-9
    assert hatz_err(eng.hatZ.cpu().numpy(), fz["hatZ"]) < RTOL_NORTH_STAR
    assert rel_err(eng.LL.cpu().numpy(), out["LL_elbo"]) < RTOL_PAIRS
    assert elem_err(eng.LL.cpu().numpy(), out["LL_elbo"]) < RTOL_PAIRS


@pytest.mark.gpu
def test_gpu_em_reproduces_em_fixture(vb):
    """The north-star check: the full EM loop on the GPU path reproduces the
    oracle trajectory; hat_Z, posteriors, ELBO within 1e-5 relative."""
    from vbhem_amd.em import vbhem_h3m_c_step_fc
    from vbhem_amd.estep import EStepEngine

    z = np.load(os.path.join(GOLDEN_DIR, "em_c2.npz"))
    base = vb.BaseSet.from_numpy({**{k[3:]: z[k] for k in z.files if k.startswith("in_")},
                                  "covmode": 1})
    P = vb.Posterior(**{k[5:]: z[k] for k in z.files if k.startswith("init_")})
    opt = vb.synth_workload("C2", N=4)[2]
    eng = EStepEngine(base, P.K, P.S, int(z["T"]), device="cuda:0")
    res = vbhem_h3m_c_step_fc(P, eng, opt)
    assert res.iters == int(z["iters"])
    np.testing.assert_allclose(res.LogLs, z["LogLs"], rtol=RTOL_NORTH_STAR)
    for k in ("alpha", "eta", "epsilon", "lam", "v", "m", "W"):
        assert post_err(getattr(res.post, k), z["post_" + k]) < RTOL_NORTH_STAR, k
    assert hatz_err(res.hatZ.cpu().numpy(), z["hat_Z"]) < RTOL_NORTH_STAR
    np.testing.assert_array_equal(res.label.cpu().numpy(), z["label"])

"""emission_db_kernel (the chunked emission GEMM double-buffered)
against the single-buffer chunked path (VBHEM_EM_NODB=1): the same accumulation order, so
the fused E-step's statistics, L_elbo and hat_Z must agree bit for bit -- at d = 16 full
(KQ = 38, the chunked path), one and several rounds of tiles per block, K S = 96 and 384
rows (4 and 12 chunks), ragged base counts (a last tile past the base range)."""
import numpy as np
import pytest
import torch

from cases import make_case

DEV = "cuda:0"


def _fused(vb, cs, env, monkeypatch):
    from vbhem_amd.estep import EStepEngine
    monkeypatch.delenv("VBHEM_EM_NODB", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    K, S = cs["consts"]["logPi"].shape
    eng = EStepEngine(vb.BaseSet.from_numpy(cs["base"]), K, S, cs["T"], device=DEV)
    eng.set_clusters(cs["consts"])
    eng.set_log_omega(np.full(K, -np.log(K)))
    tN = torch.as_tensor(100.0 * cs["base"]["omega"] * cs["base"]["prior"].shape[0], device=DEV)
    st = eng.fused(tN).cpu().numpy()
    torch.cuda.synchronize()
    return st, eng.LL.cpu().numpy(), eng.hatZ.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("N,K,S,Sb", [(37, 8, 12, 12), (1501, 8, 12, 12), (403, 32, 12, 12),
                                      (2999, 32, 12, 9)])
def test_db_emission_bit_identical(vb, monkeypatch, N, K, S, Sb):
    cs = make_case(N, K, S, Sb, 16, 1, seed=N + K + Sb, tau=10)
    ref = _fused(vb, cs, {"VBHEM_EM_NODB": "1"}, monkeypatch)
    got = _fused(vb, cs, {}, monkeypatch)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    assert np.isfinite(got[1]).all()

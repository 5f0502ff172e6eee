"""The completion word (vbhem_arm_done_word): an E-step's last kernel
stores the armed ticket once its statistics are in host memory, so a host running one
E-step ahead polls a word instead of recording an event per step (bench.py's pacing).
The tickets must arrive in order, every step's statistics must be complete when its
ticket is seen, an armed call must equal an unarmed one bit for bit, and the flag head
(fallback counters) must stay clean across armed calls."""
import numpy as np
import pytest
import torch

from cases import make_case

DEV = "cuda:0"


def _synth(vb, name, N):
    from vbhem_amd.estep import EStepEngine
    from vbhem_amd.em import tilde_n
    from vbhem_amd import host
    base, P, opt = vb.synth_workload(name, N=N)
    eng = EStepEngine(base, P.K, P.S, opt["tau"], device=DEV)
    eng.set_clusters(host.cluster_constants(P, base.covmode))
    eng.set_log_omega(host.log_omega_tilde(P.alpha))
    return eng, tilde_n(eng, opt["Nv"], N)


@pytest.mark.gpu
@pytest.mark.parametrize("name,N", [("C4", 3000), ("C3", 2000)])
def test_done_word_run_ahead(vb, name, N):
    eng, tN = _synth(vb, name, N)
    ref = eng.fused(tN).cpu().numpy()
    hs = [eng.host_stats_buffer(), eng.host_stats_buffer()]
    w = eng.done_word()
    assert w.value == 0
    for k in range(8):
        eng.fused(tN, out=hs[k % 2], done=(w, 10 + k))
        if k > 0:
            w.wait(10 + k - 1, timeout_s=30)
            # step k - 1's statistics are complete in host memory (step k + 1, which
            # overwrites the buffer, is not launched yet)
            assert np.array_equal(hs[(k - 1) % 2].numpy(), ref), k
    w.wait(17, timeout_s=30)
    torch.cuda.synchronize()
    assert w.value == 17
    assert np.array_equal(hs[1].numpy(), ref)
    # an unarmed call after armed ones: the word is left alone, results unchanged
    out = eng.fused(tN).cpu().numpy()
    torch.cuda.synchronize()
    assert w.value == 17 and np.array_equal(out, ref)


@pytest.mark.gpu
def test_done_word_with_fallback(vb):
    """Armed calls that take the exact fallback: the counters the last kernel uses for
    its blocks (the flag head) are reset, so the fallback count is the same call after
    call and equals an unarmed call's."""
    from vbhem_amd.estep import EStepEngine
    # test_gpu_parity.adversarial_case at S = Sb = 8, T = 10: cluster 0's pairs underflow
    cs = make_case(41, 2, 8, 8, 3, 1, seed=99, tau=10)
    consts = {k: np.array(v, copy=True) for k, v in cs["consts"].items()}
    lA = np.full((8, 8), -600.0)
    for r in range(8):
        lA[r, (r + 1) % 8] = 0.0
    consts["logA"][0] = lA
    consts["c"][0] = 1200.0
    consts["c"][0, 0] = 0.0
    consts["c"][1:] = 1.0e4
    base = vb.BaseSet.from_numpy(cs["base"])
    eng = EStepEngine(base, 2, 8, cs["T"], device=DEV)
    eng.set_clusters(consts)
    eng.set_log_omega(torch.zeros(2, dtype=torch.float64))
    tN = torch.as_tensor(100.0 * 41 * cs["base"]["omega"], device=DEV)
    ref = eng.fused(tN).cpu().numpy()
    n_ref = eng.fallback_count()
    assert n_ref > 0
    w = eng.done_word()
    hs = eng.host_stats_buffer()
    for k in range(3):
        eng.fused(tN, out=hs, done=(w, k + 1))
        w.wait(k + 1, timeout_s=30)
        assert np.array_equal(hs.numpy(), ref)
        assert eng.fallback_count() == n_ref

"""The .xls reader (vbhem_amd.xls; read_xls_fixations.m with a BIFF8 reader in
place of xlsread) and the demo's data path into the VB-HMM forward-backward.

CPU: RK-number and shared-string decoding on hand-built records; the reference's
demo/demodata.xls (when /root/reference is mounted) against the committed
fixture tests/golden/demo_fixations.npz.  The fixture is made by
make_demo_fixations.py from tests/golden/biff_cells.py, a second reader written
separately from vbhem_amd/xls.py (compound file + SST/LABELSST/NUMBER/RK/MULRK
only), so the check is not circular; both readers also decode the same
hand-built records.
GPU: the demo's 399 fixation sequences through vbhmm_fb (C1's first stage)
against the oracle restatement of vbhmm_fb_mex.c."""
import os
import struct
import sys

import numpy as np
import pytest

import vbhem_oracle as vo
from conftest import GOLDEN_DIR, rel_err

sys.path.insert(0, GOLDEN_DIR)
import biff_cells  # noqa: E402  (the independent reader; test infrastructure)

DEMO = "/root/reference/demo/demodata.xls"


def test_rk_decoding(vb):
    from vbhem_amd.xls import _rk
    assert _rk((123 << 2) | 2) == 123.0                    # integer
    assert _rk((123 << 2) | 3) == 1.23                     # integer / 100
    assert _rk((((1 << 30) - 5) << 2) | 2) == -5.0         # negative integer
    hi = struct.unpack("<Q", struct.pack("<d", 2.5))[0] >> 32
    assert _rk(hi << 0) == 2.5                             # top 30 bits of a double


def test_sst_with_continue(vb):
    from vbhem_amd.xls import _read_sst
    s1, s2 = "SubjectID", "FixX"
    rec = struct.pack("<II", 2, 2) + struct.pack("<HB", len(s1), 0) + s1[:4].encode()
    cont = bytes([1]) + s1[4:].encode("utf-16-le") + struct.pack("<HB", len(s2), 0) + s2.encode()
    assert _read_sst([rec, cont]) == [s1, s2]


def test_independent_reader_decodes_the_same(vb):
    """biff_cells (the fixture's reader) on the hand-built inputs above."""
    assert biff_cells._rk_value((123 << 2) | 2) == 123.0
    assert biff_cells._rk_value((123 << 2) | 3) == 1.23
    assert biff_cells._rk_value((((1 << 30) - 5) << 2) | 2) == -5.0
    hi = struct.unpack("<Q", struct.pack("<d", 2.5))[0] >> 32
    assert biff_cells._rk_value(hi) == 2.5
    s1, s2 = "SubjectID", "FixX"
    rec = struct.pack("<II", 2, 2) + struct.pack("<HB", len(s1), 0) + s1[:4].encode()
    cont = bytes([1]) + s1[4:].encode("utf-16-le") + struct.pack("<HB", len(s2), 0) + s2.encode()
    assert biff_cells._shared_strings([rec, cont]) == [s1, s2]


def test_fixture_from_independent_reader(vb):
    """The committed fixture is what biff_cells reads from the demo file."""
    if not os.path.exists(DEMO):
        pytest.skip("reference demo data not mounted")
    fx = np.load(os.path.join(GOLDEN_DIR, "demo_fixations.npz"))
    data, names, trials = biff_cells.read_fixations(DEMO)
    seqs = [t for subj in data for t in subj]
    np.testing.assert_array_equal(np.concatenate(seqs), fx["x"])
    assert list(names) == list(fx["names"])
    assert [t for tr in trials for t in tr] == list(fx["trials"])


def test_demo_file_matches_fixture(vb):
    fx = np.load(os.path.join(GOLDEN_DIR, "demo_fixations.npz"))
    assert fx["offsets"][-1] == fx["x"].shape[0] == 1010
    assert len(fx["names"]) == 10 and fx["offsets"].size - 1 == 399
    if not os.path.exists(DEMO):
        pytest.skip("reference demo data not mounted")
    from vbhem_amd.xls import read_xls_fixations
    data, names, trials = read_xls_fixations(DEMO)
    seqs = [t for subj in data for t in subj]
    assert list(names) == list(fx["names"])
    np.testing.assert_array_equal(np.concatenate(seqs), fx["x"])
    np.testing.assert_array_equal(np.cumsum([0] + [len(t) for t in seqs]), fx["offsets"])


@pytest.mark.gpu
def test_demo_sequences_through_vbhmm_fb(vb):
    from vbhem_amd import vbhmm
    fx = np.load(os.path.join(GOLDEN_DIR, "demo_fixations.npz"))
    off, x = fx["offsets"], fx["x"]
    data = [x[off[n]:off[n + 1]] for n in range(off.size - 1)]
    # a 3-state posterior of the face demo's scale (vbdemo_face.m:21-31: v0 = 10,
    # W0 = 0.001, beta0 = 1), centred on three fixation regions
    K = 3
    ctr = np.array([[150.0, 190.0], [190.0, 190.0], [170.0, 260.0]])
    vp = dict(m=ctr, W=np.stack([np.eye(2) / (30.0 ** 2) / 40.0] * K), v=np.full(K, 40.0),
              beta=np.full(K, 41.0), epsilon=np.array([[20.0, 5, 5], [5, 20, 5], [5, 5, 20]]),
              alpha=np.array([30.0, 30.0, 40.0]))
    ref = vo.c_vbhmm_fb(data, vp)
    got = vbhmm.vbhmm_fb(data, vp, device="cuda:0")
    assert rel_err(got["gamma_all"], ref["gamma"].transpose(2, 1, 0)) < 1e-12
    assert rel_err(got["phi_norm"], ref["phi_norm"]) < 1e-12
    assert rel_err(got["xi_sum"], ref["xi_sum"].transpose(1, 2, 0)) < 1e-12

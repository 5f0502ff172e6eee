"""Host-side pieces of bench.py (no GPU): the roofline line's HBM traffic comes from
the newest committed PMC summary of the config (tag order r04z < r04z3 < r04z4, not
the plain string order that put r04z_ last) and only from summaries whose PMC passes
ran the full-size launches alone."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _summary(path, traffic, N=100000, full_only=True):
    with open(path, "w") as f:
        json.dump({"N": N, "n_gpus": 1, "pmc_full_size_only": full_only,
                   "kernels": {"vbhem::fb_bwd4_kernel": {"hbm_bytes_per_launch": {"traffic": traffic}}}},
                  f)


def test_committed_traffic_takes_newest_tag(tmp_path, monkeypatch):
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    _summary(prof / "r04z_c4.json", 1.0)
    _summary(prof / "r04z4_c4.json", 4.0)
    _summary(prof / "r04z3_c4.json", 3.0)
    _summary(prof / "r03h_c4.json", 0.5)
    _summary(prof / "r04z5_c4.json", 5.0, full_only=False)  # mixed launch sizes: skipped
    _summary(prof / "r04z6_c4.json", 6.0, N=12500)          # another size: skipped
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, src = bench.committed_traffic("C4", 100000, 1, "vbhem::fb_bwd4_kernel")
    assert t == 4.0 and src == os.path.join("profiles", "r04z4_c4.json")
    assert bench.committed_traffic("C4", 100000, 2, "vbhem::fb_bwd4_kernel") == (None, None)

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


def test_resolve_world_launches_or_runs_as_rank():
    """--gpus N without WORLD_SIZE starts N ranks; under a launcher the rank count is
    WORLD_SIZE and a disagreeing --gpus is refused."""
    import pytest

    import bench
    assert bench.resolve_world(None, {}) == ("rank", 1)
    assert bench.resolve_world(1, {}) == ("rank", 1)
    assert bench.resolve_world(8, {}) == ("launch", 8)
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == ("rank", 4)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == ("rank", 4)
    with pytest.raises(ValueError):
        bench.resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(ValueError):
        bench.resolve_world(0, {})


def test_rank_launch_command_is_torchrun_on_loopback():
    import bench
    cmd = bench.rank_launch_command(4, ["--gpus", "4", "--steps", "3"], 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_bench_refuses_mismatched_world(monkeypatch):
    """A --gpus that disagrees with the launcher's WORLD_SIZE exits with status 2
    before touching torch or the GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"), "--gpus", "2"], env=env,
        capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=3" in r.stderr


def test_bench_nccl_launch_needs_a_gpu_per_rank():
    """Without enough GPUs the RCCL launch is refused up front (the gloo backend
    rehearses several ranks on fewer GPUs)."""
    import subprocess

    import torch
    if torch.cuda.device_count() >= 2:
        return
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["VBHEM_BENCH_BACKEND"] = "nccl"
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"), "--gpus", "2"], env=env,
        capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "RCCL needs one GPU per rank" in r.stderr

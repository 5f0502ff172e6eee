"""bench.py as the driver runs it for N > 1 (GPU): ``python bench.py --gpus 2`` with
no launcher starts the two rank processes itself (torch.distributed.run, loopback
rendezvous), shards the bases over them and prints ONE JSON line whose n_gpus and
collective.ranks are 2, with the per-rank shard time and the all-reduce time.
On the one-GPU box the ranks share the GPU over the gloo backend
(VBHEM_BENCH_BACKEND=gloo, host-staged all-reduce); RCCL refuses two ranks on one
GPU, so the RCCL path with N > 1 runs only on the driver's multi-GPU node.
Reference reduction point: vbhem_compute_Statistics.m:44-50."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_gpus2_launches_two_ranks():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                        "MASTER_ADDR", "MASTER_PORT")}
    env["VBHEM_BENCH_BACKEND"] = "gloo"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--N", "20000", "--em-iters", "2"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=380, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-4000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    col = res["collective"]
    assert col["ranks"] == 2
    assert col["shard_bases_per_rank"] == [10000, 10000]
    assert len(col["ms_per_step_per_rank"]) == 2
    assert abs(max(col["ms_per_step_per_rank"]) - res["ms_per_step"]) < 1e-9
    assert col["allreduce_ms"] is not None and col["allreduce_ms"] > 0
    assert len(col["allreduce_ms_per_rank"]) == 2
    assert res["value"] > 0 and res["em_iteration"]["iterations"] > 0
    assert res["roofline"]["kernel"] == "vbhem::fb_bwd4_kernel<true>"
    assert res["gated_forward"]["kernel"] == "vbhem::fb_list4_kernel<10, true>"

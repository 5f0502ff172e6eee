"""One C++ EM run (vbhem_em_run, host math on the device) on a C4 shard, for
rocprofv3 --kernel-trace --stats: the per-iteration kernels and their gaps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import pkgload  # noqa: E402

vb = pkgload.load()
from vbhem_amd import native_em  # noqa: E402
from vbhem_amd.estep import EStepEngine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12500
it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device("cuda", 0)
base, post, opt = vb.synth_workload("C4", device=dev, N=100_000, shard=(0, N))
eng = EStepEngine(base, post.K, post.S, opt["tau"], device=dev)
o = dict(opt, minDiff=0.0)
native_em.run(post, eng, o, total_N=100_000, max_iter=1)
for n in (1, it):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = native_em.run(post, eng, o, total_N=100_000, max_iter=n)
    torch.cuda.synchronize()
    print("iterations", r.iters, "ms", (time.perf_counter() - t0) * 1e3, flush=True)

"""Multi-GPU sharding of the E-step: one process per GPU, bases sharded.

Each (base i, cluster j) pair is independent and hat_Z(i,:) depends only on
L_elbo(i,:) (vbhem_h3m_c_step_fc.m:275-276), so rank r owns a contiguous block
of base HMMs and everything up to the packed statistics vector is local.  The
only exchange is ONE all-reduce (sum, fp64) of that vector per EM iteration
(6,930 doubles = 55 KB at K=16,S=8,d=8); cluster posteriors are replicated and every rank
runs the identical host M-step.  On ROCm the "nccl" backend is RCCL (xGMI);
"gloo" serves CPU tests.
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch
import torch.distributed as dist


def shard_range(N: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, near-equal block [lo, hi) of N bases for `rank`."""
    q, r = divmod(N, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def make_allreduce(group=None) -> Callable[[torch.Tensor], None]:
    """In-place SUM all-reduce of the packed statistics (no-op when not initialised
    or world size 1)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return lambda t: None

    def _ar(t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return _ar

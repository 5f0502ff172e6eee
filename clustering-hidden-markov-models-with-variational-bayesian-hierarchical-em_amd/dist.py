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

import ctypes
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


class RcclComm:
    """A native RCCL communicator for the statistics' all-reduce
    (include/vbhem_dist.h): the C++ EM loop (``native_em.run(..., comm=...)``)
    issues ``ncclAllReduce(sum, fp64)`` on its own stream once per E-step, with
    no Python callback in the loop.  Rank 0 makes the id; it travels to the
    other ranks over the already-initialised torch.distributed group (one
    broadcast at set-up).  A world of one rank is allowed (the all-reduce is
    then a local copy) so the path runs on a one-GPU box too."""

    def __init__(self, device: torch.device, rank: int = None, world: int = None, group=None):
        import ctypes

        from . import _capi
        self._lib = _capi.lib()
        inited = dist.is_available() and dist.is_initialized()
        self.rank = (dist.get_rank(group) if inited else 0) if rank is None else int(rank)
        self.world = (dist.get_world_size(group) if inited else 1) if world is None else int(world)
        self.device = torch.device(device)
        # 'cuda' without an index: the rank's current device (torch.cuda.set_device),
        # not GPU 0
        self.device_index = (self.device.index if self.device.index is not None
                             else torch.cuda.current_device())
        self.handle = None
        self.check_ranks_ready(self.rank, self.world, self.device_index, group)
        idb = (ctypes.c_char * _capi.RCCL_ID_BYTES).from_buffer_copy(
            self.exchange_id(self.rank, self.world, group))
        h = ctypes.c_void_p()
        _capi.check(self._lib.vbhem_rccl_comm_init(self.world, self.rank, idb,
                                                   int(self.device_index), ctypes.byref(h)),
                    "vbhem_rccl_comm_init")
        self.handle = h

    @staticmethod
    def local_status(device_index: int):
        """None when this process can bind RCCL and use `device_index`, else why not."""
        from . import _capi
        lib = _capi.lib()
        if lib.vbhem_rccl_available() != 0:
            return lib.vbhem_last_error().decode(errors="replace")
        if not (0 <= device_index < torch.cuda.device_count()):
            return f"device {device_index} not visible ({torch.cuda.device_count()} GPUs)"
        return None

    @classmethod
    def check_ranks_ready(cls, rank: int, world: int, device_index: int, group=None) -> None:
        """Every rank's local status gathered on every rank before any collective
        initialisation; if one rank cannot take part, all of them raise (none is left
        waiting in ncclCommInitRank for it)."""
        from . import _capi
        st = cls.local_status(device_index)
        every = [st]
        if world > 1:
            every = [None] * world
            dist.all_gather_object(every, st, group=group)
        bad = [(r, s) for r, s in enumerate(every) if s is not None]
        if bad:
            raise _capi.VbhemError("RCCL communicator not created: " +
                                   "; ".join(f"rank {r}: {s}" for r, s in bad))

    @staticmethod
    def exchange_id(rank: int, world: int, group=None) -> bytes:
        """Rank 0's communicator id on every rank.  The id -- or rank 0's error --
        reaches every rank, so no rank waits in ncclCommInitRank for a rank 0 that
        could not make one."""
        import ctypes

        from . import _capi
        lib = _capi.lib()
        idb = (ctypes.c_char * _capi.RCCL_ID_BYTES)()
        err = None
        if rank == 0 and lib.vbhem_rccl_unique_id(idb) != 0:
            err = lib.vbhem_last_error().decode(errors="replace")
        out = bytes(idb)
        if world > 1:
            obj = [err if err is not None else out]
            dist.broadcast_object_list(obj, src=0, group=group)
            if isinstance(obj[0], str):
                err = obj[0]
            else:
                out = obj[0]
        if err is not None:
            raise _capi.VbhemError(f"vbhem_rccl_unique_id failed: {err}")
        return out

    def allreduce(self, t: torch.Tensor) -> None:
        """In-place SUM of a device fp64 vector on the current stream."""
        from . import _capi
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.allreduce: a contiguous fp64 device tensor")
        st = torch.cuda.current_stream(t.device).cuda_stream
        _capi.check(self._lib.vbhem_rccl_allreduce_sum(self.handle, _capi.ptr(t), t.numel(), st),
                    "vbhem_rccl_allreduce_sum")

    def allreduce_to(self, t: torch.Tensor, out_dev: int) -> None:
        """allreduce, then the reduced vector copied in-stream by a kernel to the device
        address out_dev (EStepEngine.stats_address: the statistics' pinned host buffer)."""
        from . import _capi
        if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("RcclComm.allreduce_to: a contiguous fp64 device tensor")
        st = torch.cuda.current_stream(t.device).cuda_stream
        _capi.check(self._lib.vbhem_rccl_allreduce_to(self.handle, _capi.ptr(t), t.numel(),
                                                      ctypes.c_void_p(out_dev), st),
                    "vbhem_rccl_allreduce_to")

    def close(self) -> None:
        if self.handle:
            self._lib.vbhem_rccl_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

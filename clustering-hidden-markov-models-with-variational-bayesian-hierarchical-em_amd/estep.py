"""Device-resident E-step engine (one shard of base HMMs on one GPU).

:class:`EStepEngine` owns the HBM copies of the shard's base HMMs, the
per-iteration cluster-constant buffers, the outputs and the workspace, and
enqueues the C-ABI entry points of libvbhem_estep.so on torch's current
stream.  It replaces, per EM iteration, the MEX call of
src/vbhem/vbhem_h3m_c_step_fc.m:168-198 (``pairs``) or the MEX call plus
the responsibilities, statistics reduction and ELBO partial sums
(:270-296, vbhem_compute_Statistics.m) (``fused``).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _capi
from .h3m import COV_FULL, BaseSet

F64 = torch.float64


class EStepEngine:
    def __init__(self, base: BaseSet, K: int, S: int, T: int, device=None, trials: int = 1,
                 prepare: bool = True):
        """K clusters in total; with ``trials`` = R > 1 they are R independent EM
        trials of K / R clusters each, trial-major (vbhem_estep_fused_trials).
        ``prepare``: build the base set's emission-GEMM operand once here
        (vbhem_prepare_base) instead of in every call."""
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("EStepEngine runs on a GPU (HIP); there is no CPU path")
        self.lib = _capi.lib()
        b = base.to(self.device)
        self.base = BaseSet(b.nstates.to(torch.int32).contiguous(), b.prior.to(F64).contiguous(),
                            b.A.to(F64).contiguous(), b.centres.to(F64).contiguous(),
                            b.covars.to(F64).contiguous(), b.omega.to(F64).contiguous(), b.covmode)
        self.K, self.S, self.T = int(K), int(S), int(T)
        N, SB, d = self.base.N, self.base.SB, self.base.d
        dv = self.device
        dC = (d, d) if self.base.covmode == COV_FULL else (d,)
        self.c_logA = torch.zeros((K, S, S), dtype=F64, device=dv)
        self.c_logPi = torch.zeros((K, S), dtype=F64, device=dv)
        self.c_m = torch.zeros((K, S, d), dtype=F64, device=dv)
        self.c_P = torch.zeros((K, S) + dC, dtype=F64, device=dv)
        self.c_c = torch.zeros((K, S), dtype=F64, device=dv)
        self.logOmega = torch.zeros((K,), dtype=F64, device=dv)
        bb = self.base
        self._bt = _capi.BaseT(N, SB, d, bb.covmode, _capi.ptr(bb.nstates), _capi.ptr(bb.prior),
                               _capi.ptr(bb.A), _capi.ptr(bb.centres), _capi.ptr(bb.covars), None)
        self._U = None
        ub = int(self.lib.vbhem_prepare_base_bytes(ctypes.byref(self._bt))) if prepare else 0
        if ub > 0:
            self._U = torch.empty((ub // 8,), dtype=F64, device=dv)
            _capi.check(self.lib.vbhem_prepare_base(ctypes.byref(self._bt), _capi.ptr(self._U), ub,
                                                    self._stream()), "vbhem_prepare_base")
            self._bt.U = _capi.ptr(self._U)
        self._ct = _capi.ClusterT(K, S, _capi.ptr(self.c_logA), _capi.ptr(self.c_logPi),
                                  _capi.ptr(self.c_m), _capi.ptr(self.c_P), _capi.ptr(self.c_c))
        self.trials = int(trials)
        if self.trials < 1 or K % self.trials:
            raise ValueError("K must be a positive multiple of trials")
        self.stats_len = self.trials * int(self.lib.vbhem_stats_len(K // self.trials, S, d,
                                                                       bb.covmode))
        self.stats = torch.zeros((self.stats_len,), dtype=F64, device=dv)
        self.hatZ = torch.zeros((N, K), dtype=F64, device=dv)
        self.LL = torch.zeros((N, K), dtype=F64, device=dv)
        self._ws_fused = None
        self._ws_pairs = None
        self._mapped = {}  # host_stats_buffer data pointer -> (tensor, its device address)
        self._fused_args = {}  # pointers + stream key -> (entry point, name, ctypes arguments)

    # -- inputs -------------------------------------------------------------
    @property
    def N(self) -> int:
        return self.base.N

    def set_clusters(self, consts: dict) -> None:
        """Upload the iteration's cluster constants (host.cluster_constants)."""
        for dst, key in ((self.c_logA, "logA"), (self.c_logPi, "logPi"), (self.c_m, "m"),
                         (self.c_P, "P"), (self.c_c, "c")):
            src = consts[key]
            if isinstance(src, np.ndarray):
                src = torch.from_numpy(np.ascontiguousarray(src, dtype=np.float64))
            dst.copy_(src.reshape(dst.shape))

    def set_log_omega(self, logOmega) -> None:
        src = logOmega
        if isinstance(src, np.ndarray):
            src = torch.from_numpy(np.ascontiguousarray(src, dtype=np.float64))
        self.logOmega.copy_(src)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- MEX-equivalent per-pair outputs ------------------------------------
    def pairs(self, want_tnu: bool = False, smooth=None) -> dict:
        """LL_elbo, sum_nu_1, emit_pr, emit_mu, emit_Mu, sum_xi (+ sum_t_nu), [N][K][...].

        smooth: None = vbhem_hmm_bwd_fwd_mex; a number = the VHEM sibling
        hem_hmm_bwd_fwd_mex (cluster constants from host.vhem_cluster_constants)."""
        N, K, S, d, SB = self.N, self.K, self.S, self.base.d, self.base.SB
        dv = self.device
        dC = (d, d) if self.base.covmode == COV_FULL else (d,)
        out = dict(LL_elbo=torch.empty((N, K), dtype=F64, device=dv),
                   sum_nu_1=torch.empty((N, K, S), dtype=F64, device=dv),
                   emit_pr=torch.empty((N, K, S), dtype=F64, device=dv),
                   emit_mu=torch.empty((N, K, S, d), dtype=F64, device=dv),
                   emit_Mu=torch.empty((N, K, S) + dC, dtype=F64, device=dv),
                   sum_xi=torch.empty((N, K, S, S), dtype=F64, device=dv))
        if want_tnu:
            out["sum_t_nu"] = torch.empty((N, K, S, SB), dtype=F64, device=dv)
        if self._ws_pairs is None:
            nb = int(self.lib.vbhem_pairs_workspace_bytes(ctypes.byref(self._bt),
                                                          ctypes.byref(self._ct), self.T))
            self._ws_pairs = torch.empty((max(nb, 1),), dtype=torch.uint8, device=dv)
        outs = (_capi.ptr(out["LL_elbo"]), _capi.ptr(out["sum_nu_1"]), _capi.ptr(out["emit_pr"]),
                _capi.ptr(out["emit_mu"]), _capi.ptr(out["emit_Mu"]), _capi.ptr(out["sum_xi"]),
                _capi.ptr(out.get("sum_t_nu")), _capi.ptr(self._ws_pairs), self._ws_pairs.numel(),
                self._stream())
        if smooth is None:
            rc = self.lib.vbhem_estep_pairs(ctypes.byref(self._bt), ctypes.byref(self._ct), self.T,
                                            *outs)
            _capi.check(rc, "vbhem_estep_pairs")
        else:
            rc = self.lib.vhem_estep_pairs(ctypes.byref(self._bt), ctypes.byref(self._ct), self.T,
                                           float(smooth), *outs)
            _capi.check(rc, "vhem_estep_pairs")
        return out

    # -- fused E-step --------------------------------------------------------
    def host_stats_buffer(self) -> torch.Tensor:
        """A pinned host vector of stats_len doubles for ``fused(out=...)`` (its
        device address is resolved once, here)."""
        buf = torch.zeros((self.stats_len,), dtype=F64, pin_memory=True)
        self._mapped[buf.data_ptr()] = (buf, self._device_address(buf))
        return buf

    def _device_address(self, host: torch.Tensor) -> int:
        p = ctypes.c_void_p()
        _capi.check(self.lib.vbhem_host_device_pointer(ctypes.c_void_p(host.data_ptr()),
                                                       ctypes.byref(p)), "vbhem_host_device_pointer")
        return int(p.value)

    def stats_address(self, out: torch.Tensor) -> int:
        """The device address a kernel writes ``out`` (a statistics vector: device, or
        pinned host from host_stats_buffer) through."""
        return self._out_ptr(out)

    def _out_ptr(self, out: torch.Tensor) -> int:
        if out.dtype != F64 or not out.is_contiguous() or out.numel() != self.stats_len:
            raise ValueError(f"out must be a contiguous fp64 vector of {self.stats_len} entries")
        if out.is_cuda:
            if out.device != self.device:
                raise ValueError("out is on another device")
            return _capi.ptr(out)
        m = self._mapped.get(out.data_ptr())
        if m is not None and m[0] is out:
            return m[1]
        # pinned host memory: the kernel writes it through its device address
        return self._device_address(out)

    def done_word(self) -> "DoneWord":
        """A completion word for ``fused(done=(word, value))`` (coherent pinned host memory)."""
        return DoneWord(self.lib)

    def fused(self, tildeN: torch.Tensor, out: torch.Tensor = None, done=None) -> torch.Tensor:
        """Pairs + responsibilities + gated Z-weighted sums + ELBO partials.

        tildeN: [N] (device, fp64) virtual-sample counts of this shard.
        Returns the packed statistics vector ([stats_len]): ``self.stats`` on the
        device, or ``out`` when given -- a device vector, or a pinned host vector
        (``host_stats_buffer``) that the statistics kernel writes directly (no
        copy after the E-step; read it after synchronising the stream).  hat_Z and
        L_elbo are left in ``self.hatZ`` / ``self.LL``.  ``done=(word, value)``: the
        call's last kernel stores ``value`` into ``word`` (a DoneWord) once the
        statistics are written and visible to the host (vbhem_arm_done_word), so a host
        running ahead can wait with ``word.wait(value)`` instead of an event."""
        if self._ws_fused is None:
            nb = int(self.lib.vbhem_fused_trials_workspace_bytes(
                ctypes.byref(self._bt), ctypes.byref(self._ct), self.trials, self.T))
            self._ws_fused = torch.empty((max(nb, 1),), dtype=torch.uint8, device=self.device)
        res = self.stats if out is None else out
        sp = _capi.ptr(self.stats) if out is None else self._out_ptr(out)
        st = torch.cuda.current_stream(self.device).cuda_stream
        key = (tildeN.data_ptr(), sp, st)
        if key not in self._fused_args:
            # the call's ctypes arguments, rebuilt only when a pointer or the stream changes
            # (an EM loop repeats the same call: ~4 us of Python per E-step otherwise)
            head = (ctypes.byref(self._bt), ctypes.byref(self._ct))
            head += (self.T,) if self.trials == 1 else (self.trials, self.T)
            args = head + (_capi.ptr(tildeN), _capi.ptr(self.logOmega), sp, _capi.ptr(self.hatZ),
                           _capi.ptr(self.LL), _capi.ptr(self._ws_fused), self._ws_fused.numel(),
                           ctypes.c_void_p(st))
            fn, name = ((self.lib.vbhem_estep_fused, "vbhem_estep_fused") if self.trials == 1 else
                        (self.lib.vbhem_estep_fused_trials, "vbhem_estep_fused_trials"))
            if len(self._fused_args) >= 8:  # (a few buffers / streams alternate at most)
                self._fused_args.clear()
            self._fused_args[key] = (fn, name, args)
        fn, name, args = self._fused_args[key]
        if done is not None:
            word, value = done
            _capi.check(self.lib.vbhem_arm_done_word(ctypes.c_void_p(word.dev), int(value)),
                        "vbhem_arm_done_word")
        _capi.check(fn(*args), name)
        return res

    def fallback_count(self) -> int:
        """Pairs of the last fused call that needed the exact fallback (syncs)."""
        ws = self._ws_fused if self._ws_fused is not None else self._ws_pairs
        if ws is None:
            return 0
        n = self.lib.vbhem_last_fallback_count(self._stream(), ctypes.c_void_p(_capi.ptr(ws)))
        if n < 0:
            _capi.check(n, "vbhem_last_fallback_count")
        return int(n)


class DoneWord:
    """A 64-bit completion word in coherent pinned host memory (vbhem_done_word_alloc):
    ``EStepEngine.fused(done=(word, v))`` has the E-step's last kernel store v into it
    once the statistics are visible to the host; ``wait(v)`` spins until it reads >= v."""

    def __init__(self, lib):
        self.lib = lib
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _capi.check(lib.vbhem_done_word_alloc(ctypes.byref(h), ctypes.byref(d)), "vbhem_done_word_alloc")
        self.host, self.dev = int(h.value), int(d.value)
        self._word = ctypes.c_uint64.from_address(self.host)

    @property
    def value(self) -> int:
        return int(self._word.value)

    def wait(self, value: int, timeout_s: float = 60.0) -> None:
        """Spin until the word reads >= value (ctypes re-reads the memory every time)."""
        import time
        w = self._word
        if w.value >= value:
            return
        t0 = time.perf_counter()
        while w.value < value:
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"done word {w.value} < {value} after {timeout_s} s")

    def __del__(self):
        try:
            if self.host:
                self.lib.vbhem_done_word_free(ctypes.c_void_p(self.host))
                self.host = 0
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

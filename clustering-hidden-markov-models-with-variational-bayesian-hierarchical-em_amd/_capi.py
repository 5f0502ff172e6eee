"""ctypes binding of libvbhem_estep.so (include/vbhem_estep.h).

The library is built in-tree (``make lib`` / ``__graft_entry__.build()``) into
``<package>/lib/``.  torch is imported first so that the library binds to the
HIP runtime torch already loaded (both carry SONAME libamdhip64.so.7); device
buffers are torch tensors and the stream is torch's current stream.

There is no CPU fallback: if the library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)

HERE = os.path.dirname(os.path.abspath(__file__))
# VBHEM_LIB_PATH: another build of the same library (A/B experiments)
LIB_PATH = os.environ.get("VBHEM_LIB_PATH") or os.path.join(HERE, "lib", "libvbhem_estep.so")

VBHEM_COV_DIAG, VBHEM_COV_FULL = 0, 1
_c_int, _c_size, _vp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p


class BaseT(ctypes.Structure):
    _fields_ = [("N", _c_int), ("SB", _c_int), ("d", _c_int), ("covmode", _c_int),
                ("nstates", _vp), ("prior", _vp), ("A", _vp), ("centres", _vp), ("covars", _vp),
                ("U", _vp)]


class ClusterT(ctypes.Structure):
    _fields_ = [("K", _c_int), ("S", _c_int), ("logA", _vp), ("logPi", _vp), ("m", _vp),
                ("P", _vp), ("c", _vp)]


class PostT(ctypes.Structure):  # include/vbhem_em.h vbhem_post_t
    _fields_ = [("K", _c_int), ("S", _c_int), ("d", _c_int), ("covmode", _c_int),
                ("alpha", _vp), ("eta", _vp), ("epsilon", _vp), ("lam", _vp), ("v", _vp),
                ("m", _vp), ("W", _vp)]


class EmOptT(ctypes.Structure):  # include/vbhem_em.h vbhem_em_opt_t
    _fields_ = [("alpha0", ctypes.c_double), ("eta0", ctypes.c_double),
                ("epsilon0", ctypes.c_double), ("lambda0", ctypes.c_double),
                ("v0", ctypes.c_double), ("m0", _vp), ("W0", _vp), ("W0_len", _c_int),
                ("Nv", ctypes.c_double), ("max_iter", _c_int), ("minDiff", ctypes.c_double)]


class SeqsT(ctypes.Structure):  # include/vbhmm_fb.h vbhmm_seqs_t
    _fields_ = [("N", _c_int), ("dim", _c_int), ("maxT", _c_int), ("offsets", _vp), ("x", _vp)]


class HmmParamsT(ctypes.Structure):  # include/vbhmm_fb.h vbhmm_params_t
    _fields_ = [("K", _c_int), ("dim", _c_int), ("m", _vp), ("W", _vp), ("v", _vp), ("beta", _vp),
                ("logLambdaTilde", _vp), ("pz1", _vp), ("A", _vp),
                ("const_denominator", ctypes.c_double)]


class EmExtT(ctypes.Structure):  # include/vbhem_em.h vbhem_em_ext_t
    _fields_ = [("rccl_comm", _vp), ("iter_seconds", _vp), ("calc_deriv", _c_int), ("dLL", _vp)]


ALLREDUCE_FN = ctypes.CFUNCTYPE(_c_int, _vp, _c_size, _vp, _vp)
RCCL_ID_BYTES = 128  # include/vbhem_dist.h VBHEM_RCCL_ID_BYTES

EXPORTS = {
    "vbhem_prepare_base_bytes": (_c_size, [ctypes.POINTER(BaseT)]),
    "vbhem_prepare_base": (_c_int, [ctypes.POINTER(BaseT), _vp, _c_size, _vp]),
    "vbhem_pairs_workspace_bytes": (_c_size, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int]),
    "vbhem_estep_pairs": (_c_int, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "vbhem_estep_pairs_host": (_c_int, [_c_int, ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int,
                                        _vp, _vp, _vp, _vp, _vp, _vp]),
    "vhem_estep_pairs": (_c_int, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int,
                                  ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _c_size, _vp]),
    "vhem_estep_pairs_host": (_c_int, [_c_int, ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT),
                                       _c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _vp, _vp]),
    "vbhem_stats_nu": (_c_size, [_c_int, _c_int]),
    "vbhem_stats_len": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "vbhem_fused_workspace_bytes": (_c_size, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int]),
    "vbhem_estep_fused": (_c_int, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int,
                                   _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "vbhem_fused_trials_workspace_bytes": (_c_size, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT),
                                                     _c_int, _c_int]),
    "vbhem_estep_fused_trials": (_c_int, [ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT), _c_int,
                                          _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "vbhem_last_fallback_count": (_c_int, [_vp, _vp]),
    "vbhem_host_device_pointer": (_c_int, [_vp, ctypes.POINTER(_vp)]),
    "vbhem_arm_done_word": (_c_int, [_vp, ctypes.c_ulonglong]),
    "vbhem_done_word_alloc": (_c_int, [ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "vbhem_done_word_free": (_c_int, [_vp]),
    "vbhem_ctx_create": (_c_int, [_c_int, ctypes.POINTER(BaseT), _c_int, _c_int, _c_int, _c_int,
                                  ctypes.POINTER(_vp)]),
    "vbhem_ctx_fused": (_c_int, [_vp, ctypes.POINTER(ClusterT), _vp, _vp, _vp, _vp, _vp]),
    "vbhem_ctx_destroy": (None, [_vp]),
    "vbhem_estep_fused_host": (_c_int, [_c_int, ctypes.POINTER(BaseT), ctypes.POINTER(ClusterT),
                                        _c_int, _vp, _vp, _vp, _vp, _vp]),
    "vbhem_timing_enable": (_c_int, [_c_int]),
    "vbhem_timing_read": (_c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                                   ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_longlong)]),
    "vbhem_timing_read_emission": (_c_int, [ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_longlong)]),
    "vbhem_timing_read_gated": (_c_int, [ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_longlong)]),
    "vbhem_timing_read_em_math": (_c_int, [ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_longlong)]),
    "vbhem_set_fused_mode": (_c_int, [_c_int]),
    "vbhem_debug_extra_lds": (_c_size, [_c_size]),
    "vbhem_em_prelude": (_c_int, [ctypes.POINTER(PostT), _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "vbhem_em_lower_bound": (_c_int, [ctypes.POINTER(PostT), ctypes.POINTER(EmOptT), _vp, _vp,
                                      _vp, _vp, _vp, ctypes.POINTER(ctypes.c_double)]),
    "vbhem_em_mstep": (_c_int, [ctypes.POINTER(EmOptT), _vp, ctypes.POINTER(PostT)]),
    "vbhem_em_host_iteration": (_c_int, [ctypes.POINTER(EmOptT), _vp, ctypes.POINTER(PostT), _vp,
                                         _vp, _vp, _vp, _vp, _vp, _vp,
                                         ctypes.POINTER(ctypes.c_double)]),
    "vbhem_em_workspace_bytes": (_c_size, [ctypes.POINTER(BaseT), _c_int, _c_int, _c_int]),
    "vbhem_em_run": (_c_int, [ctypes.POINTER(BaseT), _vp, _c_int, ctypes.POINTER(EmOptT),
                              ctypes.POINTER(PostT), _vp, ctypes.POINTER(_c_int),
                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int), _vp, _vp,
                              _vp, _vp, _c_size, _vp, ALLREDUCE_FN, _vp]),
    "vbhem_em_run_ext": (_c_int, [ctypes.POINTER(BaseT), _vp, _c_int, ctypes.POINTER(EmOptT),
                                  ctypes.POINTER(PostT), _vp, ctypes.POINTER(_c_int),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int), _vp, _vp,
                                  _vp, _vp, _c_size, _vp, ALLREDUCE_FN, _vp,
                                  ctypes.POINTER(EmExtT)]),
    "vbhem_em_lower_bound_derivs": (_c_int, [ctypes.POINTER(PostT), ctypes.POINTER(EmOptT), _vp,
                                             _vp, _vp, _vp, _vp]),
    "vbhem_hmms_to_h3m": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int] + [_vp] * 15),
    "vbhem_rccl_available": (_c_int, []),
    "vbhem_rccl_unique_id": (_c_int, [_vp]),
    "vbhem_rccl_comm_init": (_c_int, [_c_int, _c_int, _vp, _c_int, ctypes.POINTER(_vp)]),
    "vbhem_rccl_comm_destroy": (_c_int, [_vp]),
    "vbhem_rccl_allreduce_sum": (_c_int, [_vp, _vp, _c_size, _vp]),
    "vbhem_rccl_allreduce_to": (_c_int, [_vp, _vp, _c_size, _vp, _vp]),
    "vbhmm_fb_workspace_bytes": (_c_size, [ctypes.POINTER(SeqsT), _c_int]),
    "vbhmm_fb": (_c_int, [ctypes.POINTER(SeqsT), ctypes.POINTER(HmmParamsT), _vp, _vp, _vp, _vp, _vp,
                          _c_size, _vp]),
    "vbhmm_fb_host": (_c_int, [_c_int, ctypes.POINTER(SeqsT), ctypes.POINTER(HmmParamsT), _vp, _vp,
                               _vp, _vp]),
    "vbhem_last_error": (ctypes.c_char_p, []),
    "vbhem_last_kernel": (ctypes.c_char_p, [_c_int]),
    "vbhem_version": (ctypes.c_char_p, []),
}

_LIB = None


class VbhemError(RuntimeError):
    pass


def lib():
    """Load (once) and return the CDLL; raises if the HIP library is absent."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libvbhem_estep.so not found at {LIB_PATH}; build it with `make lib` "
                "(or __graft_entry__.build()).  There is no CPU fallback.")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = h
    return _LIB


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().vbhem_last_error().decode(errors="replace")
        raise VbhemError(f"{what} failed (status {rc}): {msg}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def timing_enable(on: bool = True, fb_only: bool = False) -> None:
    """Kernel timing on this thread: every timed launch, or (fb_only) the fb
    launches alone (two events per E-step)."""
    lib().vbhem_timing_enable((2 if fb_only else 1) if on else 0)


def timing_read() -> dict:
    """Summed HIP-event times of the fb/stats kernel launches since the last read."""
    fb, st = ctypes.c_double(), ctypes.c_double()
    nf, npairs, ns = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong()
    check(lib().vbhem_timing_read(ctypes.byref(fb), ctypes.byref(nf), ctypes.byref(npairs),
                                  ctypes.byref(st), ctypes.byref(ns)), "vbhem_timing_read")
    em, ne = ctypes.c_double(), ctypes.c_longlong()
    check(lib().vbhem_timing_read_emission(ctypes.byref(em), ctypes.byref(ne)),
          "vbhem_timing_read_emission")
    gf, ng = ctypes.c_double(), ctypes.c_longlong()
    check(lib().vbhem_timing_read_gated(ctypes.byref(gf), ctypes.byref(ng)),
          "vbhem_timing_read_gated")
    mm, nm = ctypes.c_double(), ctypes.c_longlong()
    check(lib().vbhem_timing_read_em_math(ctypes.byref(mm), ctypes.byref(nm)),
          "vbhem_timing_read_em_math")
    return dict(fb_ms=fb.value, fb_launches=nf.value, fb_pairs=npairs.value,
                stats_ms=st.value, stats_launches=ns.value, em_ms=em.value, em_launches=ne.value,
                gated_fwd_ms=gf.value, gated_fwd_launches=ng.value, em_math_ms=mm.value,
                em_math_launches=nm.value)


def last_kernel(pass_: int) -> str:
    """The kernel this thread's last E-step ran for recursion pass 0 (every pair) or
    1 (the gate-list pass), as the kernel trace names it ("" before any)."""
    return lib().vbhem_last_kernel(int(pass_)).decode()


FUSED_GATED, FUSED_DENSE = 0, 1


def set_fused_mode(mode: int) -> int:
    """Fused E-step schedule (FUSED_GATED default, FUSED_DENSE); returns the previous one."""
    return int(lib().vbhem_set_fused_mode(int(mode)))

"""The C-ABI library (CPU side): it loads, exports every entry point that
include/*.h declare, and its size queries / argument validation
behave as documented -- without launching anything (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import LIB_PATH, ROOT

HEADER = os.path.join(ROOT, "include", "vbhem_estep.h")


def declared_functions():
    src = "".join(open(os.path.join(ROOT, "include", h)).read()
                  for h in sorted(os.listdir(os.path.join(ROOT, "include"))) if h.endswith(".h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b((?:vbhem|vhem|vbhmm)_[a-z0-9_]+)\s*\(", src)))


def header_constants():
    vals = {}
    for name, v in re.findall(r"#define\s+(VBHEM_[A-Z_]+)\s+\(?(-?\d+)\)?", open(HEADER).read()):
        vals[name] = int(v)
    return vals


def test_header_declares_the_api():
    fns = declared_functions()
    for f in ("vbhem_estep_pairs", "vbhem_estep_pairs_host", "vbhem_estep_fused",
              "vbhem_pairs_workspace_bytes", "vbhem_fused_workspace_bytes", "vbhem_stats_len",
              "vbhem_stats_nu", "vbhem_last_error", "vbhem_version", "vbhem_last_fallback_count",
              "vbhem_timing_enable", "vbhem_timing_read"):
        assert f in fns, f


def test_library_exports_every_declared_symbol(capi_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert hasattr(capi_lib, f)


def test_python_binding_table_matches_header(vb, capi_lib):
    from vbhem_amd import _capi
    assert set(_capi.EXPORTS) == set(declared_functions())


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_version_and_sizes(capi_lib):
    from vbhem_amd import host
    assert b"gfx950" in capi_lib.vbhem_version()
    c = header_constants()
    for d in (1, 2, 8, 16):
        assert capi_lib.vbhem_stats_nu(d, c["VBHEM_COV_FULL"]) == host.stats_nu(d, 1)
        assert capi_lib.vbhem_stats_nu(d, c["VBHEM_COV_DIAG"]) == host.stats_nu(d, 0)
        for K, S in ((1, 1), (16, 8), (32, 12)):
            for cov in (0, 1):
                assert capi_lib.vbhem_stats_len(K, S, d, cov) == host.stats_len(K, S, d, cov)
    assert capi_lib.vbhem_stats_len(16, 8, 8, 1) == 6930    # 55 KB all-reduce per iteration at C4


def _descs(N=10, SB=3, d=2, cov=1, K=2, S=3, fake=1 << 20):
    from vbhem_amd import _capi
    p = fake  # never dereferenced: every call below fails validation first
    b = _capi.BaseT(N, SB, d, cov, p, p, p, p, p)
    c = _capi.ClusterT(K, S, p, p, p, p, p)
    return b, c


def test_workspace_queries(capi_lib):
    b, c = _descs()
    assert capi_lib.vbhem_pairs_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 10) > 0
    assert capi_lib.vbhem_fused_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 10) > 0
    b2, c2 = _descs(N=1000)
    assert (capi_lib.vbhem_pairs_workspace_bytes(ctypes.byref(b2), ctypes.byref(c2), 10) >
            capi_lib.vbhem_pairs_workspace_bytes(ctypes.byref(b), ctypes.byref(c), 10))
    bad, cc = _descs(cov=7)
    assert capi_lib.vbhem_pairs_workspace_bytes(ctypes.byref(bad), ctypes.byref(cc), 10) == 0


def _pairs_call(lib, b, c, T, out=1 << 20, ws=1 << 20, ws_bytes=1 << 40):
    v = ctypes.c_void_p(out)
    return lib.vbhem_estep_pairs(ctypes.byref(b) if b is not None else None,
                                 ctypes.byref(c) if c is not None else None, T,
                                 v, v, v, v, v, v, None, ctypes.c_void_p(ws), ctypes.c_size_t(ws_bytes),
                                 None)


def test_argument_validation(capi_lib):
    k = header_constants()
    b, c = _descs()
    assert _pairs_call(capi_lib, None, c, 10) == k["VBHEM_ERR_ARG"]
    assert b"null" in capi_lib.vbhem_last_error()
    assert _pairs_call(capi_lib, b, c, 0) == k["VBHEM_ERR_ARG"]
    bd, cd = _descs(cov=5)
    assert _pairs_call(capi_lib, bd, cd, 10) == k["VBHEM_ERR_ARG"]
    assert b"covmode" in capi_lib.vbhem_last_error()
    bz, cz = _descs(K=0)
    assert _pairs_call(capi_lib, bz, cz, 10) == k["VBHEM_ERR_ARG"]
    bn, cn = _descs(fake=0)
    assert _pairs_call(capi_lib, bn, cn, 10) == k["VBHEM_ERR_ARG"]
    # workspace too small
    assert _pairs_call(capi_lib, b, c, 10, ws_bytes=16) == k["VBHEM_ERR_WORKSPACE"]
    assert b"workspace" in capi_lib.vbhem_last_error()
    # null outputs
    assert capi_lib.vbhem_estep_pairs(ctypes.byref(b), ctypes.byref(c), 10, None, None, None, None,
                                      None, None, None, None, ctypes.c_size_t(0), None) \
        == k["VBHEM_ERR_ARG"]
    # empty shard is a no-op (nothing launched)
    b0, c0 = _descs(N=0)
    assert _pairs_call(capi_lib, b0, c0, 10) == k["VBHEM_OK"]


def test_unsupported_shape_is_reported(capi_lib):
    k = header_constants()
    b, c = _descs(SB=30, S=30, d=2)
    assert _pairs_call(capi_lib, b, c, 10) == k["VBHEM_ERR_UNSUPPORTED"]
    assert b"LDS" in capi_lib.vbhem_last_error()
    # N*K beyond 2^31-1 pairs per call
    b2, c2 = _descs(N=2_000_000_000, K=4)
    assert _pairs_call(capi_lib, b2, c2, 10) == k["VBHEM_ERR_UNSUPPORTED"]


def test_missing_library_fails_loudly(vb, monkeypatch):
    from vbhem_amd import _capi
    monkeypatch.setattr(_capi, "LIB_PATH", os.path.join(ROOT, "nonexistent", "libvbhem_estep.so"))
    monkeypatch.setattr(_capi, "_LIB", None)
    with pytest.raises(ImportError):
        _capi.lib()


def test_engine_refuses_cpu_device(vb):
    from vbhem_amd.estep import EStepEngine
    base, P, opt = vb.synth_workload("C2", N=4)
    with pytest.raises(ValueError):
        EStepEngine(base, P.K, P.S, opt["tau"], device="cpu")

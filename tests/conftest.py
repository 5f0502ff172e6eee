"""Shared test fixtures.

Markers: ``gpu`` -- needs an MI355X and the built HIP library (run on the GPU
box with ``pytest -m gpu``); everything else runs on the CPU.  The oracle
(oracle/) is imported here only as the checker.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402  (before any ctypes load of HIP code: shares torch's HIP runtime)

import pkgload  # noqa: E402
import vbhem_oracle  # noqa: E402

PKG_DIR = pkgload.PKG_DIR
LIB_PATH = os.path.join(PKG_DIR, "lib", "libvbhem_estep.so")
GATEWAY_PATH = os.path.join(PKG_DIR, "lib", "vbhem_hmm_bwd_fwd_mex.so")
HEM_GATEWAY_PATH = os.path.join(PKG_DIR, "lib", "hem_hmm_bwd_fwd_mex.so")
FB_GATEWAY_PATH = os.path.join(PKG_DIR, "lib", "vbhmm_fb_mex.so")
FUSED_GATEWAY_PATH = os.path.join(PKG_DIR, "lib", "vbhem_estep_fused_mex.so")
MXSHIM_PATH = os.path.join(ROOT, "tests", "mxshim", "libmxshim.so")
MATHCHECK_PATH = os.path.join(ROOT, "tests", "mathcheck", "libmathcheck.so")
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")

# Parity tolerance for floating-point outputs (SURVEY.md section 8c / BASELINE.json
# north_star): hat_Z, posteriors and ELBO within 1e-5 relative.  The per-pair
# outputs are checked much tighter (RTOL_PAIRS) because the GPU path is an exact
# re-association of the same arithmetic.
RTOL_NORTH_STAR = 1e-5
RTOL_PAIRS = 1e-10


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: multi-process or large CPU test")


def _have_gpu():
    try:
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _have_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def _make(*targets):
    subprocess.run(["make", "-C", ROOT, *targets], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def vb():
    return pkgload.load()


@pytest.fixture(scope="session")
def vo():
    vbhem_oracle.load_c_oracle()
    return vbhem_oracle


@pytest.fixture(scope="session")
def capi_lib():
    """libvbhem_estep.so loaded through the product's loader (fails if missing)."""
    if not os.path.exists(LIB_PATH):
        _make("lib")
    vb_ = pkgload.load()
    from vbhem_amd import _capi
    del vb_
    return _capi.lib()


@pytest.fixture(scope="session")
def gateway():
    """(mexFunction, mxshim) -- the MEX gateway built against the mx test double."""
    if not (os.path.exists(GATEWAY_PATH) and os.path.exists(MXSHIM_PATH)):
        _make("mex")
    shim = ctypes.CDLL(MXSHIM_PATH, mode=ctypes.RTLD_GLOBAL)
    gw = ctypes.CDLL(GATEWAY_PATH, mode=ctypes.RTLD_GLOBAL)
    return gw, shim


@pytest.fixture(scope="session")
def hem_gateway():
    """(mexFunction of the VHEM sibling gateway, mxshim)."""
    if not (os.path.exists(HEM_GATEWAY_PATH) and os.path.exists(MXSHIM_PATH)):
        _make("mex")
    shim = ctypes.CDLL(MXSHIM_PATH, mode=ctypes.RTLD_GLOBAL)
    gw = ctypes.CDLL(HEM_GATEWAY_PATH, mode=ctypes.RTLD_GLOBAL)
    return gw, shim


@pytest.fixture(scope="session")
def fb_gateway():
    """(mexFunction of the vbhmm_fb_mex gateway, mxshim)."""
    if not (os.path.exists(FB_GATEWAY_PATH) and os.path.exists(MXSHIM_PATH)):
        _make("mex")
    shim = ctypes.CDLL(MXSHIM_PATH, mode=ctypes.RTLD_GLOBAL)
    gw = ctypes.CDLL(FB_GATEWAY_PATH, mode=ctypes.RTLD_GLOBAL)
    return gw, shim


@pytest.fixture(scope="session")
def fused_gateway():
    """(mexFunction of the fused E-step gateway, mxshim)."""
    if not (os.path.exists(FUSED_GATEWAY_PATH) and os.path.exists(MXSHIM_PATH)):
        _make("mex")
    shim = ctypes.CDLL(MXSHIM_PATH, mode=ctypes.RTLD_GLOBAL)
    gw = ctypes.CDLL(FUSED_GATEWAY_PATH, mode=ctypes.RTLD_GLOBAL)
    return gw, shim


@pytest.fixture(scope="session")
def mathcheck():
    if not os.path.exists(MATHCHECK_PATH):
        _make("mathcheck")
    lib = ctypes.CDLL(MATHCHECK_PATH)
    dp = ctypes.POINTER(ctypes.c_double)
    lib.mathcheck_host.argtypes = [ctypes.c_int, dp, dp, dp, dp]
    lib.mathcheck_host.restype = None
    lib.mathcheck_device.argtypes = [ctypes.c_int, dp, dp, dp, dp]
    lib.mathcheck_device.restype = ctypes.c_int
    lib.logtab_host.argtypes = [ctypes.c_int, dp, dp, dp]
    lib.logtab_host.restype = None
    lib.logtab_device.argtypes = [ctypes.c_int, dp, dp, dp]
    lib.logtab_device.restype = ctypes.c_int
    for name in ("logtabf_host", "logtabc_host", "logtabe_host"):
        getattr(lib, name).argtypes = [ctypes.c_int, dp, dp, dp]
        getattr(lib, name).restype = None
    for name in ("logtabf_device", "logtabc_device", "logtabe_device"):
        getattr(lib, name).argtypes = [ctypes.c_int, dp, dp, dp]
        getattr(lib, name).restype = ctypes.c_int
    return lib


def rel_err(a, b, floor=1e-300):
    """Normwise: max|a - b| / max|b| (an extra check; the parity gates use elem_err)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.size == 0:
        return 0.0
    scale = max(np.abs(b).max(), floor)
    return float(np.abs(a - b).max() / scale)


# hat_Z entries below 1e-8 are compared in absolute terms (Nv = 100
# makes hat_Z nearly one-hot); everything else element by element.
ZHAT_ABS_FLOOR = 1e-8


def elem_err(a, b, floor_abs=0.0, floor_rel=0.0):
    """Elementwise relative error  max_i |a_i - b_i| / max(|b_i|, floor),
    floor = max(floor_abs, floor_rel * max|b|): every entry at or above the floor
    is held to the relative bound on its own, entries below it to rtol * floor
    absolutely.  NaN in either operand counts as an infinite error unless both
    are NaN at the same place."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.size == 0:
        return 0.0
    both_nan = np.isnan(a) & np.isnan(b)
    if (np.isnan(a) ^ np.isnan(b)).any():
        return float("inf")
    floor = max(floor_abs, floor_rel * float(np.abs(np.where(both_nan, 0.0, b)).max()), 1e-300)
    d = np.where(both_nan, 0.0, np.abs(a - b))
    return float((d / np.maximum(np.abs(np.where(both_nan, 1.0, b)), floor)).max())


def hatz_err(a, b):
    """hat_Z parity metric (elementwise, absolute below ZHAT_ABS_FLOOR)."""
    return elem_err(a, b, floor_abs=ZHAT_ABS_FLOOR)


def post_err(a, b):
    """Posterior parity metric (north-star 1e-5): elementwise relative, with an
    absolute floor of 1e-8 of the array's largest entry (entries that are zero up
    to cancellation, e.g. a mean coordinate at the origin)."""
    return elem_err(a, b, floor_rel=1e-8)


def stat_err(a, b):
    """Statistics parity metric for the tight (1e-9 .. 1e-10) bounds: elementwise
    relative with a floor of 1e-5 of the largest entry.  Sums whose terms cancel
    (first moments of means near the origin) are only determined to ~1e-16 of
    the sum of |terms|, so entries far below the largest are held absolutely."""
    return elem_err(a, b, floor_rel=1e-5)

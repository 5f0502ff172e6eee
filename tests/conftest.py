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
    for name in ("logtabf_host",):
        getattr(lib, name).argtypes = [ctypes.c_int, dp, dp, dp]
        getattr(lib, name).restype = None
    lib.logtabf_device.argtypes = [ctypes.c_int, dp, dp, dp]
    lib.logtabf_device.restype = ctypes.c_int
    return lib


def rel_err(a, b, floor=1e-300):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.size == 0:
        return 0.0
    scale = max(np.abs(b).max(), floor)
    return float(np.abs(a - b).max() / scale)

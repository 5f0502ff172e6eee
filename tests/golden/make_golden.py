"""Generate the golden fixtures in tests/golden/ (inputs + expected outputs).

PARITY UNPINNED: the reference repository ships no fixtures or golden vectors,
MATLAB/Octave are not available, and the reference MEX cannot be built here
(it needs MATLAB's mex.h/libmx).  These vectors therefore come from the C
restatement of the MEX (oracle/vbhem_oracle.c, cross-checked against the numpy
twin restatement and closed-form answers in tests/test_oracle.py).  They pin
the oracle and the HIP path against regressions and make the GPU parity tests
independent of re-running the oracle.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402,F401

import pkgload  # noqa: E402
import vbhem_oracle as vo  # noqa: E402
from cases import make_case, post_dict  # noqa: E402

vb = pkgload.load()

PAIR_KEYS = ("LL_elbo", "sum_nu_1", "sum_xi", "emit_pr", "emit_mu", "emit_Mu")


def fused_expected(base, consts, alpha, T, pairs):
    N = base["prior"].shape[0]
    tN = 100.0 * N * base["omega"]
    logOmega, hz, Z, Nj = vo.responsibilities(pairs["LL_elbo"], tN, alpha)
    st = vo.c_statistics(Z, pairs, base["covmode"])
    return dict(tildeN=tN, logOmega=logOmega, hatZ=hz, Nj=st["Nj"], N1=st["N1"], M=st["M"],
                Nr=st["Nr"], Y=st["Y"], SC=st["SC"], Lt1=float((Z * pairs["LL_elbo"]).sum()),
                Lt7=float((hz * np.log(hz)).sum()))


def save_pairs_case(name, base, consts, alpha, T, want_tnu=True):
    pairs = vo.c_estep_pairs(base, consts, T, nthreads=4, want_tnu=want_tnu)
    fz = fused_expected(base, consts, alpha, T, pairs)
    arrays = {"in_" + k: np.asarray(base[k]) for k in ("nstates", "prior", "A", "centres", "covars",
                                                       "omega")}
    arrays.update({"c_" + k: np.asarray(consts[k]) for k in ("logA", "logPi", "m", "P", "c")})
    arrays.update({"out_" + k: v for k, v in pairs.items()})
    arrays.update({"fz_" + k: np.asarray(v) for k, v in fz.items()})
    arrays.update(covmode=np.int32(base["covmode"]), T=np.int32(T), alpha=np.asarray(alpha))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    return path


def main():
    out = []
    # C2 (Synthetic_experiment/exprmt1: 2 GT HMMs, d=2, Sb=2, S=3, K=4, tau=50), 12 bases
    base, P, opt = vb.synth_workload("C2", N=12)
    b = base.numpy()
    out.append(save_pairs_case("pairs_c2", b, vb.host.cluster_constants(P, 1), P.alpha, opt["tau"]))
    # C3-shaped (diag, d=2), ragged state counts, perturbed clusters
    cs = make_case(10, 8, 5, 5, 2, 0, seed=303, ragged=True, tau=10)
    out.append(save_pairs_case("pairs_c3_ragged_diag", cs["base"], cs["consts"], cs["post"]["alpha"], 10))
    # C4-shaped (full, d=8, S=Sb=8, K=16), 2 bases
    cs = make_case(2, 16, 8, 8, 8, 1, seed=404, tau=10)
    out.append(save_pairs_case("pairs_c4", cs["base"], cs["consts"], cs["post"]["alpha"], 10))
    # C5-shaped (full, d=16, S=Sb=12, K=32), 1 base
    cs = make_case(1, 32, 12, 12, 16, 1, seed=505, tau=10)
    out.append(save_pairs_case("pairs_c5", cs["base"], cs["consts"], cs["post"]["alpha"], 10,
                               want_tnu=False))
    # EM trajectory: full C2 config (N=100), oracle loop-style EM to convergence
    base, P, opt = vb.synth_workload("C2")
    b = base.numpy()
    ref = vo.em_step_fc(post_dict(P), b, opt)
    arrays = {"in_" + k: np.asarray(b[k]) for k in ("nstates", "prior", "A", "centres", "covars",
                                                    "omega")}
    arrays.update({"init_" + k: np.asarray(v) for k, v in post_dict(P).items() if k != "W0mode"})
    arrays.update({"post_" + k: np.asarray(v) for k, v in ref["post"].items() if k != "W0mode"})
    arrays.update(LogLs=ref["LogLs"], LL=ref["LL"], hat_Z=ref["hat_Z"], label=ref["label"],
                  iters=ref["iters"], covmode=np.int32(1), T=np.int32(opt["tau"]))
    path = os.path.join(HERE, "em_c2.npz")
    np.savez_compressed(path, **arrays)
    out.append(path)
    for p in out:
        print(f"{os.path.relpath(p, ROOT)}: {os.path.getsize(p)} bytes")


if __name__ == "__main__":
    main()

"""Generates tests/golden/demo_fixations.npz: the fixation sequences of the
reference's demo/demodata.xls, flattened: x [sum T][2], offsets [n_trials+1],
subject index per trial, and the subject / trial names.

The cells come from tests/golden/biff_cells.py, a minimal compound-file + BIFF8
walker written separately from vbhem_amd/xls.py (the reader the fixture checks),
with the row loop of read_xls_fixations.m:84-138.  Run in a container that has
/root/reference mounted:

    python tests/golden/make_demo_fixations.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import biff_cells  # noqa: E402

SRC = "/root/reference/demo/demodata.xls"


def main():
    data, names, trials = biff_cells.read_fixations(SRC)
    seqs = [t for subj in data for t in subj]
    subj = np.array([s for s, subjd in enumerate(data) for _ in subjd], dtype=np.int32)
    off = np.zeros(len(seqs) + 1, dtype=np.int32)
    off[1:] = np.cumsum([len(t) for t in seqs])
    np.savez_compressed(os.path.join(os.path.dirname(__file__), "demo_fixations.npz"),
                        x=np.concatenate(seqs), offsets=off, subject=subj,
                        names=np.array(names), trials=np.array([t for tr in trials for t in tr]))


if __name__ == "__main__":
    main()

"""Clustering scores of the reference's synthetic experiments
(Synthetic_experiment/evaluate_vbhem_jounarl.m:86-122, syn_evluate.m): the Rand
indices of src/compare_mtds/eva/valid_RandIndex.m and the purity of
src/compare_mtds/eva/Purity.m, restated for numpy label vectors (any integer
labels; the reference's are 1-based)."""
from __future__ import annotations

import numpy as np


def contingency(c1, c2) -> np.ndarray:
    """valid_RandIndex.m:44-55: counts of (c1 label, c2 label) pairs."""
    a = np.unique(np.asarray(c1), return_inverse=True)[1].ravel()
    b = np.unique(np.asarray(c2), return_inverse=True)[1].ravel()
    C = np.zeros((a.max() + 1 if a.size else 0, b.max() + 1 if b.size else 0))
    np.add.at(C, (a, b), 1.0)
    return C


def rand_index(c1, c2):
    """(RI, AR, MI, HI) of valid_RandIndex(c1, c2) (:18-42): the Rand index, the
    Hubert-Arabie adjusted Rand index, Mirkin's and Hubert's indices."""
    c1 = np.asarray(c1).ravel()
    c2 = np.asarray(c2).ravel()
    if c1.size != c2.size or c1.size < 2:
        raise ValueError("rand_index: two label vectors of the same length >= 2")
    C = contingency(c1, c2)
    n = C.sum()
    nis = (C.sum(axis=1) ** 2).sum()
    njs = (C.sum(axis=0) ** 2).sum()
    t1 = n * (n - 1) / 2.0
    t2 = (C ** 2).sum()
    t3 = 0.5 * (nis + njs)
    nc = (n * (n ** 2 + 1) - (n + 1) * nis - (n + 1) * njs + 2 * (nis * njs) / n) / (2 * (n - 1))
    A = t1 + t2 - t3
    D = -t2 + t3
    AR = 0.0 if t1 == nc else (A - nc) / (t1 - nc)
    return A / t1, AR, D / t1, (A - D) / t1


def purity(labels, clusters) -> float:
    """Purity.m:7-19: the fraction of items whose cluster's majority label is theirs."""
    labels = np.asarray(labels).ravel()
    clusters = np.asarray(clusters).ravel()
    if labels.size != clusters.size:
        raise ValueError("purity: label vectors of different lengths")
    overlap = 0
    for k in np.unique(clusters):
        _, cnt = np.unique(labels[clusters == k], return_counts=True)
        overlap += int(cnt.max())
    return overlap / labels.size

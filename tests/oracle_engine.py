"""TEST INFRASTRUCTURE: a CPU stand-in for vbhem_amd.estep.EStepEngine whose
``fused`` step is computed by the oracle (C restatement of the MEX + the
oracle's responsibilities and statistics), packed in the layout of
include/vbhem_estep.h.  Lets the product EM loop (vbhem_amd.em) and its
multi-rank path be tested on the CPU; never used by the product.
"""
from __future__ import annotations

import numpy as np
import torch

import vbhem_oracle as vo


def pack_stats(Nj, N1, M, Lt1, Lt7, Nr, Y, SC, covmode):
    """[Nj | N1 | M | Lt1 | Lt7 | U[K][S][NU]], U = [Nr, Y, triu(SC) | SC]."""
    K, S, d = Y.shape
    if covmode == 1:
        iu = np.triu_indices(d)
        sc = SC[..., iu[0], iu[1]]
    else:
        sc = SC
    U = np.concatenate([Nr[..., None], Y, sc], axis=-1)
    return np.concatenate([Nj.ravel(), N1.ravel(), M.ravel(), [Lt1, Lt7], U.ravel()])


class OracleEngine:
    def __init__(self, base, K, S, T, nthreads=2, trials=1):
        """K clusters in total; trials = R > 1: R consecutive groups of K / R
        (the layout of vbhem_estep_fused_trials)."""
        self.base = base                       # vbhem_amd.BaseSet on the CPU
        self._np = base.numpy()
        self.K, self.S, self.T = K, S, T
        self.nthreads = nthreads
        self.trials = trials
        self.consts = None
        self.logOmega = None
        self.hatZ = torch.zeros((base.N, K), dtype=torch.float64)
        self.LL = torch.zeros((base.N, K), dtype=torch.float64)
        self.calls = 0

    @property
    def N(self):
        return self.base.N

    def set_clusters(self, consts):
        self.consts = {k: np.asarray(v) for k, v in consts.items()}

    def set_log_omega(self, logOmega):
        self.logOmega = np.asarray(logOmega, dtype=np.float64)

    def fused(self, tildeN):
        self.calls += 1
        tN = tildeN.cpu().numpy() if torch.is_tensor(tildeN) else np.asarray(tildeN)
        cov = self.base.covmode
        KT = self.K // self.trials
        vecs, hzs, lls = [], [], []
        for r in range(self.trials):
            sl = slice(r * KT, (r + 1) * KT)
            consts = {k: v[sl] for k, v in self.consts.items()}
            pairs = vo.c_estep_pairs(self._np, consts, self.T, nthreads=self.nthreads)
            hz, Z = vo.c_responsibilities(pairs["LL_elbo"], tN, self.logOmega[sl])
            st = vo.c_statistics(Z, pairs, cov)
            Lt1 = float((Z * pairs["LL_elbo"]).sum())
            Lt7 = float((hz * np.log(hz)).sum())
            hzs.append(hz)
            lls.append(pairs["LL_elbo"])
            vecs.append(pack_stats(st["Nj"], st["N1"], st["M"], Lt1, Lt7, st["Nr"], st["Y"],
                                   st["SC"], cov))
        self.hatZ = torch.from_numpy(np.concatenate(hzs, axis=1))
        self.LL = torch.from_numpy(np.concatenate(lls, axis=1))
        return torch.from_numpy(np.concatenate(vecs))

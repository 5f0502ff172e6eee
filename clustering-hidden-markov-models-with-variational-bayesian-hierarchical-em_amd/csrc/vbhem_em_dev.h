// vbhem_em_dev.h -- the EM loop's per-iteration host math as device kernels
// (vbhem_em_dev.hip), used by vbhem_em_run (vbhem_em.hip).  Internal.
#pragma once
#include <hip/hip_runtime.h>

namespace vbhem {

constexpr int kEmDevMaxD = 16;  // register-resident d x d factorisations (padded to 2/4/8/16)

enum { kEmPrelude = 0, kEmIterate = 1 };

struct EmDevArgs {
  int K, S, d, covmode, NU;
  // posterior read (device; mode kEmPrelude / kEmBound)
  const double *alpha, *eta, *eps, *lam, *v, *m, *W;
  // posterior written by the M-step (kEmMstepPrelude; the prelude then reads it)
  double *alpha_o, *eta_o, *eps_o, *lam_o, *v_o, *m_o, *W_o;
  const double *stats;  // packed E-step statistics (device)
  // hyperparameters and their precomputed constants (host side, once per run)
  double alpha0, eta0, epsilon0, lambda0, v0;
  double logCalpha0, logCeta0, logCepsilon0, logB0;
  const double *m0;     // [d]
  const double *W0inv;  // [d][d]
  // prelude outputs: the E-step's cluster constants, and for the bound
  // logLambdaTilde and log det W of every (k, s)
  double *logA, *logPi, *cm, *P, *c, *lLT, *logOmega, *logdetW;
  double *part;  // [K S][13] bound partial sums
  int *ticket;   // 0 between launches (the last wave of a launch resets it)
  int *flag;     // optional (mapped host memory): set to seq after *L_out is written
  int seq;
};

bool em_dev_supported(int d, int S);
// kEmPrelude: prelude of (alpha .. W); kEmIterate: the bound of (alpha .. W) with
// this iteration's prelude outputs and stats, written to *L_out (device or mapped
// host), then the M-step of (stats) into (alpha_o .. W_o) and its prelude.
hipError_t launch_em_dev(const EmDevArgs &a, int mode, double *L_out, hipStream_t st);

}  // namespace vbhem

/*
 * vbhem_em.h -- the VBHEM-H3M EM host loop in C++ around the device E-step
 * (SURVEY.md 8f, rank 1): vbhem_h3m_c_step_fc.m:1-449 with the psi prelude
 * (:118-165), the fused E-step (vbhem_estep_fused), the lower bound
 * (vbhemh3m_lb.m:64-186), the convergence test (:311-354) and the M-step
 * (vbhem_mstep_component.m:42-70, :396) -- no Python in the loop.
 *
 * All posterior / option arrays are HOST arrays, row-major, as in
 * vbhem_amd/h3m.py::Posterior.  Status codes as in vbhem_estep.h.
 */
#ifndef VBHEM_EM_H
#define VBHEM_EM_H

#include <stddef.h>

#include "vbhem_dist.h"
#include "vbhem_estep.h"

#ifdef __cplusplus
extern "C" {
#endif

/* h3m_r variational posteriors (vbhemhmm_init.m:77-99, vbhem_mstep_component.m:42-69) */
typedef struct {
  int K, S, d, covmode;
  double *alpha;    /* [K]                                   */
  double *eta;      /* [K][S]                                */
  double *epsilon;  /* [K][S][S]                             */
  double *lam;      /* [K][S]                                */
  double *v;        /* [K][S]                                */
  double *m;        /* [K][S][d]                             */
  double *W;        /* [K][S][d][d] (full) | [K][S][d] (diag) */
} vbhem_post_t;

/* hyper-parameters and loop options (vbhem_h3m_cluster.m:150-229, the subset used) */
typedef struct {
  double alpha0, eta0, epsilon0, lambda0, v0;
  const double *m0;  /* [d]                                               */
  const double *W0;  /* [W0_len]: 1 -> W0*eye(d), d -> diag(W0)           */
  int W0_len;
  double Nv;         /* virtual samples (tilde_N = Nv * N * omega)        */
  int max_iter;
  double minDiff;
} vbhem_em_opt_t;

/* psi prelude (step_fc.m:118-165, 180-191, 271-273) into caller arrays:
 * logA [K][S][S], logPi [K][S], m [K][S][d], P [K][S][d][d]|[K][S][d], c [K][S],
 * logLambdaTilde [K][S], logOmega [K]. */
int vbhem_em_prelude(const vbhem_post_t *post, double *logA, double *logPi, double *m, double *P,
                     double *c, double *logLambdaTilde, double *logOmega);

/* vbhemh3m_lb.m:64-186 (value) from the packed E-step statistics (host copy,
 * layout of vbhem_estep_fused) and this iteration's prelude outputs. */
int vbhem_em_lower_bound(const vbhem_post_t *post, const vbhem_em_opt_t *opt,
                         const double *stats, const double *logLambdaTilde, const double *logA,
                         const double *logPi, const double *logOmega, double *L);

/* vbhem_compute_Statistics.m:57-82 + vbhem_mstep_component.m:42-70 + alpha update
 * (step_fc.m:396): the posterior is updated in place. */
int vbhem_em_mstep(const vbhem_em_opt_t *opt, const double *stats, vbhem_post_t *post);

/* The per-iteration host math of vbhem_em_run in one call: the bound of the
 * iteration whose statistics are given (with that iteration's prelude outputs
 * logA, logPi, logLambdaTilde, logOmega), then -- unless the bound is NaN -- the
 * M-step (post updated in place) and the prelude of the next iteration (all seven
 * prelude arrays overwritten).  *L receives the bound. */
int vbhem_em_host_iteration(const vbhem_em_opt_t *opt, const double *stats, vbhem_post_t *post,
                            double *logA, double *logPi, double *m, double *P, double *c,
                            double *logLambdaTilde, double *logOmega, double *L);

/* Optional cross-device reduction of the packed statistics (device pointer, n
 * doubles, the launch stream): called once per iteration between the E-step and
 * the host math.  Return 0 on success. */
typedef int (*vbhem_allreduce_fn)(double *stats_dev, size_t n, void *stream, void *ctx);

/* Device workspace of vbhem_em_run: the fused workspace + the cluster constants. */
size_t vbhem_em_workspace_bytes(const vbhem_base_t *base, int K, int S, int T);

/* The EM loop on this device's base set (device pointers in `base`, tildeN_dev,
 * stats_dev [vbhem_stats_len], hatZ_dev / LL_dev [N][K]).  `post` (host) holds the
 * initial posteriors and receives the final ones; LogLs [max_iter + 1] receives the
 * lower bound of every iteration (before its M-step); *iters, *L_final, *stable as
 * in vbhem_h3m_c_step_fc.m:311-374 (L = -inf and no M-step when the bound is NaN).
 * hatZ_dev / LL_dev receive the last accepted E-step's hat_Z and L_elbo.
 * For d <= 16 and S <= 32 the per-iteration host math (bound, M-step, prelude) runs
 * on the device (vbhem_em_dev.hip) and the loop keeps the next iteration queued
 * while it reads this one's bound (one iteration ahead: a converging run computes
 * one E-step it then discards, so stats_dev holds the statistics of the last E-step
 * RUN); otherwise, or with VBHEM_EM_HOST_MATH set, the host math runs in C++ on the
 * host between synchronous E-steps.  The all-reduce callback always reduces
 * stats_dev, once per E-step run, in the same order on every rank. */
int vbhem_em_run(const vbhem_base_t *base, const double *tildeN_dev, int T,
                 const vbhem_em_opt_t *opt, vbhem_post_t *post, double *LogLs, int *iters,
                 double *L_final, int *stable, double *stats_dev, double *hatZ_dev,
                 double *LL_dev, void *workspace_dev, size_t workspace_bytes, void *stream,
                 vbhem_allreduce_fn allreduce, void *allreduce_ctx);

/* Number of raw bound derivatives (vbhem_em_lower_bound_derivs): alpha0, eta0,
 * epsilon0, v0, lambda0, W0[W0_len], m0[d]. */
#define VBHEM_DLL_LEN(d, W0_len) (5 + (W0_len) + (d))

/* Optional extensions of vbhem_em_run (zero-initialise, set what is used). */
typedef struct {
  /* RCCL communicator (include/vbhem_dist.h): the packed statistics are SUM
   * all-reduced in-stream after every E-step run, in the loop itself (no host
   * callback; the callback must then be NULL). */
  void *rccl_comm;
  /* [max_iter + 1] or NULL: host steady-clock seconds at which each accepted
   * iteration's bound reached the host (the loop's own per-iteration clock). */
  double *iter_seconds;
  /* vbhemh3m_lb.m:202-345 (calc_LLderiv, vbhem_h3m_c_step_fc.m:356-368): raw
   * derivatives of the last accepted iteration's bound, taken before its M-step,
   * into dLL [VBHEM_DLL_LEN(d, W0_len)]; all NaN when the run ends unstable. */
  int calc_deriv;
  double *dLL;
} vbhem_em_ext_t;

int vbhem_em_run_ext(const vbhem_base_t *base, const double *tildeN_dev, int T,
                     const vbhem_em_opt_t *opt, vbhem_post_t *post, double *LogLs, int *iters,
                     double *L_final, int *stable, double *stats_dev, double *hatZ_dev,
                     double *LL_dev, void *workspace_dev, size_t workspace_bytes, void *stream,
                     vbhem_allreduce_fn allreduce, void *allreduce_ctx, const vbhem_em_ext_t *ext);

/* vbhemh3m_lb.m:202-345: the raw derivatives of the bound with respect to the
 * hyperparameters (posterior held fixed; no clipping, no change of variables --
 * vbhem_amd/hyp.py applies :326-356), from the posterior and its prelude outputs. */
int vbhem_em_lower_bound_derivs(const vbhem_post_t *post, const vbhem_em_opt_t *opt,
                                const double *logLambdaTilde, const double *logA,
                                const double *logPi, const double *logOmega, double *dLL);

#ifdef __cplusplus
}
#endif
#endif /* VBHEM_EM_H */

/*
 * include/vbhem_estep.h -- C ABI of the MI355X-native VBHEM-H3M E-step
 * (libvbhem_estep.so, gfx950).
 *
 * Drop-in boundary for the reference's only native call on the EM path:
 *   [LL_elbo, nu_1, emit_pr, emit_mu, emit_Mu, sum_xi] =
 *       vbhem_hmm_bwd_fwd_mex(h3m_b.hmm, h3m_r.hmm, T, maxN, maxN2
 *                             [, logdetCovPlusDdivlamR, invCovR])
 *   called at src/vbhem/vbhem_h3m_c_step_fc.m:175-176 (diag) and :193-194 (full),
 *   implemented by src/vbhem/vbhem_hmm_bwd_fwd_mex.c:288-1472.
 * The MATLAB-facing gateway that binds these entry points lives in
 * integration/vbhem_hmm_bwd_fwd_mex.c.
 *
 * Conventions
 *   - All arrays are dense, row-major (C order), IEEE fp64 unless noted.
 *   - Base HMMs are zero-padded to SB = max states (maxN in the reference);
 *     nstates[i] <= SB holds the true count.  Zero prior/A rows and columns are
 *     exact no-ops in the recursions (mex.c:964-971, 1054-1058, 1196-1206).
 *   - covmode: VBHEM_COV_DIAG (covars/P are [..][d]) or VBHEM_COV_FULL ([..][d][d]).
 *   - Pointers inside vbhem_base_t / vbhem_cluster_t and every *_dev argument
 *     are DEVICE pointers; `stream` is a hipStream_t (NULL = default stream).
 *   - Functions return VBHEM_OK (0) or a negative status; vbhem_last_error()
 *     gives a message.  Nothing synchronises the stream except the *_host
 *     convenience entry point.
 *   - Re-entrant: the library keeps no state shared between host threads (the
 *     error message, the fused schedule and the timing records are per thread;
 *     the launch-attribute caches are per device and locked).  Each concurrent
 *     call needs its own workspace.
 *   - The device-pointer entry points enqueue kernels and memsets only (no
 *     allocation, no host synchronisation, no per-call host state in device
 *     memory), so a call may be captured into a HIP graph and replayed; the
 *     workspace's fallback counters reset themselves on the device.
 *   - A workspace's contents on entry are arbitrary.  Its first 32 bytes carry the
 *     fallback counters and a per-process tag from one fused call to the next: a
 *     call that finds the tag skips zeroing the counters (the short-K1 schedule
 *     zeroes them inside its first kernel otherwise).  Memory reused for anything
 *     else overwrites the leading tag first; a caller that writes into a live
 *     workspace between calls should clear its first 8 bytes.
 */
#ifndef VBHEM_ESTEP_H
#define VBHEM_ESTEP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VBHEM_COV_DIAG 0
#define VBHEM_COV_FULL 1

#define VBHEM_OK 0
#define VBHEM_ERR_ARG (-1)       /* invalid sizes / pointers                    */
#define VBHEM_ERR_UNSUPPORTED (-2) /* shape outside the built kernels' limits   */
#define VBHEM_ERR_WORKSPACE (-3) /* workspace too small                          */
#define VBHEM_ERR_HIP (-4)       /* HIP runtime error (message has details)     */

/* h3m_b: the N base HMMs (reference fields hmm_b.prior/A/emit{k}.centres/covars,
 * read at mex.c:459-473). */
typedef struct {
  int N;                 /* number of base HMMs (Kb)                           */
  int SB;                /* padded states per base HMM (maxN)                  */
  int d;                 /* emission dimension                                 */
  int covmode;           /* VBHEM_COV_DIAG | VBHEM_COV_FULL                    */
  const int *nstates;    /* [N]        true state counts (<= SB)               */
  const double *prior;   /* [N][SB]    hmm_b.prior (may be sub-stochastic)     */
  const double *A;       /* [N][SB][SB] hmm_b.A, A[i][from][to]                */
  const double *centres; /* [N][SB][d] emit{k}.centres                          */
  const double *covars;  /* [N][SB][d][d] | [N][SB][d]   emit{k}.covars         */
  /* Optional: the base set's operand of the emission GEMM, prepared once by
   * vbhem_prepare_base (device memory, cluster independent), or NULL -- then every
   * call builds it for the bases it processes in its workspace.  Ignored by the
   * *_host entry points (they prepare their own). */
  const double *U;
} vbhem_base_t;

/* h3m_r: the K cluster HMMs' variational constants for this EM iteration
 * (mex.c:433-457; built on the MATLAB side at step_fc.m:118-165, 180-191). */
typedef struct {
  int K;                 /* number of clusters (Kr)                            */
  int S;                 /* states per cluster (maxN2; all clusters equal)     */
  const double *logA;    /* [K][S][S]  logATilde[rho][sigma]                   */
  const double *logPi;   /* [K][S]     logPiTilde                              */
  const double *m;       /* [K][S][d]  emit{k}.m                               */
  const double *P;       /* [K][S][d][d] invCovR = v.*W  | [K][S][d] v*W (diag) */
  const double *c;       /* [K][S]     logdetCovPlusDdivlamR = -logLambdaTilde + d/lambda */
} vbhem_cluster_t;

/* The base set's side of the emission GEMM (K1), prepared once per base set:
 * E[(i,b),(j,s)] = bias'(j,s) + sum_e W'(e,(j,s)) U(e,(i,b)) with U built from the
 * base covariances and the base means shifted by z = the mean of the valid base
 * means (a fixed, cluster-independent shift: the quadratic form is shift invariant,
 * the shift keeps its expanded terms small).  vbhem_prepare_base_bytes: the device
 * bytes of U for `base` (0: unsupported descriptor); vbhem_prepare_base fills them
 * (device pointers in `base`, enqueued on `stream`).  Pass the buffer as base->U to
 * the device entry points; it stays valid while the base arrays are unchanged. */
size_t vbhem_prepare_base_bytes(const vbhem_base_t *base);
int vbhem_prepare_base(const vbhem_base_t *base, double *U_dev, size_t bytes, void *stream);

/* src/vbhem/hmms_to_h3m_hem.m:42-140 on the device: N learned VB-HMMs, zero-padded
 * to SB states, into the base-set arrays above.  Inputs (device): nstates [N] (0 =
 * an empty entry, which becomes a one-state dummy HMM with weight 0), the variational
 * counts alpha [N][SB], epsilon [N][SB][SB], beta [N][SB] (use_post = 1: prior =
 * exp(psi(alpha) - psi(sum alpha)), A rows likewise from epsilon, covariances times
 * (beta + 1) / beta) or the point estimates prior_in [N][SB], trans_in [N][SB][SB]
 * (use_post = 0), the means centres_in [N][SB][d] and FULL covariances
 * covars_in [N][SB][d][d] (diag mode keeps their diagonals).  Outputs: prior, A,
 * centres, covars (layout of covmode) and omega [N] = 1 / (number of non-empty
 * entries) or 0.  workspace: 4 bytes of device memory.  Replaces the MATLAB host loop
 * the reference runs once per vbhem_h3m_cluster call (vbhem_h3m_cluster.m:237). */
int vbhem_hmms_to_h3m(int N, int SB, int d, int covmode, int use_post, const int *nstates,
                      const double *alpha, const double *epsilon, const double *beta,
                      const double *prior_in, const double *trans_in, const double *centres_in,
                      const double *covars_in, double *prior, double *A, double *centres,
                      double *covars, double *omega, void *workspace, void *stream);

/* Per-pair outputs of the reference MEX (mex.c:396-409), laid out [N][K][...]:
 *   LL_elbo [N][K]; sum_nu_1 [N][K][S]; emit_pr [N][K][S]; emit_mu [N][K][S][d];
 *   emit_Mu [N][K][S][d][d] (full) | [N][K][S][d] (diag); sum_xi [N][K][S][S].
 * sum_t_nu [N][K][S][SB] (the forward occupancy sum, mex.c:1148-1297) is an
 * optional extra output (NULL to skip). */
size_t vbhem_pairs_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T);
int vbhem_estep_pairs(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      double *LL_elbo_dev, double *sum_nu_1_dev, double *emit_pr_dev,
                      double *emit_mu_dev, double *emit_Mu_dev, double *sum_xi_dev,
                      double *sum_t_nu_dev, void *workspace_dev, size_t workspace_bytes,
                      void *stream);

/* Same as vbhem_estep_pairs, with HOST arrays in and out (allocates, copies,
 * computes on `device`, copies back, frees).  This is what the MEX gateway
 * calls; base/clus pointers are host pointers here. */
int vbhem_estep_pairs_host(int device, const vbhem_base_t *base_host,
                           const vbhem_cluster_t *clus_host, int T, double *LL_elbo,
                           double *sum_nu_1, double *emit_pr, double *emit_mu,
                           double *emit_Mu, double *sum_xi);

/* VHEM sibling: replaces src/compare_mtds/hem/vhem_h3m/hem_hmm_bwd_fwd_mex.c
 * (called at hem_h3m_c_step.m:191-192 / :208-209).  The same recursions on
 * point-estimate reduced HMMs, with the expected emission log-likelihood
 * divided by `smooth` (hem_hmm_bwd_fwd_mex.c:848-860; smooth > 0).  The cluster
 * descriptor then carries (hem_hmm_bwd_fwd_mex.c:565-600, 906-922, 1004-1019):
 *   logA  = log(hmm_r.A)            logPi = log(hmm_r.prior)
 *   m     = emit{k}.centres
 *   P     = inv(emit{k}.covars) = invCovR      | 1 ./ covars (diag)
 *   c     = log(det(emit{k}.covars)) = logdetCovR | sum(log(covars)) (diag)
 * Workspace: vbhem_pairs_workspace_bytes.  Outputs as vbhem_estep_pairs. */
int vhem_estep_pairs(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T, double smooth,
                     double *LL_elbo_dev, double *sum_nu_1_dev, double *emit_pr_dev,
                     double *emit_mu_dev, double *emit_Mu_dev, double *sum_xi_dev,
                     double *sum_t_nu_dev, void *workspace_dev, size_t workspace_bytes,
                     void *stream);
int vhem_estep_pairs_host(int device, const vbhem_base_t *base_host,
                          const vbhem_cluster_t *clus_host, int T, double smooth,
                          double *LL_elbo, double *sum_nu_1, double *emit_pr, double *emit_mu,
                          double *emit_Mu, double *sum_xi);

/* Fused E-step for one EM iteration on this device's shard of base HMMs:
 *   pairs (mex.c) -> responsibilities (step_fc.m:271-283) -> gated, Z-weighted
 *   statistic sums (vbhem_compute_Statistics.m:33-55) -> ELBO partials
 *   (vbhemh3m_lb.m:90,107).
 * Inputs: tildeN_dev [N] = Nv*Kb*omega (step_fc.m:26-30) for this shard,
 *         logOmega_dev [K] = psi(alpha) - psi(sum alpha) (step_fc.m:271-273).
 * Outputs: hatZ_dev [N][K] (hat_Z incl. +1e-50), LL_elbo_dev [N][K],
 *          stats_dev [vbhem_stats_len(...)] laid out as
 *   [ Nj[K] | N1[K][S] | M[K][S][S] | Lt1 | Lt7 | U[K][S][NU] ]
 *   where Nj = sum_i Z (no gate, no +1e-50), N1 = sum_i g Z nu_1, M = sum_i g Z sum_xi,
 *   Lt1 = sum Z.*L_elbo, Lt7 = sum hat_Z.*log(hat_Z), g = [Z > 1e-8], and
 *   U[j][s][:] = sum_i g Z(i,j) sum_b sum_t_nu(i,j,s,b) * u(i,b,:) with
 *   u = [1, mu (d), Sigma+mu mu' packed upper-triangular (d(d+1)/2)] (full) or
 *   u = [1, mu (d), mu.^2 + sigma (d)] (diag); NU = vbhem_stats_nu(d, covmode).
 * All terms are plain sums over this shard's bases: shards combine by summation
 * (one all-reduce).  Results are deterministic for a fixed shard. */
size_t vbhem_stats_nu(int d, int covmode);
size_t vbhem_stats_len(int K, int S, int d, int covmode);
size_t vbhem_fused_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T);
int vbhem_estep_fused(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      const double *tildeN_dev, const double *logOmega_dev,
                      double *stats_dev, double *hatZ_dev, double *LL_elbo_dev,
                      void *workspace_dev, size_t workspace_bytes, void *stream);

/* R independent EM trials (vbhem_h3m_c.m:28-67, `parfor it = 1:numits`, each from its
 * own initialisation) batched as one launch over the same base set: `clus` holds
 * R * KT clusters, trial-major (trial r = clusters [r KT, (r+1) KT)).  hat_Z is
 * normalised within each trial; stats_dev holds R consecutive vectors of
 * vbhem_stats_len(KT, S, d, covmode), each laid out as above for its trial;
 * logOmega_dev [R*KT] is each trial's psi(alpha) - psi(sum alpha); hatZ_dev /
 * LL_elbo_dev are [N][R*KT].  R = 1 is vbhem_estep_fused.  Needs the gated schedule
 * (S <= 16, Sb <= S) and R * KT <= 256; else VBHEM_ERR_UNSUPPORTED. */
size_t vbhem_fused_trials_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus,
                                          int R, int T);
int vbhem_estep_fused_trials(const vbhem_base_t *base, const vbhem_cluster_t *clus, int R, int T,
                             const double *tildeN_dev, const double *logOmega_dev,
                             double *stats_dev, double *hatZ_dev, double *LL_elbo_dev,
                             void *workspace_dev, size_t workspace_bytes, void *stream);

/* Host-array entry points of the fused E-step (what a MATLAB gateway binds; see
 * integration/vbhem_estep_fused_mex.c and INTEGRATION.md).
 *
 * A context keeps one base set resident on `device` (uploaded once) together
 * with the workspace and output buffers for K clusters of S states (R batched
 * trials, K a multiple of R); each vbhem_ctx_fused call uploads only the
 * cluster constants (tens of KB), runs vbhem_estep_fused_trials and copies
 * back the packed statistics (and, when the pointers are non-NULL, hat_Z and
 * L_elbo as [N][K]).  Host arrays in/out, synchronous.  A context is used by
 * one host thread at a time.
 *   clus_host: K, S must match the context; tildeN_host [N]; logOmega_host [K];
 *   stats_host [R * vbhem_stats_len(K/R, S, d, covmode)].
 * vbhem_estep_fused_host is the one-shot form (create, one call, destroy). */
typedef struct vbhem_ctx vbhem_ctx_t;
int vbhem_ctx_create(int device, const vbhem_base_t *base_host, int K, int S, int R, int T,
                     vbhem_ctx_t **ctx_out);
int vbhem_ctx_fused(vbhem_ctx_t *ctx, const vbhem_cluster_t *clus_host, const double *tildeN_host,
                    const double *logOmega_host, double *stats_host, double *hatZ_host,
                    double *LL_elbo_host);
void vbhem_ctx_destroy(vbhem_ctx_t *ctx);
int vbhem_estep_fused_host(int device, const vbhem_base_t *base_host,
                           const vbhem_cluster_t *clus_host, int T, const double *tildeN_host,
                           const double *logOmega_host, double *stats_host, double *hatZ_host,
                           double *LL_elbo_host);

/* Fused E-step schedule of the calling host thread (default VBHEM_FUSED_GATED,
 * or VBHEM_FUSED_DENSE=1 in the environment).  Both give the same outputs:
 *   VBHEM_FUSED_GATED  backward sweep + log-likelihood for every pair, then the
 *                      forward sweep and statistics only for the pairs the gate
 *                      Z > 1e-8 of vbhem_compute_Statistics.m:35 keeps (the
 *                      reference computes the others and discards them);
 *   VBHEM_FUSED_DENSE  both sweeps for every pair (mex.c order of work).
 * Returns the previous mode. */
#define VBHEM_FUSED_GATED 0
#define VBHEM_FUSED_DENSE 1
int vbhem_set_fused_mode(int mode);

/* Number of pairs the last call on this thread had to recompute with the
 * exact (reference-order, Theta-storing) fallback because the factorised
 * log-sum-exp fell below its safe range.  Synchronises `stream`. */
int vbhem_last_fallback_count(void *stream, const void *workspace_dev);

/* Device address of pinned (page-locked, mapped) host memory, for callers that
 * let vbhem_estep_fused write its statistics straight into host memory (the
 * host M-step's input: no device-to-host copy after the E-step; the kernel's
 * stores cross the bus).  The host reads the vector after synchronising the
 * stream.  VBHEM_ERR_ARG if host_ptr is not registered pinned memory. */
int vbhem_host_device_pointer(void *host_ptr, void **dev_ptr);

/* Completion word for the NEXT vbhem_estep_fused call of this process (one-shot; no
 * reference counterpart -- the MEX returns synchronously): once that call's
 * statistics are written and visible to the host, its last kernel stores `value`
 * into the 64-bit word at `word` (a device address, e.g. vbhem_host_device_pointer of
 * a pinned host word), after the statistics, at system scope.  A host that runs
 * E-steps ahead of itself can poll the word instead of recording an event after each
 * call (an event is a queue marker: ~5.7 us of idle GPU per E-step on MI355X).
 * word = NULL disarms.  The statistics must themselves be host memory or be read
 * after a stream synchronisation. */
int vbhem_arm_done_word(void *word, unsigned long long value);
/* A zeroed 64-bit completion word in coherent (fine-grained) pinned host memory:
 * *host_ptr for the host's reads, *dev_ptr for vbhem_arm_done_word.  Free with
 * vbhem_done_word_free(host_ptr). */
int vbhem_done_word_alloc(void **host_ptr, void **dev_ptr);
int vbhem_done_word_free(void *host_ptr);

/* Kernel timing for benchmarking/profiling, per host thread: while enabled,
 * hipEvents are recorded on the launch stream around the kernel launches of this
 * thread (never into a stream that is capturing a graph: such launches are simply
 * not timed).  on = 1: every fb / emission / stats / gated-forward launch; on = 2:
 * the fb (backward or dense) launches only -- two events per E-step, for timing
 * the dominant kernel inside a timed region at negligible cost; 0: off.
 * vbhem_timing_read synchronises on them, returns the summed elapsed
 * milliseconds, the launch counts and the number of (i,j) pairs the fb launches
 * covered, and resets. */
int vbhem_timing_enable(int on);
int vbhem_timing_read(double *fb_ms, long long *fb_launches, long long *fb_pairs,
                      double *stats_ms, long long *stats_launches);
/* Summed time and launch count of the K1 emission GEMM (emission_kernel) since
 * the last call; same event mechanism as vbhem_timing_read. */
int vbhem_timing_read_emission(double *em_ms, long long *em_launches);
/* Summed time and launch count of the gated forward pass (fb_split_kernel in
 * list mode; VBHEM_FUSED_GATED only) since the last call. */
int vbhem_timing_read_gated(double *fwd_ms, long long *fwd_launches);
/* Summed time and launch count of the EM loop's per-iteration math kernel
 * (vbhem_em_run's bound + M-step + next prelude on the device, em_dev_kernel) since
 * the last call; recorded while vbhem_timing_enable(1) is on. */
int vbhem_timing_read_em_math(double *ms, long long *launches);

/* Test hook (fault injection, no reference counterpart): add `bytes` of dynamic LDS
 * to the next fb_bwd2_kernel launches of this process, so the runtime refuses them
 * (tests/test_robustness.py: a refused launch must not leave a HIP error pending).
 * 0 turns it off; returns the previous value.  Never set in production: unlike an
 * environment variable, nothing outside the calling program can switch it on. */
size_t vbhem_debug_extra_lds(size_t bytes);

const char *vbhem_last_error(void);
const char *vbhem_version(void);
/* The kernel the calling thread's last E-step ran for a recursion pass, as the
 * kernel trace names it: pass 0 the every-pair pass (backward-only in the gated
 * schedule, K2-K4 in the dense one), pass 1 the gated schedule's gate-list pass;
 * "" before any such launch.  Benchmark labelling only (no reference
 * counterpart). */
const char *vbhem_last_kernel(int pass);

#ifdef __cplusplus
}
#endif
#endif /* VBHEM_ESTEP_H */

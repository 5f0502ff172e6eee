/*
 * oracle/vbhem_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64, libm exp/log) of the reference VBHEM-H3M
 * E-step as implemented by the reference MEX
 *     /root/reference/src/vbhem/vbhem_hmm_bwd_fwd_mex.c   (USEPTRS branch)
 * plus the responsibilities and the statistics reduction of
 *     src/vbhem/vbhem_h3m_c_step_fc.m:270-283
 *     src/vbhem/vbhem_compute_Statistics.m:33-55
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / reported CPU baseline.  The
 * product path (the HIP library) never links or calls it.
 *
 * PARITY UNPINNED: the reference ships no golden vectors or tests, MATLAB is
 * not available, and the reference MEX needs mex.h/libmx (absent from the
 * image), so it is not built here.  This restatement is cross-checked against
 * an independent numpy restatement of the MATLAB twin
 * (src/vbhem/vbhem_hmm_bwd_fwd_fast.m, see oracle/vbhem_oracle.py) and against
 * closed-form known answers (tests/test_oracle.py).
 *
 * Loop orders follow the MEX so that floating-point summation order matches:
 *   pairs: for j (cluster) { for i (base) }               mex.c:505,520
 *   K1 emission E[beta,sigma]                             mex.c:716-864
 *   K2 backward  t=T-1..1, rho, logtrick over sigma       mex.c:915-1015, 211-269
 *   K3 termination                                        mex.c:1020-1080
 *   K4 forward   t=1..T-1, sigma                          mex.c:1093-1298
 *   K5 emission statistics                                mex.c:1348-1469
 *
 * Data layout (row-major C, zero-padded base states to SB):
 *   nstates[N], prior[N][SB], A[N][SB][SB] (A[i][from][to]),
 *   centres[N][SB][d], covars[N][SB][d][d] (full) or [N][SB][d] (diag);
 *   logA[K][S][S] (logATilde[rho][sigma]), logPi[K][S], m[K][S][d],
 *   P[K][S][d][d] (= v*W, full) or [K][S][d] (= v*W_diag, diag),
 *   c[K][S] (= logLambdaTildePlusDdivlamda = -logLambdaTilde + d/lambda).
 * Per-pair outputs are laid out [N][K][...].
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define ORACLE_COV_DIAG 0
#define ORACLE_COV_FULL 1

typedef struct {
  int N, SB, d, covmode;
  const int *nstates;
  const double *prior, *A, *centres, *covars;
} oracle_base;

typedef struct {
  int K, S;
  const double *logA, *logPi, *m, *P, *c;
  double smooth;           /* E /= smooth when != 1 (VHEM, hem mex.c:848-860)        */
  const double *vcov;      /* VHEM diag: [K][S][d] covars of the reduced HMMs, or NULL */
} oracle_cluster;

/* column log-sum-exp: max first, then sum of exp(x - max) in index order
 * (restates logtrick, mex.c:211-269 / logtrick.m:15-18).  x has n entries
 * spaced by `stride`. */
static double lse_strided(const double *x, int n, int stride) {
  double mv = x[0];
  for (int k = 1; k < n; k++)
    if (x[k * stride] > mv) mv = x[k * stride];
  double acc = 0.0;
  for (int k = 0; k < n; k++) acc += exp(x[k * stride] - mv);
  return mv + log(acc);
}

/* Expected Gaussian log-likelihood E_{beta}[log N(y | m_sigma, (v W)^-1)]
 * in the MEX's accumulation order (full: mex.c:796-843; diag: :744-759). */
static double emission_term(const oracle_base *b, const oracle_cluster *r,
                            int i, int beta, int j, int sigma) {
  const int d = b->d;
  const double *mu = b->centres + ((size_t)i * b->SB + beta) * d;
  const double *mm = r->m + ((size_t)j * r->S + sigma) * d;
  if (r->vcov) {
    /* VHEM diag (hem_hmm_bwd_fwd_mex.c:711-733): log, trace and Mahalanobis terms by
     * division, per dimension */
    const double *sr = r->vcov + ((size_t)j * r->S + sigma) * d;
    const double *C = b->covars + ((size_t)i * b->SB + beta) * d;
    double ell = d * log(2.0 * M_PI);
    for (int a = 0; a < d; a++) {
      ell += log(sr[a]);
      ell += C[a] / sr[a];
      double x = mu[a] - mm[a];
      ell += x * x / sr[a];
    }
    ell *= -0.5;
    return r->smooth != 1.0 ? ell / r->smooth : ell;
  }
  double ell = d * log(2.0 * M_PI) + r->c[(size_t)j * r->S + sigma];
  if (b->covmode == ORACLE_COV_FULL) {
    const double *P = r->P + ((size_t)j * r->S + sigma) * d * d;
    const double *C = b->covars + ((size_t)i * b->SB + beta) * d * d;
    /* trace <P, Sigma_beta>: one pass over the d*d entries */
    for (int k = 0; k < d * d; k++) ell += P[k] * C[k];
    /* Mahalanobis term: for each column a, (x' P[:,a]) * x[a] */
    for (int a = 0; a < d; a++) {
      double col = 0.0;
      for (int q = 0; q < d; q++) col += (mu[q] - mm[q]) * P[q * d + a];
      ell += col * (mu[a] - mm[a]);
    }
  } else {
    const double *P = r->P + ((size_t)j * r->S + sigma) * d;
    const double *C = b->covars + ((size_t)i * b->SB + beta) * d;
    for (int a = 0; a < d; a++) {
      double x = mu[a] - mm[a];
      ell += P[a] * C[a];
      ell += P[a] * (x * x);
    }
  }
  return r->smooth != 1.0 ? (-0.5 * ell) / r->smooth : -0.5 * ell;
}

/* One (base i, cluster j) pair.  Scratch `w` must hold
 * 5*S*Sb + S*S*Sb*T doubles. */
static void pair_estep(const oracle_base *b, const oracle_cluster *r, int T,
                       int i, int j, double *w, double *LL_out,
                       double *nu1_out, double *xi_out, double *pr_out,
                       double *mu_out, double *Mu_out, double *tnu_out) {
  const int Sb = b->nstates[i], S = r->S, d = b->d, SB = b->SB;
  const double *Ab = b->A + (size_t)i * SB * SB;   /* Ab[from*SB + to] */
  const double *pib = b->prior + (size_t)i * SB;
  const double *lA = r->logA + (size_t)j * S * S;  /* lA[rho*S + sigma] */
  const double *lPi = r->logPi + (size_t)j * S;

  /* matrices indexed [sigma][beta] */
  double *E = w;                 /* S*Sb */
  double *L = E + S * Sb;        /* S*Sb : LL_old (gamma -> index beta) */
  double *Ln = L + S * Sb;       /* S*Sb : LL_new */
  double *lt = Ln + S * Sb;      /* S*Sb : logtheta[sigma][beta] */
  double *nu = lt + S * Sb;      /* S*Sb */
  double *Th = nu + S * Sb;      /* Theta[t][rho][sigma][beta] */

  /* K1 */
  for (int s = 0; s < S; s++)
    for (int be = 0; be < Sb; be++) E[s * Sb + be] = emission_term(b, r, i, be, j, s);

  /* K2: backward recursion */
  for (int k = 0; k < S * Sb; k++) L[k] = 0.0;
  for (int t = T - 1; t >= 1; t--) {
    for (int rho = 0; rho < S; rho++) {
      for (int s = 0; s < S; s++)
        for (int be = 0; be < Sb; be++)
          lt[s * Sb + be] = lA[rho * S + s] + E[s * Sb + be] + L[s * Sb + be];
      for (int be = 0; be < Sb; be++) {
        double ls = lse_strided(lt + be, S, Sb);
        /* keep the column's log-sum in Ln's row rho for a moment */
        nu[be] = ls;
        double *th = Th + (((size_t)t * S + rho) * S) * Sb;
        for (int s = 0; s < S; s++) th[s * Sb + be] = exp(lt[s * Sb + be] - ls);
      }
      /* LL_new(gamma, rho) = sum_beta Ab(gamma,beta) * logsum(beta) */
      for (int g = 0; g < Sb; g++) {
        double acc = 0.0;
        for (int be = 0; be < Sb; be++) acc += Ab[g * SB + be] * nu[be];
        Ln[rho * Sb + g] = acc;
      }
    }
    memcpy(L, Ln, sizeof(double) * S * Sb);
  }

  /* K3: termination */
  for (int s = 0; s < S; s++)
    for (int be = 0; be < Sb; be++) lt[s * Sb + be] = lPi[s] + E[s * Sb + be] + L[s * Sb + be];
  double LL = 0.0;
  for (int be = 0; be < Sb; be++) {
    double ls = lse_strided(lt + be, S, Sb);
    LL += pib[be] * ls;
    for (int s = 0; s < S; s++) lt[s * Sb + be] = exp(lt[s * Sb + be] - ls); /* Theta_1 */
  }
  *LL_out = LL;

  /* K4: forward recursion */
  double *tnu = Ln;  /* sum_t nu, [sigma][beta] */
  for (int s = 0; s < S; s++)
    for (int be = 0; be < Sb; be++) nu[s * Sb + be] = pib[be] * lt[s * Sb + be];
  for (int s = 0; s < S; s++) {
    double acc = 0.0;
    for (int be = 0; be < Sb; be++) acc += nu[s * Sb + be];
    nu1_out[s] = acc;
  }
  memcpy(tnu, nu, sizeof(double) * S * Sb);
  for (int k = 0; k < S * S; k++) xi_out[k] = 0.0;
  double *foo = E;  /* E no longer needed */
  for (int t = 1; t < T; t++) {
    for (int g = 0; g < Sb; g++)
      for (int rho = 0; rho < S; rho++) {
        double acc = 0.0;
        for (int be = 0; be < Sb; be++) acc += nu[rho * Sb + be] * Ab[be * SB + g];
        foo[rho * Sb + g] = acc;
      }
    for (int s = 0; s < S; s++) {
      /* xi_foo(rho,gamma) = foo(rho,gamma) * Theta(rho,s,gamma,t) */
      const double *th = Th + ((size_t)t * S) * S * Sb;
      for (int rho = 0; rho < S; rho++) {
        double acc = 0.0;
        for (int g = 0; g < Sb; g++)
          acc += foo[rho * Sb + g] * th[(rho * S + s) * Sb + g];
        xi_out[rho * S + s] += acc;
      }
      for (int g = 0; g < Sb; g++) {
        double acc = 0.0;
        for (int rho = 0; rho < S; rho++)
          acc += foo[rho * Sb + g] * th[(rho * S + s) * Sb + g];
        nu[s * Sb + g] = acc;
      }
    }
    for (int k = 0; k < S * Sb; k++) tnu[k] += nu[k];
  }
  if (tnu_out) {
    for (int s = 0; s < S; s++)
      for (int be = 0; be < SB; be++) tnu_out[s * SB + be] = be < Sb ? tnu[s * Sb + be] : 0.0;
  }

  /* K5: emission statistics (sum_w_pr = 1, sum_w_mu = mu, sum_w_Mu = mu mu' + Sigma) */
  const double *mu = b->centres + (size_t)i * SB * d;
  for (int s = 0; s < S; s++) {
    double acc = 0.0;
    for (int be = 0; be < Sb; be++) acc += tnu[s * Sb + be] * 1.0;
    pr_out[s] = acc;
    for (int a = 0; a < d; a++) {
      acc = 0.0;
      for (int be = 0; be < Sb; be++) acc += tnu[s * Sb + be] * mu[be * d + a];
      mu_out[s * d + a] = acc;
    }
    if (b->covmode == ORACLE_COV_FULL) {
      const double *C = b->covars + (size_t)i * SB * d * d;
      for (int q = 0; q < d; q++)
        for (int a = 0; a < d; a++) {
          acc = 0.0;
          for (int be = 0; be < Sb; be++)
            acc += tnu[s * Sb + be] *
                   (mu[be * d + q] * mu[be * d + a] + C[(be * d + q) * d + a]);
          Mu_out[(s * d + a) * d + q] = acc;
        }
    } else {
      const double *C = b->covars + (size_t)i * SB * d;
      for (int a = 0; a < d; a++) {
        acc = 0.0;
        for (int be = 0; be < Sb; be++)
          acc += tnu[s * Sb + be] * (mu[be * d + a] * mu[be * d + a] + C[be * d + a]);
        Mu_out[s * d + a] = acc;
      }
    }
  }
}

static int run_pairs(const oracle_base *bp, const oracle_cluster *rp, int T, double *LL_elbo,
                     double *sum_nu_1, double *sum_xi, double *emit_pr, double *emit_mu,
                     double *emit_Mu, double *sum_t_nu, int nthreads);

/* All pairs; outputs [N][K][...].  tnu_out (sum_t nu, [N][K][S][SB]) may be NULL.
 * nthreads > 1 parallelises over pairs (the reference MEX is single-threaded). */
int oracle_estep_pairs(int N, int SB, int d, int covmode, const int *nstates,
                       const double *prior, const double *A, const double *centres,
                       const double *covars, int K, int S, const double *logA,
                       const double *logPi, const double *m, const double *P,
                       const double *c, int T, double *LL_elbo, double *sum_nu_1,
                       double *sum_xi, double *emit_pr, double *emit_mu,
                       double *emit_Mu, double *sum_t_nu, int nthreads) {
  if (N < 0 || K < 0 || S < 1 || SB < 1 || d < 1 || T < 1) return -1;
  for (int i = 0; i < N; i++)
    if (nstates[i] < 1 || nstates[i] > SB) return -2;
  oracle_base b = {N, SB, d, covmode, nstates, prior, A, centres, covars};
  oracle_cluster r = {K, S, logA, logPi, m, P, c, 1.0, NULL};
  return run_pairs(&b, &r, T, LL_elbo, sum_nu_1, sum_xi, emit_pr, emit_mu, emit_Mu, sum_t_nu,
                   nthreads);
}

/* VHEM sibling (src/compare_mtds/hem/vhem_h3m/hem_hmm_bwd_fwd_mex.c): point-estimate
 * reduced HMMs Ar [K][S][S], priorr [K][S], centresr [K][S][d], covarsr [K][S][d|d*d];
 * full covariances read logdetCov [K][S] and invCov [K][S][d][d] (hem_h3m_c_step.m:
 * 198-205); log(Ar), log(priorr) as at hem mex.c:906-922, 1004-1019; E /= smooth. */
int oracle_vhem_estep_pairs(int N, int SB, int d, int covmode, const int *nstates,
                            const double *prior, const double *A, const double *centres,
                            const double *covars, int K, int S, const double *Ar,
                            const double *priorr, const double *centresr, const double *covarsr,
                            const double *logdetCov, const double *invCov, int T, double smooth,
                            double *LL_elbo, double *sum_nu_1, double *sum_xi, double *emit_pr,
                            double *emit_mu, double *emit_Mu, double *sum_t_nu, int nthreads) {
  if (N < 0 || K < 0 || S < 1 || SB < 1 || d < 1 || T < 1 || !(smooth > 0.0)) return -1;
  for (int i = 0; i < N; i++)
    if (nstates[i] < 1 || nstates[i] > SB) return -2;
  double *lA = (double *)malloc(sizeof(double) * ((size_t)K * S * S + 1));
  double *lP = (double *)malloc(sizeof(double) * ((size_t)K * S + 1));
  if (!lA || !lP) {
    free(lA);
    free(lP);
    return -3;
  }
  for (size_t k = 0; k < (size_t)K * S * S; k++) lA[k] = log(Ar[k]);
  for (size_t k = 0; k < (size_t)K * S; k++) lP[k] = log(priorr[k]);
  oracle_base b = {N, SB, d, covmode, nstates, prior, A, centres, covars};
  oracle_cluster r = {K, S, lA, lP, centresr, invCov, logdetCov, smooth,
                      covmode == ORACLE_COV_FULL ? NULL : covarsr};
  const int rc = run_pairs(&b, &r, T, LL_elbo, sum_nu_1, sum_xi, emit_pr, emit_mu, emit_Mu,
                           sum_t_nu, nthreads);
  free(lA);
  free(lP);
  return rc;
}

static int run_pairs(const oracle_base *bp, const oracle_cluster *rp, int T, double *LL_elbo,
                     double *sum_nu_1, double *sum_xi, double *emit_pr, double *emit_mu,
                     double *emit_Mu, double *sum_t_nu, int nthreads) {
  const oracle_base b = *bp;
  const oracle_cluster r = *rp;
  const int N = b.N, K = r.K, S = r.S, SB = b.SB, d = b.d, covmode = b.covmode;
  const size_t scratch = (size_t)5 * S * SB + (size_t)S * S * SB * T;
  const size_t dMu = covmode == ORACLE_COV_FULL ? (size_t)d * d : (size_t)d;
  int err = 0;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
  {
    double *w = (double *)malloc(sizeof(double) * scratch);
    if (!w) {
      err = -3;
    } else {
      long long npairs = (long long)N * K;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
      for (long long q = 0; q < npairs; q++) {
        /* MEX order: j outer, i inner (mex.c:505,520) */
        int j = (int)(q / (N > 0 ? N : 1)), i = (int)(q % (N > 0 ? N : 1));
        size_t p = (size_t)i * K + j;
        pair_estep(&b, &r, T, i, j, w, LL_elbo + p, sum_nu_1 + p * S, sum_xi + p * S * S,
                   emit_pr + p * S, emit_mu + p * S * d, emit_Mu + p * S * dMu,
                   sum_t_nu ? sum_t_nu + p * S * SB : NULL);
      }
      free(w);
    }
  }
  (void)nthreads;
  return err;
}

/* Responsibilities (vbhem_h3m_c_step_fc.m:275-283):
 *   log_Z(i,j) = tildeN(i) * (logOmega(j) + L_elbo(i,j))
 *   hat_Z = exp(log_Z - logtrick over j) + 1e-50;  Z = hat_Z * tildeN(i)       */
void oracle_responsibilities(int N, int K, const double *LL_elbo, const double *tildeN,
                             const double *logOmega, double *hatZ, double *Z) {
  double *lz = (double *)malloc(sizeof(double) * (K > 0 ? K : 1));
  for (int i = 0; i < N; i++) {
    for (int j = 0; j < K; j++) lz[j] = tildeN[i] * (logOmega[j] + LL_elbo[(size_t)i * K + j]);
    double ls = lse_strided(lz, K, 1);
    for (int j = 0; j < K; j++) {
      double h = exp(lz[j] - ls) + 1e-50;
      hatZ[(size_t)i * K + j] = h;
      Z[(size_t)i * K + j] = h * tildeN[i];
    }
  }
  free(lz);
}

/* Un-normalised, gated statistic sums for every cluster j
 * (vbhem_compute_Statistics.m:33-55, loop over i in order, gate Z > 1e-8):
 *   Nj[j]        = sum_i Z(i,j)                         (step_fc:282, before +1e-50)
 *   N1[j][S]     = sum_i Z * sum_nu_1
 *   M[j][S][S]   = sum_i Z * sum_xi
 *   Nr[j][S]     = sum_i Z * emit_pr
 *   Y[j][S][d]   = sum_i Z * emit_mu
 *   SC[j][S][dM] = sum_i Z * emit_Mu
 * Nj is NOT gated (it is a plain column sum of Z). */
void oracle_statistics(int N, int K, int S, int d, int covmode, const double *Z,
                       const double *sum_nu_1, const double *sum_xi,
                       const double *emit_pr, const double *emit_mu,
                       const double *emit_Mu, double *Nj, double *N1, double *M,
                       double *Nr, double *Y, double *SC) {
  const size_t dMu = covmode == ORACLE_COV_FULL ? (size_t)d * d : (size_t)d;
  for (int j = 0; j < K; j++) {
    double nj = 0.0;
    double *n1 = N1 + (size_t)j * S, *mm = M + (size_t)j * S * S, *nr = Nr + (size_t)j * S;
    double *y = Y + (size_t)j * S * d, *sc = SC + (size_t)j * S * dMu;
    memset(n1, 0, sizeof(double) * S);
    memset(mm, 0, sizeof(double) * S * S);
    memset(nr, 0, sizeof(double) * S);
    memset(y, 0, sizeof(double) * S * d);
    memset(sc, 0, sizeof(double) * S * dMu);
    for (int i = 0; i < N; i++) {
      size_t p = (size_t)i * K + j;
      double z = Z[p];
      nj += z;
      if (!(z > 1e-8)) continue;
      for (int s = 0; s < S; s++) n1[s] += z * sum_nu_1[p * S + s];
      for (int k = 0; k < S * S; k++) mm[k] += z * sum_xi[p * S * S + k];
      for (int s = 0; s < S; s++) nr[s] += z * emit_pr[p * S + s];
      for (size_t k = 0; k < (size_t)S * d; k++) y[k] += z * emit_mu[p * S * d + k];
      for (size_t k = 0; k < (size_t)S * dMu; k++) sc[k] += z * emit_Mu[p * S * dMu + k];
    }
    Nj[j] = nj;
  }
}

/*
 * integration/h3m_mex_common.h -- shared by the two MEX gateways
 * (vbhem_hmm_bwd_fwd_mex.c, hem_hmm_bwd_fwd_mex.c): scalar/field parsing, the
 * host buffers, the base-HMM repack (column-major cells -> row-major, padded to
 * maxN states), the cluster repack (clusters of different sizes: mex.c:436-437,
 * 506) and the per-pair outputs scattered into MATLAB cells.  The two reference
 * gateways share this code too (mex.c:288-409, 459-473, 1108-1122, 1312-1345 /
 * hem_hmm_bwd_fwd_mex.c:288-409).
 */
#ifndef H3M_MEX_COMMON_H
#define H3M_MEX_COMMON_H
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "vbhem_estep.h"

/* the reference's scalar parser (mex.c:77-86): must be a 1x1 double */
static inline double parse_scalar(const mxArray *mx) {
  if (!mx || !mxIsDouble(mx) || mxGetNumberOfElements(mx) != 1)
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "arg must be scalar.");
  return mxGetScalar(mx);
}

static inline const double *field_pr(const mxArray *s, const char *name, size_t numel_expected,
                              const char *what) {
  const mxArray *f = mxGetField(s, 0, name);
  if (!f || !mxIsDouble(f))
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "%s: field '%s' missing or not double", what,
                      name);
  if (numel_expected && mxGetNumberOfElements(f) != numel_expected)
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "%s: field '%s' has %d elements, expected %d",
                      what, name, (int)mxGetNumberOfElements(f), (int)numel_expected);
  return mxGetPr(f);
}

typedef struct {
  int SB;                                  /* base stride (maxN)             */
  int *N2;                                 /* [Kr] cluster state counts       */
  int *nstates;
  double *prior, *A, *centres, *covars;
  double *logA, *logPi, *m, *P, *c;
  double *LL, *nu1, *pr, *mu, *Mu, *xi;
} buffers_t;

static inline void free_buffers(buffers_t *b) {
  mxFree(b->N2);
  mxFree(b->nstates);
  mxFree(b->prior);
  mxFree(b->A);
  mxFree(b->centres);
  mxFree(b->covars);
  mxFree(b->logA);
  mxFree(b->logPi);
  mxFree(b->m);
  mxFree(b->P);
  mxFree(b->c);
  mxFree(b->LL);
  mxFree(b->nu1);
  mxFree(b->pr);
  mxFree(b->mu);
  mxFree(b->Mu);
  mxFree(b->xi);
}

/* base HMMs (mex.c:459-473): fills b->nstates, prior, A, centres, covars */
static inline void pack_bases(buffers_t *bp, const mxArray *h3m_b, int Kb, int SB, int d,
                              int covmode) {
  buffers_t b = *bp;
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  b.SB = SB;
  b.nstates = (int *)mxCalloc((size_t)(Kb ? Kb : 1), sizeof(int));
  b.prior = (double *)mxCalloc((size_t)Kb * SB + 1, sizeof(double));
  b.A = (double *)mxCalloc((size_t)Kb * SB * SB + 1, sizeof(double));
  b.centres = (double *)mxCalloc((size_t)Kb * SB * d + 1, sizeof(double));
  b.covars = (double *)mxCalloc((size_t)Kb * SB * dd + 1, sizeof(double));
  for (int i = 0; i < Kb; i++) {
    const mxArray *hb = mxGetCell(h3m_b, i);
    const mxArray *mA = hb ? mxGetField(hb, 0, "A") : NULL;
    const int n = mA ? (int)mxGetM(mA) : -1;
    if (!mA || n < 1 || n > SB || (int)mxGetN(mA) != n) {
      *bp = b;
      free_buffers(bp);
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_b{%d}.A must be NxN with N <= maxN", i + 1);
    }
    b.nstates[i] = n;
    const double *pA = mxGetPr(mA);
    const double *pp = field_pr(hb, "prior", (size_t)n, "h3m_b");
    for (int r = 0; r < n; r++) {
      b.prior[(size_t)i * SB + r] = pp[r];
      for (int s = 0; s < n; s++) b.A[((size_t)i * SB + r) * SB + s] = pA[r + (size_t)s * n];
    }
    const mxArray *emit = mxGetField(hb, 0, "emit");
    for (int k = 0; k < n; k++) {
      const mxArray *ek = emit ? mxGetCell(emit, k) : NULL;
      if (!ek) {
        *bp = b;
        free_buffers(bp);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_b{%d}.emit{%d} missing", i + 1, k + 1);
      }
      const double *pc = field_pr(ek, "centres", (size_t)d, "h3m_b emit");
      const double *pv = field_pr(ek, "covars", dd, "h3m_b emit");
      double *dc = b.centres + ((size_t)i * SB + k) * d;
      double *dv = b.covars + ((size_t)i * SB + k) * dd;
      for (int a = 0; a < d; a++) dc[a] = pc[a];
      if (covmode == VBHEM_COV_FULL) {
        for (int a = 0; a < d; a++)
          for (int c2 = 0; c2 < d; c2++) dv[(size_t)a * d + c2] = pv[a + (size_t)c2 * d];
      } else {
        for (int a = 0; a < d; a++) dv[a] = pv[a];
      }
    }
  }

  *bp = b;
}


/* Cluster state counts (mex.c:436-437: N2 = rows of the cluster's transition
 * field, one per cluster, looped with at :506).  Fills N2[Kr]; returns S = max N2,
 * the stride the clusters are packed at.  Every N2 must be square and <= maxN2. */
static inline int cluster_sizes(const mxArray *h3m_r, int Kr, const char *afield, int maxN2,
                                int *N2) {
  int S = 0;
  for (int j = 0; j < Kr; j++) {
    const mxArray *hr = mxGetCell(h3m_r, j);
    if (!hr || !mxIsStruct(hr))
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{%d} must be a struct", j + 1);
    const mxArray *lA = mxGetField(hr, 0, afield);
    const int n = lA ? (int)mxGetM(lA) : 0;
    if (!lA || n < 1 || (int)mxGetN(lA) != n || n > maxN2)
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{%d}.%s must be N2 x N2 with N2 <= maxN2",
                        j + 1, afield);
    N2[j] = n;
    if (n > S) S = n;
  }
  return S;
}

static inline void alloc_clusters(buffers_t *b, int Kr, int S, int d, size_t dd) {
  b->N2 = (int *)mxCalloc((size_t)Kr, sizeof(int));
  b->logA = (double *)mxCalloc((size_t)Kr * S * S, sizeof(double));
  b->logPi = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
  b->m = (double *)mxCalloc((size_t)Kr * S * d, sizeof(double));
  b->P = (double *)mxCalloc((size_t)Kr * S * dd, sizeof(double));
  b->c = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
}

/* Padding of a cluster with N2 < S states to the common stride S (only the fused
 * gateway runs padded clusters: its responsibilities need every cluster in one
 * launch).  Padded states are unreachable: no transition into them and zero
 * prior (log = -inf), so their forward occupancy is 0 up to the restricted exp's
 * floor exp(-700) ~ 1e-304 (vbhem_math.h), and the real states' recursions see
 * them only through A' = exp(-inf) = 0.  A padded row moves uniformly to every
 * state (log 1/S), so its own column sums stay well above the underflow guard;
 * its emission constants (m = 0, P = 0, c = 0) give a finite E = -d log(2 pi)/2. */
static inline void pad_clusters(buffers_t *b, int Kr, int S, int d, size_t dd) {
  for (int j = 0; j < Kr; j++) {
    const int n = b->N2[j];
    for (int r = 0; r < S; r++) {
      for (int s = 0; s < S; s++) {
        double *a = b->logA + ((size_t)j * S + r) * S + s;
        if (r >= n) *a = -log((double)S);
        else if (s >= n) *a = -INFINITY;
      }
      if (r >= n) {
        b->logPi[(size_t)j * S + r] = -INFINITY;
        b->c[(size_t)j * S + r] = 0.0;
        memset(b->m + ((size_t)j * S + r) * d, 0, sizeof(double) * (size_t)d);
        memset(b->P + ((size_t)j * S + r) * dd, 0, sizeof(double) * dd);
      }
    }
  }
}

/* cluster HMMs (mex.c:433-457), N2[j] <= S states each, packed at stride S.
 * Fills b->N2, logA, logPi, m, P, c; full covariances take c and P from
 * logdetCovPlusDdivlamR / invCovR (mex.c:785-830: {1 x N2} and [d x d x N2]),
 * diagonal ones from the emit fields (mex.c:718-760).  Returns S. */
static inline int pack_clusters(buffers_t *bp, const mxArray *h3m_r, int Kr, int maxN2, int d,
                                int covmode, const mxArray *logdetR, const mxArray *invCovR) {
  buffers_t b = *bp;
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  int *n2 = (int *)mxCalloc((size_t)Kr, sizeof(int));
  const int S = cluster_sizes(h3m_r, Kr, "logATilde", maxN2, n2);
  alloc_clusters(&b, Kr, S, d, dd);
  memcpy(b.N2, n2, sizeof(int) * (size_t)Kr);
  mxFree(n2);
  for (int j = 0; j < Kr; j++) {
    const mxArray *hr = mxGetCell(h3m_r, j);
    const int n = b.N2[j];
    const double *pA = mxGetPr(mxGetField(hr, 0, "logATilde"));
    const double *pPi = field_pr(hr, "logPiTilde", (size_t)n, "h3m_r");
    for (int r = 0; r < n; r++) {
      b.logPi[(size_t)j * S + r] = pPi[r];
      for (int s = 0; s < n; s++) b.logA[((size_t)j * S + r) * S + s] = pA[r + (size_t)s * n];
    }
    const mxArray *emit = mxGetField(hr, 0, "emit");
    const double *ldet = NULL, *icov = NULL;
    if (covmode == VBHEM_COV_FULL) {
      const mxArray *lc = mxGetCell(logdetR, j), *ic = mxGetCell(invCovR, j);
      if (!lc || mxGetNumberOfElements(lc) != (size_t)n || !ic ||
          mxGetNumberOfElements(ic) != (size_t)n * d * d) {
        *bp = b;
        free_buffers(bp);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                          "logdetCovPlusDdivlamR{%d} / invCovR{%d} have wrong sizes", j + 1, j + 1);
      }
      ldet = mxGetPr(lc);
      icov = mxGetPr(ic);
    }
    for (int s = 0; s < n; s++) {
      const mxArray *es = emit ? mxGetCell(emit, s) : NULL;
      if (!es) {
        *bp = b;
        free_buffers(bp);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{%d}.emit{%d} missing", j + 1, s + 1);
      }
      const double *pm = field_pr(es, "m", (size_t)d, "h3m_r emit");
      double *dm = b.m + ((size_t)j * S + s) * d;
      for (int a = 0; a < d; a++) dm[a] = pm[a];
      double *dP = b.P + ((size_t)j * S + s) * dd;
      if (covmode == VBHEM_COV_FULL) {
        b.c[(size_t)j * S + s] = ldet[s];
        /* invCovR{j}(a,b,s) at a + b*d + s*d*d (column-major) */
        for (int a = 0; a < d; a++)
          for (int c2 = 0; c2 < d; c2++)
            dP[(size_t)a * d + c2] = icov[a + (size_t)c2 * d + (size_t)s * d * d];
      } else {
        const double *pW = field_pr(es, "W", (size_t)d, "h3m_r emit");
        const double v = field_pr(es, "v", 1, "h3m_r emit")[0];
        b.c[(size_t)j * S + s] = field_pr(es, "logLambdaTildePlusDdivlamda", 1, "h3m_r emit")[0];
        for (int a = 0; a < d; a++) dP[a] = v * pW[a];
      }
    }
  }
  pad_clusters(&b, Kr, S, d, dd);
  *bp = b;
  return S;
}

/* The per-pair entry points (vbhem_estep_pairs_host / vhem_estep_pairs_host)
 * behind one signature. */
typedef int (*pairs_host_fn)(void *ctx, const vbhem_base_t *base, const vbhem_cluster_t *clus,
                             int T, double *LL, double *nu1, double *pr, double *mu, double *Mu,
                             double *xi);

/* The per-pair gateways' computation and outputs (mex.c:396-409, 1108-1122,
 * 1312-1345; column-major, N2[j]-shaped cells per cluster).  Clusters of
 * different sizes (mex.c:506) run as one library call per distinct N2 on the
 * clusters of that size, unpadded: every pair's outputs are those of a call with
 * only its own cluster, as in the reference's per-cluster loop. */
static inline void run_pairs_grouped(mxArray *plhs[], buffers_t *bp, int Kb, int Kr, int S,
                                     int d, int covmode, int T, pairs_host_fn fn, void *ctx,
                                     const char *fname) {
  const buffers_t b = *bp;
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  plhs[0] = mxCreateDoubleMatrix(Kb, Kr, mxREAL);
  for (int k = 1; k < 6; k++) plhs[k] = mxCreateCellMatrix(Kb, Kr);
  double *LLo = mxGetPr(plhs[0]);
  int *idx = (int *)mxCalloc((size_t)Kr, sizeof(int));
  for (int n = 1; n <= S; n++) {
    int cnt = 0;
    for (int j = 0; j < Kr; j++)
      if (b.N2[j] == n) idx[cnt++] = j;
    if (cnt == 0) continue;
    /* this size's clusters, compact at stride n */
    double *gA = (double *)mxCalloc((size_t)cnt * n * n, sizeof(double));
    double *gPi = (double *)mxCalloc((size_t)cnt * n, sizeof(double));
    double *gm = (double *)mxCalloc((size_t)cnt * n * d, sizeof(double));
    double *gP = (double *)mxCalloc((size_t)cnt * n * dd, sizeof(double));
    double *gc = (double *)mxCalloc((size_t)cnt * n, sizeof(double));
    for (int g = 0; g < cnt; g++) {
      const int j = idx[g];
      for (int r = 0; r < n; r++) {
        gPi[(size_t)g * n + r] = b.logPi[(size_t)j * S + r];
        gc[(size_t)g * n + r] = b.c[(size_t)j * S + r];
        for (int s = 0; s < n; s++)
          gA[((size_t)g * n + r) * n + s] = b.logA[((size_t)j * S + r) * S + s];
        memcpy(gm + ((size_t)g * n + r) * d, b.m + ((size_t)j * S + r) * d, sizeof(double) * d);
        memcpy(gP + ((size_t)g * n + r) * dd, b.P + ((size_t)j * S + r) * dd, sizeof(double) * dd);
      }
    }
    const size_t np = (size_t)Kb * cnt;
    double *LL = (double *)mxCalloc(np + 1, sizeof(double));
    double *nu1 = (double *)mxCalloc(np * n + 1, sizeof(double));
    double *pr = (double *)mxCalloc(np * n + 1, sizeof(double));
    double *mu = (double *)mxCalloc(np * n * d + 1, sizeof(double));
    double *Mu = (double *)mxCalloc(np * n * dd + 1, sizeof(double));
    double *xi = (double *)mxCalloc(np * n * n + 1, sizeof(double));
    if (Kb > 0) {
      vbhem_base_t base = {Kb, b.SB, d, covmode, b.nstates, b.prior, b.A, b.centres, b.covars, NULL};
      vbhem_cluster_t clus = {cnt, n, gA, gPi, gm, gP, gc};
      const int st = fn(ctx, &base, &clus, T, LL, nu1, pr, mu, Mu, xi);
      if (st != VBHEM_OK) {
        free_buffers(bp);
        mexErrMsgIdAndTxt("vbhem_mex:gpu", "%s failed (%d): %s", fname, st, vbhem_last_error());
      }
    }
    for (int i = 0; i < Kb; i++) {
      for (int g = 0; g < cnt; g++) {
        const int j = idx[g];
        const size_t p = (size_t)i * cnt + g;           /* row-major pair index of the call */
        const size_t cell = (size_t)i + (size_t)j * Kb;  /* IX(i,j,Kb,Kr) */
        LLo[cell] = LL[p];
        mxArray *a_nu = mxCreateDoubleMatrix(1, n, mxREAL);
        mxArray *a_pr = mxCreateDoubleMatrix(n, 1, mxREAL);
        mxArray *a_mu = mxCreateDoubleMatrix(n, d, mxREAL);
        mxArray *a_Mu;
        if (covmode == VBHEM_COV_FULL) {
          mwSize dims[3] = {(mwSize)n, (mwSize)d, (mwSize)d};
          a_Mu = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
        } else {
          a_Mu = mxCreateDoubleMatrix(n, d, mxREAL);
        }
        mxArray *a_xi = mxCreateDoubleMatrix(n, n, mxREAL);
        double *o_nu = mxGetPr(a_nu), *o_pr = mxGetPr(a_pr), *o_mu = mxGetPr(a_mu);
        double *o_Mu = mxGetPr(a_Mu), *o_xi = mxGetPr(a_xi);
        for (int s = 0; s < n; s++) {
          o_nu[s] = nu1[p * n + s];
          o_pr[s] = pr[p * n + s];
          for (int a = 0; a < d; a++) {
            o_mu[s + (size_t)a * n] = mu[(p * n + s) * d + a];
            if (covmode == VBHEM_COV_FULL) {
              for (int c2 = 0; c2 < d; c2++)
                o_Mu[s + (size_t)a * n + (size_t)c2 * n * d] = Mu[((p * n + s) * d + a) * d + c2];
            } else {
              o_Mu[s + (size_t)a * n] = Mu[(p * n + s) * d + a];
            }
          }
          for (int s2 = 0; s2 < n; s2++) o_xi[s + (size_t)s2 * n] = xi[(p * n + s) * n + s2];
        }
        mxSetCell(plhs[1], cell, a_nu);
        mxSetCell(plhs[2], cell, a_pr);
        mxSetCell(plhs[3], cell, a_mu);
        mxSetCell(plhs[4], cell, a_Mu);
        mxSetCell(plhs[5], cell, a_xi);
      }
    }
    mxFree(gA);
    mxFree(gPi);
    mxFree(gm);
    mxFree(gP);
    mxFree(gc);
    mxFree(LL);
    mxFree(nu1);
    mxFree(pr);
    mxFree(mu);
    mxFree(Mu);
    mxFree(xi);
  }
  mxFree(idx);
}

#endif /* H3M_MEX_COMMON_H */

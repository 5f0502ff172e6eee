/*
 * integration/h3m_mex_common.h -- shared by the two MEX gateways
 * (vbhem_hmm_bwd_fwd_mex.c, hem_hmm_bwd_fwd_mex.c): scalar/field parsing, the
 * host buffers, the base-HMM repack (column-major cells -> row-major, padded to
 * maxN states) and the output scatter into MATLAB cells.  The two reference
 * gateways share this code too (mex.c:288-409, 459-473, 1108-1122, 1312-1345 /
 * hem_hmm_bwd_fwd_mex.c:288-409).
 */
#ifndef H3M_MEX_COMMON_H
#define H3M_MEX_COMMON_H
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
  int *nstates;
  double *prior, *A, *centres, *covars;
  double *logA, *logPi, *m, *P, *c;
  double *LL, *nu1, *pr, *mu, *Mu, *xi;
} buffers_t;

static inline void free_buffers(buffers_t *b) {
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


/* cluster HMMs (mex.c:433-457): every cluster has S = maxN2 states.  Fills
 * b->logA, logPi, m, P, c; full covariances take c and P from
 * logdetCovPlusDdivlamR / invCovR (mex.c:785-830), diagonal ones from the emit
 * fields (mex.c:718-760). */
static inline void pack_clusters(buffers_t *bp, const mxArray *h3m_r, int Kr, int S, int d,
                                 int covmode, const mxArray *logdetR, const mxArray *invCovR) {
  buffers_t b = *bp;
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  b.logA = (double *)mxCalloc((size_t)Kr * S * S, sizeof(double));
  b.logPi = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
  b.m = (double *)mxCalloc((size_t)Kr * S * d, sizeof(double));
  b.P = (double *)mxCalloc((size_t)Kr * S * dd, sizeof(double));
  b.c = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
  for (int j = 0; j < Kr; j++) {
    const mxArray *hr = mxGetCell(h3m_r, j);
    if (!hr || !mxIsStruct(hr)) {
      *bp = b;
      free_buffers(bp);
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{%d} must be a struct", j + 1);
    }
    const mxArray *lA = mxGetField(hr, 0, "logATilde");
    if (!lA || (int)mxGetM(lA) != S || (int)mxGetN(lA) != S) {
      *bp = b;
      free_buffers(bp);
      mexErrMsgIdAndTxt("vbhem_mex:unsupported",
                        "h3m_r{%d}.logATilde must be maxN2 x maxN2 (all clusters equal size)", j + 1);
    }
    const double *pA = mxGetPr(lA);
    const double *pPi = field_pr(hr, "logPiTilde", (size_t)S, "h3m_r");
    for (int r = 0; r < S; r++) {
      b.logPi[(size_t)j * S + r] = pPi[r];
      for (int s = 0; s < S; s++) b.logA[((size_t)j * S + r) * S + s] = pA[r + (size_t)s * S];
    }
    const mxArray *emit = mxGetField(hr, 0, "emit");
    const double *ldet = NULL, *icov = NULL;
    if (covmode == VBHEM_COV_FULL) {
      const mxArray *lc = mxGetCell(logdetR, j), *ic = mxGetCell(invCovR, j);
      if (!lc || mxGetNumberOfElements(lc) != (size_t)S || !ic ||
          mxGetNumberOfElements(ic) != (size_t)S * d * d) {
        *bp = b;
      free_buffers(bp);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                          "logdetCovPlusDdivlamR{%d} / invCovR{%d} have wrong sizes", j + 1, j + 1);
      }
      ldet = mxGetPr(lc);
      icov = mxGetPr(ic);
    }
    for (int s = 0; s < S; s++) {
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

  *bp = b;
}

/* outputs (mex.c:396-409, 1108-1122, 1312-1345), column-major */
static inline void scatter_outputs(mxArray *plhs[], const buffers_t *bp, int Kb, int Kr, int S,
                                   int d, int covmode) {
  const buffers_t b = *bp;
  plhs[0] = mxCreateDoubleMatrix(Kb, Kr, mxREAL);
  for (int k = 1; k < 6; k++) plhs[k] = mxCreateCellMatrix(Kb, Kr);
  double *LL = mxGetPr(plhs[0]);
  for (int i = 0; i < Kb; i++) {
    for (int j = 0; j < Kr; j++) {
      const size_t p = (size_t)i * Kr + j;       /* row-major pair index */
      const size_t cell = (size_t)i + (size_t)j * Kb; /* IX(i,j,Kb,Kr) */
      LL[cell] = b.LL[p];
      mxArray *a_nu = mxCreateDoubleMatrix(1, S, mxREAL);
      mxArray *a_pr = mxCreateDoubleMatrix(S, 1, mxREAL);
      mxArray *a_mu = mxCreateDoubleMatrix(S, d, mxREAL);
      mxArray *a_Mu;
      if (covmode == VBHEM_COV_FULL) {
        mwSize dims[3] = {(mwSize)S, (mwSize)d, (mwSize)d};
        a_Mu = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
      } else {
        a_Mu = mxCreateDoubleMatrix(S, d, mxREAL);
      }
      mxArray *a_xi = mxCreateDoubleMatrix(S, S, mxREAL);
      double *o_nu = mxGetPr(a_nu), *o_pr = mxGetPr(a_pr), *o_mu = mxGetPr(a_mu);
      double *o_Mu = mxGetPr(a_Mu), *o_xi = mxGetPr(a_xi);
      for (int s = 0; s < S; s++) {
        o_nu[s] = b.nu1[p * S + s];
        o_pr[s] = b.pr[p * S + s];
        for (int a = 0; a < d; a++) {
          o_mu[s + (size_t)a * S] = b.mu[(p * S + s) * d + a];
          if (covmode == VBHEM_COV_FULL) {
            for (int c2 = 0; c2 < d; c2++)
              o_Mu[s + (size_t)a * S + (size_t)c2 * S * d] =
                  b.Mu[((p * S + s) * d + a) * d + c2];
          } else {
            o_Mu[s + (size_t)a * S] = b.Mu[(p * S + s) * d + a];
          }
        }
        for (int s2 = 0; s2 < S; s2++) o_xi[s + (size_t)s2 * S] = b.xi[(p * S + s) * S + s2];
      }
      mxSetCell(plhs[1], cell, a_nu);
      mxSetCell(plhs[2], cell, a_pr);
      mxSetCell(plhs[3], cell, a_mu);
      mxSetCell(plhs[4], cell, a_Mu);
      mxSetCell(plhs[5], cell, a_xi);
    }
  }
}

#endif /* H3M_MEX_COMMON_H */

/*
 * integration/vbhem_hmm_bwd_fwd_mex.c -- MATLAB MEX gateway that replaces the
 * reference's src/vbhem/vbhem_hmm_bwd_fwd_mex.c with a call into the MI355X
 * E-step (libvbhem_estep.so, include/vbhem_estep.h).
 *
 * Same MATLAB signature, argument checks, error identifiers and output shapes
 * as the reference gateway (mex.c:288-409, output cells mex.c:1108-1122,
 * 1312-1345):
 *
 *   [LL_elbo, sum_nu_1, update_emit_pr, update_emit_mu, update_emit_Mu, sum_xi] =
 *       vbhem_hmm_bwd_fwd_mex(h3m_b.hmm, h3m_r.hmm, T, maxN, maxN2
 *                             [, logdetCovPlusDdivlamR, invCovR])
 *
 * 5 inputs = diagonal covariances, 7 inputs = full (mex.c:335-346).  The
 * gateway only repacks MATLAB's column-major cell/struct data into the dense
 * row-major arrays of vbhem_base_t / vbhem_cluster_t, calls
 * vbhem_estep_pairs_host(), and scatters the results back into MATLAB cells.
 *
 * Emission constants, as the reference kernel reads them:
 *   full: c = logdetCovPlusDdivlamR{j}(rho), P = invCovR{j}(:,:,rho)   (mex.c:785-830)
 *   diag: c = emit{rho}.logLambdaTildePlusDdivlamda, P = emit{rho}.v * emit{rho}.W
 *                                                                        (mex.c:718-760)
 * The GPU device is taken from the environment variable VBHEM_DEVICE (default 0).
 *
 * Build (MATLAB):  mex -R2017b -I../include vbhem_hmm_bwd_fwd_mex.c -L../lib -lvbhem_estep
 * (see INTEGRATION.md).  In this repository the file is also built against a
 * test double of the mx API (tests/mxshim) so the gateway itself is tested.
 */
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "vbhem_estep.h"

/* the reference's scalar parser (mex.c:77-86): must be a 1x1 double */
static double parse_scalar(const mxArray *mx) {
  if (!mx || !mxIsDouble(mx) || mxGetNumberOfElements(mx) != 1)
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "arg must be scalar.");
  return mxGetScalar(mx);
}

static const double *field_pr(const mxArray *s, const char *name, size_t numel_expected,
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

static void free_buffers(buffers_t *b) {
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

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if ((nrhs != 5) && (nrhs != 7))
    mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nrhs", "5 or 7 inputs required.");
  if (nlhs != 6) mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nlhs", "6 output required.");
  const int covmode = (nrhs == 7) ? VBHEM_COV_FULL : VBHEM_COV_DIAG;
  if (!mxIsCell(prhs[0])) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "1st arg must be cell");
  if (!mxIsCell(prhs[1])) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "2nd arg must be cell");
  const mxArray *h3m_b = prhs[0], *h3m_r = prhs[1];
  const int Kr = (int)mxGetNumberOfElements(h3m_r);
  const int Kb = (int)mxGetNumberOfElements(h3m_b);
  const int T = (int)parse_scalar(prhs[2]);
  const int maxN = (int)parse_scalar(prhs[3]);
  const int maxN2 = (int)parse_scalar(prhs[4]);
  const mxArray *logdetR = NULL, *invCovR = NULL;
  if (covmode == VBHEM_COV_FULL) {
    logdetR = prhs[5];
    invCovR = prhs[6];
    if (!mxIsCell(logdetR) || (int)mxGetNumberOfElements(logdetR) != Kr)
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "6th arg must be a cell {1xKr}");
    if (!mxIsCell(invCovR) || (int)mxGetNumberOfElements(invCovR) != Kr)
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "7th arg must be a cell {1xKr}");
  }
  if (Kr < 1 || Kb < 0 || T < 1 || maxN < 1 || maxN2 < 1)
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "invalid sizes (Kr=%d Kb=%d T=%d maxN=%d maxN2=%d)",
                      Kr, Kb, T, maxN, maxN2);

  /* ---- cluster HMMs (mex.c:433-457): all clusters must have maxN2 states -------- */
  int d = -1;
  {
    const mxArray *hr = mxGetCell(h3m_r, 0);
    const mxArray *e = hr ? mxGetField(hr, 0, "emit") : NULL;
    const mxArray *e0 = e ? mxGetCell(e, 0) : NULL;
    const mxArray *m0 = e0 ? mxGetField(e0, 0, "m") : NULL;
    if (!m0) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{1}.emit{1}.m missing");
    d = (int)mxGetN(m0);
  }
  const int S = maxN2, SB = maxN;
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  buffers_t b;
  memset(&b, 0, sizeof(b));
  b.logA = (double *)mxCalloc((size_t)Kr * S * S, sizeof(double));
  b.logPi = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
  b.m = (double *)mxCalloc((size_t)Kr * S * d, sizeof(double));
  b.P = (double *)mxCalloc((size_t)Kr * S * dd, sizeof(double));
  b.c = (double *)mxCalloc((size_t)Kr * S, sizeof(double));
  for (int j = 0; j < Kr; j++) {
    const mxArray *hr = mxGetCell(h3m_r, j);
    if (!hr || !mxIsStruct(hr)) {
      free_buffers(&b);
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{%d} must be a struct", j + 1);
    }
    const mxArray *lA = mxGetField(hr, 0, "logATilde");
    if (!lA || (int)mxGetM(lA) != S || (int)mxGetN(lA) != S) {
      free_buffers(&b);
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
        free_buffers(&b);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                          "logdetCovPlusDdivlamR{%d} / invCovR{%d} have wrong sizes", j + 1, j + 1);
      }
      ldet = mxGetPr(lc);
      icov = mxGetPr(ic);
    }
    for (int s = 0; s < S; s++) {
      const mxArray *es = emit ? mxGetCell(emit, s) : NULL;
      if (!es) {
        free_buffers(&b);
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

  /* ---- base HMMs (mex.c:459-473), zero-padded to maxN states ------------------- */
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
      free_buffers(&b);
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
        free_buffers(&b);
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

  /* ---- compute on the GPU ---------------------------------------------------- */
  const size_t np = (size_t)Kb * Kr;
  b.LL = (double *)mxCalloc(np + 1, sizeof(double));
  b.nu1 = (double *)mxCalloc(np * S + 1, sizeof(double));
  b.pr = (double *)mxCalloc(np * S + 1, sizeof(double));
  b.mu = (double *)mxCalloc(np * S * d + 1, sizeof(double));
  b.Mu = (double *)mxCalloc(np * S * dd + 1, sizeof(double));
  b.xi = (double *)mxCalloc(np * S * S + 1, sizeof(double));
  if (Kb > 0) {
    vbhem_base_t base = {Kb, SB, d, covmode, b.nstates, b.prior, b.A, b.centres, b.covars};
    vbhem_cluster_t clus = {Kr, S, b.logA, b.logPi, b.m, b.P, b.c};
    const char *dev_env = getenv("VBHEM_DEVICE");
    const int device = dev_env ? atoi(dev_env) : 0;
    const int st = vbhem_estep_pairs_host(device, &base, &clus, T, b.LL, b.nu1, b.pr, b.mu, b.Mu,
                                          b.xi);
    if (st != VBHEM_OK) {
      free_buffers(&b);
      mexErrMsgIdAndTxt("vbhem_mex:gpu", "vbhem_estep_pairs_host failed (%d): %s", st,
                        vbhem_last_error());
    }
  }

  /* ---- outputs (mex.c:396-409, 1108-1122, 1312-1345), column-major ----------- */
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
  free_buffers(&b);
}

/*
 * integration/hem_hmm_bwd_fwd_mex.c -- MATLAB MEX gateway that replaces the
 * reference's VHEM sibling src/compare_mtds/hem/vhem_h3m/hem_hmm_bwd_fwd_mex.c
 * with a call into the MI355X E-step (vhem_estep_pairs_host, include/vbhem_estep.h).
 *
 * Same MATLAB signature, argument checks, error identifiers and output shapes
 * as the reference gateway (hem_hmm_bwd_fwd_mex.c:288-409):
 *
 *   [LL_elbo, sum_nu_1, update_emit_pr, update_emit_mu, update_emit_Mu, sum_xi] =
 *       hem_hmm_bwd_fwd_mex(h3m_b.hmm, h3m_r.hmm, T, smooth, maxN, maxN2
 *                           [, logdetCovR, invCovR])
 *
 * 6 inputs = diagonal covariances, 8 inputs = full (:334-346), called from
 * hem_h3m_c_step.m:191-192 / :208-209.  The reduced HMMs are point estimates
 * {A, prior, emit{k}.centres, emit{k}.covars}; the gateway turns them into the
 * cluster constants the kernels read:
 *   logA = log(A) (:906-922), logPi = log(prior) (:1004-1019), m = centres,
 *   full: c = logdetCovR{j}(k), P = invCovR{j}(:,:,k)  (:585-600)
 *   diag: c = sum(log(covars)), P = 1 ./ covars        (:711-733)
 * and the kernels divide the expected emission log-likelihood by `smooth`
 * (:848-860).  The GPU device is taken from VBHEM_DEVICE (default 0).
 */
#include <math.h>

#include "h3m_mex_common.h"

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if ((nrhs != 6) && (nrhs != 8))
    mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nrhs", "4 or 6 inputs required.");
  if (nlhs != 6) mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nlhs", "6 output required.");
  const int covmode = (nrhs == 8) ? VBHEM_COV_FULL : VBHEM_COV_DIAG;
  if (!mxIsCell(prhs[0])) mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "1st arg must be cell");
  if (!mxIsCell(prhs[1])) mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "2nd arg must be cell");
  const mxArray *h3m_b = prhs[0], *h3m_r = prhs[1];
  const int Kr = (int)mxGetNumberOfElements(h3m_r);
  const int Kb = (int)mxGetNumberOfElements(h3m_b);
  const int T = (int)parse_scalar(prhs[2]);
  const double smooth = parse_scalar(prhs[3]);
  const int maxN = (int)parse_scalar(prhs[4]);
  const int maxN2 = (int)parse_scalar(prhs[5]);
  const mxArray *logdetR = NULL, *invCovR = NULL;
  if (covmode == VBHEM_COV_FULL) {
    logdetR = prhs[6];
    invCovR = prhs[7];
    if (!mxIsCell(logdetR) || (int)mxGetNumberOfElements(logdetR) != Kr)
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "7th arg must be a cell {1xKr}");
    if (!mxIsCell(invCovR) || (int)mxGetNumberOfElements(invCovR) != Kr)
      mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "8th arg must be a cell {1xKr}");
  }
  if (Kr < 1 || Kb < 0 || T < 1 || maxN < 1 || maxN2 < 1 || !(smooth > 0.0))
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                      "invalid sizes (Kr=%d Kb=%d T=%d maxN=%d maxN2=%d smooth=%g)", Kr, Kb, T,
                      maxN, maxN2, smooth);

  /* ---- reduced HMMs (:428-447): all clusters must have maxN2 states ----------------- */
  int d = -1;
  {
    const mxArray *hr = mxGetCell(h3m_r, 0);
    const mxArray *e = hr ? mxGetField(hr, 0, "emit") : NULL;
    const mxArray *e0 = e ? mxGetCell(e, 0) : NULL;
    const mxArray *c0 = e0 ? mxGetField(e0, 0, "centres") : NULL;
    if (!c0) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{1}.emit{1}.centres missing");
    d = (int)mxGetNumberOfElements(c0);
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
    const mxArray *mA = mxGetField(hr, 0, "A");
    if (!mA || (int)mxGetM(mA) != S || (int)mxGetN(mA) != S) {
      free_buffers(&b);
      mexErrMsgIdAndTxt("vbhem_mex:unsupported",
                        "h3m_r{%d}.A must be maxN2 x maxN2 (all clusters equal size)", j + 1);
    }
    const double *pA = mxGetPr(mA);
    const double *pPi = field_pr(hr, "prior", (size_t)S, "h3m_r");
    for (int r = 0; r < S; r++) {
      b.logPi[(size_t)j * S + r] = log(pPi[r]);
      for (int s = 0; s < S; s++) b.logA[((size_t)j * S + r) * S + s] = log(pA[r + (size_t)s * S]);
    }
    const mxArray *emit = mxGetField(hr, 0, "emit");
    const double *ldet = NULL, *icov = NULL;
    if (covmode == VBHEM_COV_FULL) {
      const mxArray *lc = mxGetCell(logdetR, j), *ic = mxGetCell(invCovR, j);
      if (!lc || mxGetNumberOfElements(lc) != (size_t)S || !ic ||
          mxGetNumberOfElements(ic) != (size_t)S * d * d) {
        free_buffers(&b);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                          "logdetCovR{%d} / invCovR{%d} have wrong sizes", j + 1, j + 1);
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
      const double *pm = field_pr(es, "centres", (size_t)d, "h3m_r emit");
      double *dm = b.m + ((size_t)j * S + s) * d;
      for (int a = 0; a < d; a++) dm[a] = pm[a];
      double *dP = b.P + ((size_t)j * S + s) * dd;
      if (covmode == VBHEM_COV_FULL) {
        b.c[(size_t)j * S + s] = ldet[s];
        for (int a = 0; a < d; a++)
          for (int c2 = 0; c2 < d; c2++)
            dP[(size_t)a * d + c2] = icov[a + (size_t)c2 * d + (size_t)s * d * d];
      } else {
        const double *pv = field_pr(es, "covars", (size_t)d, "h3m_r emit");
        double lsum = 0.0;
        for (int a = 0; a < d; a++) {
          lsum += log(pv[a]);
          dP[a] = 1.0 / pv[a];
        }
        b.c[(size_t)j * S + s] = lsum;
      }
    }
  }

  pack_bases(&b, h3m_b, Kb, SB, d, covmode);

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
    const int st = vhem_estep_pairs_host(device, &base, &clus, T, smooth, b.LL, b.nu1, b.pr, b.mu,
                                         b.Mu, b.xi);
    if (st != VBHEM_OK) {
      free_buffers(&b);
      mexErrMsgIdAndTxt("vbhem_mex:gpu", "vhem_estep_pairs_host failed (%d): %s", st,
                        vbhem_last_error());
    }
  }

  scatter_outputs(plhs, &b, Kb, Kr, S, d, covmode);
  free_buffers(&b);
}

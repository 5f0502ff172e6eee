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
 * (:848-860).  Reduced HMMs may have different state counts N2 <= maxN2: one
 * library call per distinct N2.  The GPU device is taken from VBHEM_DEVICE (default 0).
 */
#include <math.h>

#include "h3m_mex_common.h"

static int call_pairs(void *ctx, const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      double *LL, double *nu1, double *pr, double *mu, double *Mu, double *xi) {
  const char *dev_env = getenv("VBHEM_DEVICE");
  const int device = dev_env ? atoi(dev_env) : 0;
  return vhem_estep_pairs_host(device, base, clus, T, *(const double *)ctx, LL, nu1, pr, mu, Mu,
                               xi);
}

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

  /* ---- reduced HMMs (:428-447; N2 per cluster) -------------------------------- */
  int d = -1;
  {
    const mxArray *hr = mxGetCell(h3m_r, 0);
    const mxArray *e = hr ? mxGetField(hr, 0, "emit") : NULL;
    const mxArray *e0 = e ? mxGetCell(e, 0) : NULL;
    const mxArray *c0 = e0 ? mxGetField(e0, 0, "centres") : NULL;
    if (!c0) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{1}.emit{1}.centres missing");
    d = (int)mxGetNumberOfElements(c0);
  }
  const size_t dd = (covmode == VBHEM_COV_FULL) ? (size_t)d * d : (size_t)d;
  buffers_t b;
  memset(&b, 0, sizeof(b));
  int *n2 = (int *)mxCalloc((size_t)Kr, sizeof(int));
  const int S = cluster_sizes(h3m_r, Kr, "A", maxN2, n2);
  alloc_clusters(&b, Kr, S, d, dd);
  memcpy(b.N2, n2, sizeof(int) * (size_t)Kr);
  mxFree(n2);
  for (int j = 0; j < Kr; j++) {
    const mxArray *hr = mxGetCell(h3m_r, j);
    const int n = b.N2[j];
    const double *pA = mxGetPr(mxGetField(hr, 0, "A"));
    const double *pPi = field_pr(hr, "prior", (size_t)n, "h3m_r");
    for (int r = 0; r < n; r++) {
      b.logPi[(size_t)j * S + r] = log(pPi[r]);
      for (int s = 0; s < n; s++) b.logA[((size_t)j * S + r) * S + s] = log(pA[r + (size_t)s * n]);
    }
    const mxArray *emit = mxGetField(hr, 0, "emit");
    const double *ldet = NULL, *icov = NULL;
    if (covmode == VBHEM_COV_FULL) {
      const mxArray *lc = mxGetCell(logdetR, j), *ic = mxGetCell(invCovR, j);
      if (!lc || mxGetNumberOfElements(lc) != (size_t)n || !ic ||
          mxGetNumberOfElements(ic) != (size_t)n * d * d) {
        free_buffers(&b);
        mexErrMsgIdAndTxt("vbhem_mex:invalidinput",
                          "logdetCovR{%d} / invCovR{%d} have wrong sizes", j + 1, j + 1);
      }
      ldet = mxGetPr(lc);
      icov = mxGetPr(ic);
    }
    for (int s = 0; s < n; s++) {
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

  pack_bases(&b, h3m_b, Kb, maxN, d, covmode);

  /* ---- compute on the GPU, one call per distinct cluster size ----------------- */
  double sm = smooth;
  run_pairs_grouped(plhs, &b, Kb, Kr, S, d, covmode, T, call_pairs, &sm, "vhem_estep_pairs_host");
  free_buffers(&b);
}

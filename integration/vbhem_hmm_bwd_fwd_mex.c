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
 * Clusters may have different state counts N2 <= maxN2 (mex.c:436-437, 506): one
 * library call per distinct N2, outputs shaped per cluster as the reference's.
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
#include "h3m_mex_common.h"

static int call_pairs(void *ctx, const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      double *LL, double *nu1, double *pr, double *mu, double *Mu, double *xi) {
  (void)ctx;
  const char *dev_env = getenv("VBHEM_DEVICE");
  const int device = dev_env ? atoi(dev_env) : 0;
  return vbhem_estep_pairs_host(device, base, clus, T, LL, nu1, pr, mu, Mu, xi);
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

  /* ---- cluster HMMs (mex.c:433-457; N2 per cluster, :436-437) ---------------- */
  int d = -1;
  {
    const mxArray *hr = mxGetCell(h3m_r, 0);
    const mxArray *e = hr ? mxGetField(hr, 0, "emit") : NULL;
    const mxArray *e0 = e ? mxGetCell(e, 0) : NULL;
    const mxArray *m0 = e0 ? mxGetField(e0, 0, "m") : NULL;
    if (!m0) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{1}.emit{1}.m missing");
    d = (int)mxGetN(m0);
  }
  buffers_t b;
  memset(&b, 0, sizeof(b));
  const int S = pack_clusters(&b, h3m_r, Kr, maxN2, d, covmode, logdetR, invCovR);
  pack_bases(&b, h3m_b, Kb, maxN, d, covmode);

  /* ---- compute on the GPU, one call per distinct cluster size ----------------- */
  run_pairs_grouped(plhs, &b, Kb, Kr, S, d, covmode, T, call_pairs, NULL,
                    "vbhem_estep_pairs_host");
  free_buffers(&b);
}

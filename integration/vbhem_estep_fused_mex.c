/*
 * integration/vbhem_estep_fused_mex.c -- MATLAB MEX gateway for the FUSED E-step
 * of one EM iteration: the per-pair recursions (vbhem_hmm_bwd_fwd_mex), the
 * responsibilities (vbhem_h3m_c_step_fc.m:270-283), the gated Z-weighted
 * statistic sums (vbhem_compute_Statistics.m:33-55) and the ELBO partial sums
 * (vbhemh3m_lb.m:90,107) in one call, with the base HMMs kept resident on the
 * GPU between calls.
 *
 *   [LL_elbo, hat_Z, stats] = vbhem_estep_fused_mex(h3m_b.hmm, h3m_r.hmm, T, maxN, maxN2,
 *                                 [logdetCovPlusDdivlamR, invCovR,] tilde_N_k, logOmegaTilde
 *                                 [, base_key])
 *   vbhem_estep_fused_mex()      % no arguments: free the resident base set
 *
 * Inputs 1-5 (and 6-7 for full covariances) are exactly the arguments of
 * vbhem_hmm_bwd_fwd_mex (mex.c:288-473); 7 inputs = diagonal, 9 = full (8 / 10
 * with base_key).  Clusters may have different state counts N2 <= maxN2
 * (mex.c:436-437): they run padded to S = max N2 (h3m_mex_common.h:
 * pad_clusters), and cluster j's entries of stats for states >= N2(j) are zero
 * (up to ~1e-304); the caller reads states 1..N2(j).
 * tilde_N_k [Kb x 1] = Nv*Kb*omega (step_fc.m:26-30), logOmegaTilde [1 x Kr]
 * (step_fc.m:271-273).  Outputs: LL_elbo and hat_Z [Kb x Kr] (hat_Z includes the
 * +1e-50 of step_fc.m:277), stats [L x 1] the packed vector of
 * include/vbhem_estep.h: [Nj(Kr) | N1(Kr,S) | M(Kr,S,S) | Lt1 | Lt7 | U(Kr,S,NU)]
 * (C order; INTEGRATION.md gives the MATLAB unpacking and the patch of
 * vbhem_h3m_c_step_fc.m:168-296 that uses it).
 *
 * The base set is uploaded once and reused while the same base set is passed
 * again.  Without base_key the gateway decides that from a fingerprint of the
 * sizes and of the CONTENTS of every base field (prior, A, centres, covars: a
 * 64-bit hash read at memory speed, ~30 ms at N = 100 000), so an h3m_b rebuilt
 * in freed memory or edited in place is re-uploaded.  With base_key (a double
 * scalar) the caller vouches for the base set: it is reused while the key (and
 * the sizes) stay the same, and no base data is read -- a new key must be passed
 * whenever h3m_b changes.  The device is VBHEM_DEVICE (default 0).  Error
 * identifiers as the reference.
 */
#include <stdint.h>

#include "h3m_mex_common.h"

static vbhem_ctx_t *g_ctx = NULL;
static uint64_t g_fp = 0;

static void release(void) {
  if (g_ctx) vbhem_ctx_destroy(g_ctx);
  g_ctx = NULL;
  g_fp = 0;
}

static uint64_t mix64(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  return h;
}

/* contents of n doubles, four independent multiply-xor lanes (memory speed) */
static uint64_t hash_doubles(uint64_t h, const double *p, size_t n) {
  if (!p) return mix64(h, 0x5bd1e995ULL);
  const unsigned char *c = (const unsigned char *)p;
  uint64_t a[4] = {h, h ^ 0x243f6a8885a308d3ULL, h ^ 0x13198a2e03707344ULL, h ^ 0xa4093822299f31d0ULL};
  size_t i = 0;
  for (; i + 4 <= n; i += 4)
    for (int k = 0; k < 4; k++) {
      uint64_t w;
      memcpy(&w, c + 8 * (i + k), 8);
      a[k] = (a[k] ^ w) * 0x100000001b3ULL;
    }
  for (; i < n; i++) {
    uint64_t w;
    memcpy(&w, c + 8 * i, 8);
    a[0] = (a[0] ^ w) * 0x100000001b3ULL;
  }
  for (int k = 0; k < 4; k++) h = mix64(h, a[k]);
  return mix64(h, (uint64_t)n);
}

static uint64_t field_hash(uint64_t h, const mxArray *s, const char *name) {
  const mxArray *f = s ? mxGetField(s, 0, name) : NULL;
  return f ? hash_doubles(h, mxGetPr(f), mxGetNumberOfElements(f)) : mix64(h, 0x9e37ULL);
}

/* sizes (+ the caller's key, or the contents of every base field) */
static uint64_t base_fingerprint(const mxArray *h3m_b, int Kb, int SB, int d, int covmode,
                                 int Kr, int S, int T, int device, const mxArray *key) {
  uint64_t h = 1469598103934665603ULL;
  const int ints[] = {Kb, SB, d, covmode, Kr, S, T, device};
  for (int k = 0; k < 8; k++) h = mix64(h, (uint64_t)(uint32_t)ints[k]);
  if (key) {
    double kv = mxGetScalar(key);
    uint64_t w;
    memcpy(&w, &kv, 8);
    return mix64(mix64(h, 0x6b6579ULL), w);
  }
  for (int i = 0; i < Kb; i++) {
    const mxArray *hb = mxGetCell(h3m_b, i);
    h = field_hash(h, hb, "A");
    h = field_hash(h, hb, "prior");
    const mxArray *emit = hb ? mxGetField(hb, 0, "emit") : NULL;
    const int n = emit ? (int)mxGetNumberOfElements(emit) : 0;
    for (int s = 0; s < n; s++) {
      const mxArray *es = mxGetCell(emit, s);
      h = field_hash(h, es, "centres");
      h = field_hash(h, es, "covars");
    }
  }
  return h;
}

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  mexAtExit(release);
  if (nrhs == 0) {
    release();
    return;
  }
  if (nrhs < 7 || nrhs > 10)
    mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nrhs", "7 or 9 inputs required.");
  if (nlhs != 3) mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nlhs", "3 output required.");
  /* 7 / 9 inputs: diagonal / full; one more: base_key */
  const int covmode = (nrhs >= 9) ? VBHEM_COV_FULL : VBHEM_COV_DIAG;
  const mxArray *key = (nrhs == 8 || nrhs == 10) ? prhs[nrhs - 1] : NULL;
  if (key && (!mxIsDouble(key) || mxGetNumberOfElements(key) != 1))
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "base_key must be a double scalar");
  if (key) nrhs -= 1;
  if (!mxIsCell(prhs[0])) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "1st arg must be cell");
  if (!mxIsCell(prhs[1])) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "2nd arg must be cell");
  const mxArray *h3m_b = prhs[0], *h3m_r = prhs[1];
  const int Kr = (int)mxGetNumberOfElements(h3m_r);
  const int Kb = (int)mxGetNumberOfElements(h3m_b);
  const int T = (int)parse_scalar(prhs[2]);
  const int maxN = (int)parse_scalar(prhs[3]);
  const int maxN2 = (int)parse_scalar(prhs[4]);
  const mxArray *logdetR = covmode == VBHEM_COV_FULL ? prhs[5] : NULL;
  const mxArray *invCovR = covmode == VBHEM_COV_FULL ? prhs[6] : NULL;
  const mxArray *tN = prhs[nrhs - 2], *lOm = prhs[nrhs - 1];
  if (covmode == VBHEM_COV_FULL &&
      (!mxIsCell(logdetR) || (int)mxGetNumberOfElements(logdetR) != Kr || !mxIsCell(invCovR) ||
       (int)mxGetNumberOfElements(invCovR) != Kr))
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "6th/7th args must be cells {1xKr}");
  if (Kr < 1 || Kb < 0 || T < 1 || maxN < 1 || maxN2 < 1)
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "invalid sizes (Kr=%d Kb=%d T=%d maxN=%d maxN2=%d)",
                      Kr, Kb, T, maxN, maxN2);
  if (!mxIsDouble(tN) || (int)mxGetNumberOfElements(tN) != Kb)
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "tilde_N_k must be a double vector of Kb elements");
  if (!mxIsDouble(lOm) || (int)mxGetNumberOfElements(lOm) != Kr)
    mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "logOmegaTilde must be a double vector of Kr elements");

  int d = -1;
  {
    const mxArray *hr = mxGetCell(h3m_r, 0);
    const mxArray *e = hr ? mxGetField(hr, 0, "emit") : NULL;
    const mxArray *e0 = e ? mxGetCell(e, 0) : NULL;
    const mxArray *m0 = e0 ? mxGetField(e0, 0, "m") : NULL;
    if (!m0) mexErrMsgIdAndTxt("vbhem_mex:invalidinput", "h3m_r{1}.emit{1}.m missing");
    d = (int)mxGetN(m0);
  }
  const int SB = maxN;
  buffers_t b;
  memset(&b, 0, sizeof(b));
  const int S = pack_clusters(&b, h3m_r, Kr, maxN2, d, covmode, logdetR, invCovR);

  const char *dev_env = getenv("VBHEM_DEVICE");
  const int device = dev_env ? atoi(dev_env) : 0;
  const uint64_t fp = base_fingerprint(h3m_b, Kb, SB, d, covmode, Kr, S, T, device, key);
  if (!g_ctx || fp != g_fp) {
    release();
    pack_bases(&b, h3m_b, Kb, SB, d, covmode);
    vbhem_base_t base = {Kb, SB, d, covmode, b.nstates, b.prior, b.A, b.centres, b.covars, NULL};
    const int st = vbhem_ctx_create(device, &base, Kr, S, 1, T, &g_ctx);
    if (st != VBHEM_OK) {
      free_buffers(&b);
      g_ctx = NULL;
      mexErrMsgIdAndTxt("vbhem_mex:gpu", "vbhem_ctx_create failed (%d): %s", st, vbhem_last_error());
    }
    g_fp = fp;
  }
  const size_t L = vbhem_stats_len(Kr, S, d, covmode);
  plhs[0] = mxCreateDoubleMatrix(Kb, Kr, mxREAL);
  plhs[1] = mxCreateDoubleMatrix(Kb, Kr, mxREAL);
  plhs[2] = mxCreateDoubleMatrix(L, 1, mxREAL);
  double *LLrm = (double *)mxCalloc((size_t)Kb * Kr + 1, sizeof(double));
  double *Zrm = (double *)mxCalloc((size_t)Kb * Kr + 1, sizeof(double));
  vbhem_cluster_t clus = {Kr, S, b.logA, b.logPi, b.m, b.P, b.c};
  const int st = vbhem_ctx_fused(g_ctx, &clus, mxGetPr(tN), mxGetPr(lOm), mxGetPr(plhs[2]), Zrm,
                                 LLrm);
  if (st != VBHEM_OK) {
    mxFree(LLrm);
    mxFree(Zrm);
    free_buffers(&b);
    mexErrMsgIdAndTxt("vbhem_mex:gpu", "vbhem_ctx_fused failed (%d): %s", st, vbhem_last_error());
  }
  double *oLL = mxGetPr(plhs[0]), *oZ = mxGetPr(plhs[1]);
  for (int i = 0; i < Kb; i++)
    for (int j = 0; j < Kr; j++) {
      oLL[(size_t)i + (size_t)j * Kb] = LLrm[(size_t)i * Kr + j];
      oZ[(size_t)i + (size_t)j * Kb] = Zrm[(size_t)i * Kr + j];
    }
  mxFree(LLrm);
  mxFree(Zrm);
  free_buffers(&b);
}

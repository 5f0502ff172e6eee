/*
 * integration/vbhmm_fb_mex.c -- MATLAB MEX gateway that replaces the reference's
 * src/hmm/vbhmm_fb_mex.c with a call into the MI355X VB-HMM forward-backward
 * (libvbhem_estep.so, include/vbhmm_fb.h).
 *
 * Same MATLAB signature, argument checks, error identifiers and output shapes
 * as the reference gateway (vbhmm_fb_mex.c:185-296):
 *
 *   [logrho_Saved, gamma_all, xi_sum, phi_norm] = vbhmm_fb_mex(data, K, N, dim, maxT,
 *        m, W, v, beta, logLambdaTilde, const_denominator, t_pz1, t_tpztzt1)
 *
 *   data {Nx1} of [T_n x dim]; m [dim x K]; W [dim x dim x K]; v, beta [K x 1];
 *   logLambdaTilde, t_pz1 [1 x K]; t_tpztzt1 [K x K] (row format p(j | i));
 *   outputs logrho_Saved, gamma_all [K x N x maxT], xi_sum [K x K x N], phi_norm [1 x N].
 *
 * The gateway repacks MATLAB's column-major inputs into the row-major arrays of
 * vbhmm_seqs_t / vbhmm_params_t, calls vbhmm_fb_host(), and writes the outputs
 * back (logrho / gamma are the same memory order; xi_sum is transposed per
 * sequence).  The GPU device is taken from VBHEM_DEVICE (default 0).
 *
 * Build (MATLAB):  mex -R2017b -I../include vbhmm_fb_mex.c -L../lib -lvbhem_estep
 * (INTEGRATION.md).  Here it is also built against the mx API test double
 * (tests/mxshim) so the gateway itself is tested.
 */
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "vbhmm_fb.h"

/* vbhmm_fb_mex.c:80-85 */
static double fb_scalar(const mxArray *mx) {
  if (!mx || !mxIsDouble(mx) || mxIsComplex(mx))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "arg must be scalar.");
  return mxGetScalar(mx);
}

/* vbhmm_fb_mex.c:89-118: M x N double (0 = any) */
static const double *fb_matrix(const mxArray *mx, int M, int N) {
  if (!mx || !mxIsDouble(mx) || mxIsComplex(mx))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "arg must be double.");
  if (mxGetNumberOfDimensions(mx) != 2)
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "parseMatrix: invalid num dimensions.");
  if ((((int)mxGetM(mx) != M) && (M != 0)) || (((int)mxGetN(mx) != N) && (N != 0)))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "parseMatrix: invalid size.");
  return mxGetPr(mx);
}

/* vbhmm_fb_mex.c:122-149: M x N x D double */
static const double *fb_matrix3(const mxArray *mx, int M, int N, int D) {
  if (!mx || !mxIsDouble(mx) || mxIsComplex(mx))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "arg must be double.");
  const int nd = (int)mxGetNumberOfDimensions(mx);
  if (!(((nd == 3) && (D > 1)) || ((nd == 2) && (D == 1))))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "parseMatrix3: invalid num dimensions.");
  const mwSize *dims = mxGetDimensions(mx);
  if (((int)dims[0] != M) || ((int)dims[1] != N) || ((D > 1) && ((int)dims[2] != D)))
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "parseMatrix3: invalid size.");
  return mxGetPr(mx);
}

static mxArray *create3(int D1, int D2, int D3) {
  mwSize dims[3] = {(mwSize)D1, (mwSize)D2, (mwSize)D3};
  return mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
}

void mexFunction(int nlhs, mxArray *plhs[], int nrhs, const mxArray *prhs[]) {
  if (nrhs != 13) mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nrhs", "13 inputs required.");
  if (nlhs != 4) mexErrMsgIdAndTxt("MyToolbox:arrayProduct:nlhs", "One output required.");
  if (!mxIsCell(prhs[0])) mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "1st arg must be cell");
  const int K = (int)fb_scalar(prhs[1]);
  const int N = (int)fb_scalar(prhs[2]);
  const int dim = (int)fb_scalar(prhs[3]);
  const int maxT = (int)fb_scalar(prhs[4]);
  const double *m = fb_matrix(prhs[5], dim, K);
  const double *W = fb_matrix3(prhs[6], dim, dim, K);
  const double *v = fb_matrix(prhs[7], K, 1);
  const double *beta = fb_matrix(prhs[8], K, 1);
  const double *lLT = fb_matrix(prhs[9], 1, K);
  const double cden = fb_scalar(prhs[10]);
  const double *pz1 = fb_matrix(prhs[11], 1, K);
  const double *Acm = fb_matrix(prhs[12], K, K);
  if (K < 1 || N < 0 || dim < 1 || maxT < 0 || (int)mxGetNumberOfElements(prhs[0]) < N)
    mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "invalid sizes (K=%d N=%d dim=%d maxT=%d)", K,
                      N, dim, maxT);

  /* outputs (vbhmm_fb_mex.c:288-296), zero-initialised */
  plhs[0] = create3(K, N, maxT);
  plhs[1] = create3(K, N, maxT);
  plhs[2] = create3(K, K, N);
  plhs[3] = mxCreateDoubleMatrix(1, (mwSize)N, mxREAL);
  if (N == 0) return;

  /* sequences: data{n} is [T_n x dim] column-major -> x[(off + t) dim + a] */
  int *offsets = (int *)mxMalloc(sizeof(int) * (N + 1));
  offsets[0] = 0;
  for (int n = 0; n < N; n++) {
    const mxArray *c = mxGetCell(prhs[0], n);
    fb_matrix(c, 0, dim);
    const int T = (int)mxGetM(c);
    if (T > maxT) mexErrMsgIdAndTxt("vbhmm_fb_mex:invalidinput", "sequence %d longer than maxT", n + 1);
    offsets[n + 1] = offsets[n] + T;
  }
  double *x = (double *)mxMalloc(sizeof(double) * ((size_t)offsets[N] * dim + 1));
  for (int n = 0; n < N; n++) {
    const mxArray *c = mxGetCell(prhs[0], n);
    const double *pr = mxGetPr(c);
    const int T = offsets[n + 1] - offsets[n];
    for (int t = 0; t < T; t++)
      for (int a = 0; a < dim; a++) x[(size_t)(offsets[n] + t) * dim + a] = pr[t + (size_t)a * T];
  }
  /* W(:,:,k) column-major -> W[k][a][b]; t_tpztzt1 column-major -> A[i][j] */
  double *Wr = (double *)mxMalloc(sizeof(double) * (size_t)K * dim * dim);
  for (int k = 0; k < K; k++)
    for (int a = 0; a < dim; a++)
      for (int b = 0; b < dim; b++)
        Wr[((size_t)k * dim + a) * dim + b] = W[a + (size_t)b * dim + (size_t)k * dim * dim];
  double *A = (double *)mxMalloc(sizeof(double) * (size_t)K * K);
  for (int i = 0; i < K; i++)
    for (int j = 0; j < K; j++) A[i * K + j] = Acm[i + (size_t)j * K];
  double *xi = (double *)mxMalloc(sizeof(double) * (size_t)N * K * K);

  vbhmm_seqs_t s = {N, dim, maxT, offsets, x};
  /* m [dim x K] column-major is m[k][a] row-major: same memory */
  vbhmm_params_t q = {K, dim, m, Wr, v, beta, lLT, pz1, A, cden};
  const char *dev_env = getenv("VBHEM_DEVICE");
  const int rc = vbhmm_fb_host(dev_env ? atoi(dev_env) : 0, &s, &q, mxGetPr(plhs[0]),
                               mxGetPr(plhs[1]), xi, mxGetPr(plhs[3]));
  if (rc != VBHEM_OK) {
    mxFree(offsets); mxFree(x); mxFree(Wr); mxFree(A); mxFree(xi);
    mexErrMsgIdAndTxt("vbhmm_fb_mex:gpu", "vbhmm_fb failed (%d): %s", rc, vbhem_last_error());
  }
  /* xi[n][i][j] -> xi_sum(i, j, n) column-major */
  double *xs = mxGetPr(plhs[2]);
  for (int n = 0; n < N; n++)
    for (int i = 0; i < K; i++)
      for (int j = 0; j < K; j++)
        xs[i + (size_t)j * K + (size_t)n * K * K] = xi[((size_t)n * K + i) * K + j];
  mxFree(offsets); mxFree(x); mxFree(Wr); mxFree(A); mxFree(xi);
}

/*
 * oracle/vbhmm_fb_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64, libm exp/log) of the reference VB-HMM
 * forward-backward MEX
 *     /root/reference/src/hmm/vbhmm_fb_mex.c   (USEPTRS branch, :313-961)
 * called by src/hmm/vbhmm_fb.m:144-145.  Same loop and
 * summation orders as the MEX, so results agree to the last bits up to libm.
 * Only tests/ load it; the product path (libvbhem_estep.so) never does.
 *
 * PARITY UNPINNED (as the VBHEM oracle): no golden vectors ship with the
 * reference and MATLAB is absent; cross-checked against a numpy restatement of
 * the MATLAB path vbhmm_fb.m:227-379 (oracle/vbhem_oracle.py) and closed forms
 * (tests/test_vbhmm_fb.py).
 *
 * Layout (row-major C):
 *   sequences: offsets[N+1], x[offsets[N]][dim] (observation t of sequence n at
 *              x[(offsets[n] + t) * dim + a]); maxT >= every length;
 *   m[K][dim], W[K][dim][dim], v[K], beta[K], logLambdaTilde[K], pz1[K],
 *   A[K][K] (A[i][j] = p(z_t = j | z_{t-1} = i), t_tpztzt1 "row format");
 *   outputs logrho[maxT][N][K] and gamma[maxT][N][K] (the MEX's K x N x maxT
 *   column-major arrays), xi_sum[N][K][K] ([n][i][j], from i to j), phi_norm[N].
 *   Entries for t >= length stay 0, as in the MEX's zero-initialised outputs.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

int oracle_vbhmm_fb(int N, int K, int dim, int maxT, const int *offsets, const double *x,
                    const double *m, const double *W, const double *v, const double *beta,
                    const double *logLambdaTilde, double const_denominator, const double *pz1,
                    const double *A, double *logrho, double *gamma, double *xi_sum,
                    double *phi_norm) {
  const size_t NK = (size_t)N * K;
  double *delta = malloc(sizeof(double) * K * (maxT > 0 ? maxT : 1));
  double *diff = malloc(sizeof(double) * dim);
  double *diff2 = malloc(sizeof(double) * dim);
  double *alpha = malloc(sizeof(double) * K * (maxT > 0 ? maxT : 1));   /* [t][k] */
  double *Delta = malloc(sizeof(double) * K);
  double *bet = malloc(sizeof(double) * K * (maxT > 0 ? maxT : 1));     /* [t][k] */
  double *c = malloc(sizeof(double) * (maxT > 0 ? maxT : 1));
  double *px = malloc(sizeof(double) * K * (maxT > 0 ? maxT : 1));      /* [t][k] */
  double *bpi = malloc(sizeof(double) * K);
  double *mx = malloc(sizeof(double) * (maxT > 0 ? maxT : 1));
  if (!delta || !diff || !diff2 || !alpha || !Delta || !bet || !c || !px || !bpi || !mx) return -1;
  memset(logrho, 0, sizeof(double) * NK * maxT);
  memset(gamma, 0, sizeof(double) * NK * maxT);
  memset(xi_sum, 0, sizeof(double) * N * K * K);
  memset(phi_norm, 0, sizeof(double) * N);
  for (int n = 0; n < N; n++) {
    const int tT = offsets[n + 1] - offsets[n];
    const double *xn = x + (size_t)offsets[n] * dim;
    /* delta(k,t) = dim/beta(k) + v(k) (x_t - m_k)' W_k (x_t - m_k)   mex.c:334-432 */
    for (int k = 0; k < K; k++) {
      for (int t = 0; t < tT; t++) {
        for (int a = 0; a < dim; a++) diff[a] = xn[t * dim + a] - m[k * dim + a];
        for (int a = 0; a < dim; a++) {   /* row a of W'diff (W(:,a,k) . diff, :371-383) */
          double tmp = 0.0;
          for (int b = 0; b < dim; b++) tmp += W[((size_t)k * dim + b) * dim + a] * diff[b];
          diff2[a] = tmp;
        }
        for (int a = 0; a < dim; a++) diff2[a] *= diff[a];
        double tmp = 0.0;
        for (int a = 0; a < dim; a++) tmp += diff2[a];
        delta[t * K + k] = dim / beta[k] + v[k] * tmp;
      }
    }
    /* logrho = 0.5 (logLambdaTilde - delta) - const_denominator        :438-453 */
    for (int t = 0; t < tT; t++)
      for (int k = 0; k < K; k++)
        logrho[(size_t)t * NK + (size_t)n * K + k] =
            0.5 * (logLambdaTilde[k] - delta[t * K + k]) - const_denominator;
    /* p(x_t|z_t) / max_k                                                  :501-533 */
    for (int t = 0; t < tT; t++) {
      const double *lr = logrho + (size_t)t * NK + (size_t)n * K;
      double tmp = lr[0];
      for (int k = 1; k < K; k++)
        if (lr[k] > tmp) tmp = lr[k];
      mx[t] = tmp;
      for (int k = 0; k < K; k++) px[t * K + k] = exp(lr[k] - tmp);
    }
    if (tT < 1) continue;
    /* forward, scaled                                                     :560-694 */
    for (int k = 0; k < K; k++) Delta[k] = pz1[k] * px[k];
    {
      double tmp = 0.0;
      for (int k = 0; k < K; k++) tmp += Delta[k];
      c[0] = tmp;
    }
    for (int k = 0; k < K; k++) alpha[k] = Delta[k] / c[0];
    for (int t = 1; t < tT; t++) {
      for (int j = 0; j < K; j++) {
        double tmp = 0.0;
        for (int i = 0; i < K; i++) tmp += alpha[(t - 1) * K + i] * A[i * K + j];
        Delta[j] = tmp * px[t * K + j];
      }
      double tmp = 0.0;
      for (int k = 0; k < K; k++) tmp += Delta[k];
      c[t] = tmp;
      for (int k = 0; k < K; k++) alpha[t * K + k] = Delta[k] / c[t];
    }
    /* backward                                                            :703-884 */
    double *gn = gamma + (size_t)n * K;
    double *xs = xi_sum + (size_t)n * K * K;
    for (int k = 0; k < K; k++) bet[(tT - 1) * K + k] = 1.0;
    for (int k = 0; k < K; k++)
      gn[(size_t)(tT - 1) * NK + k] = alpha[(tT - 1) * K + k] * bet[(tT - 1) * K + k];
    for (int t = tT - 2; t >= 0; t--) {
      for (int k = 0; k < K; k++) bpi[k] = bet[(t + 1) * K + k] * px[(t + 1) * K + k];
      for (int i = 0; i < K; i++) {
        double tmp = 0.0;
        for (int j = 0; j < K; j++) tmp += bpi[j] * A[i * K + j];
        bet[t * K + i] = tmp / c[t + 1];
      }
      for (int k = 0; k < K; k++) gn[(size_t)t * NK + k] = alpha[t * K + k] * bet[t * K + k];
      for (int j = 0; j < K; j++)
        for (int i = 0; i < K; i++)
          xs[i * K + j] += A[i * K + j] * alpha[t * K + i] * bpi[j] / c[t + 1];
    }
    /* phi_norm = sum(log(c)) + sum(max)  (accumulated per t)             :939-951 */
    {
      double tmp = 0.0;
      for (int t = 0; t < tT; t++) tmp += log(c[t]) + mx[t];
      phi_norm[n] = tmp;
    }
  }
  free(delta); free(diff); free(diff2); free(alpha); free(Delta); free(bet); free(c);
  free(px); free(bpi); free(mx);
  return 0;
}

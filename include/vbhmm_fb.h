/*
 * vbhmm_fb.h -- C-ABI of the VB-HMM forward-backward E-step on MI355X
 * (SURVEY.md 8f rank 3): the computation of the reference MEX
 *     src/hmm/vbhmm_fb_mex.c:185-984
 *   [logrho_Saved, gamma_all, xi_sum, phi_norm] = vbhmm_fb_mex(data, K, N, dim, maxT,
 *        m, W, v, beta, logLambdaTilde, const_denominator, t_pz1, t_tpztzt1)
 * called by src/hmm/vbhmm_fb.m:144-145 (and :169-170 per group) inside vbhmm_em.m,
 * which learns the base HMMs that VBHEM clusters.  One lane per sequence; the
 * scaled forward-backward of vbhmm_fb_mex.c:547-956 in fp64.
 *
 * Layouts (row-major, plain pointers; status codes of vbhem_estep.h):
 *   sequences: offsets[N+1] (int), x[offsets[N]][dim] -- observation t of
 *              sequence n at x[(offsets[n] + t) * dim + a] (data{n} rows);
 *   params:    m[K][dim], W[K][dim][dim], v[K], beta[K], logLambdaTilde[K],
 *              pz1[K] = exp(logPiTilde), A[K][K] = exp(logATilde) (A[i][j] = p(j | i));
 *   outputs:   logrho[maxT][N][K], gamma[maxT][N][K] (the MEX's K x N x maxT
 *              column-major arrays; entries t >= length are 0), xi_sum[N][K][K]
 *              ([n][from][to]; the MEX's K x K x N holds the transpose per n),
 *              phi_norm[N].
 * Limits: 1 <= K <= 16, 1 <= dim <= 8 (else VBHEM_ERR_UNSUPPORTED).
 */
#ifndef VBHMM_FB_H
#define VBHMM_FB_H

#include <stddef.h>

#include "vbhem_estep.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int N, dim, maxT;
  const int *offsets;  /* [N+1] */
  const double *x;     /* [offsets[N]][dim] */
} vbhmm_seqs_t;

typedef struct {
  int K, dim;
  const double *m, *W, *v, *beta, *logLambdaTilde, *pz1, *A;
  double const_denominator; /* dim * log(2 pi) / 2 (vbhmm_fb.m:61) */
} vbhmm_params_t;

/* Device pointers; the outputs are fully written (zeros past each length).
 * workspace: vbhmm_fb_workspace_bytes (scaling constants + per-step maxima). */
size_t vbhmm_fb_workspace_bytes(const vbhmm_seqs_t *seqs, int K);
int vbhmm_fb(const vbhmm_seqs_t *seqs_dev, const vbhmm_params_t *params_dev, double *logrho_dev,
             double *gamma_dev, double *xi_sum_dev, double *phi_norm_dev, void *workspace_dev,
             size_t workspace_bytes, void *stream);
/* Host pointers: copies in, runs on `device`, copies out (the MEX gateway's call). */
int vbhmm_fb_host(int device, const vbhmm_seqs_t *seqs_host, const vbhmm_params_t *params_host,
                  double *logrho, double *gamma, double *xi_sum, double *phi_norm);

#ifdef __cplusplus
}
#endif
#endif /* VBHMM_FB_H */

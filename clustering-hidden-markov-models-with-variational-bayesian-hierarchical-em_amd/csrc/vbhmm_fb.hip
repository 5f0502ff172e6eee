// vbhmm_fb.hip -- the VB-HMM forward-backward E-step:
// the computation of src/hmm/vbhmm_fb_mex.c:313-961 for every sequence of a
// batch, one lane per sequence (include/vbhmm_fb.h).
//
// Per sequence n (length T, K states, dim-dimensional observations):
//   delta(k,t)  = dim/beta_k + v_k (x_t - m_k)' W_k (x_t - m_k)        mex.c:334-432
//   logrho(k,t) = (logLambdaTilde_k - delta(k,t)) / 2 - const_denominator  :438-453
//   p(k,t)      = exp(logrho(k,t) - max_k logrho(., t))                :501-533
//   scaled forward  alpha_t = (alpha_{t-1} A) .* p_t / c_t            :560-694
//   scaled backward beta_t = (A (beta_{t+1} .* p_{t+1})) / c_{t+1}, gamma = alpha .* beta,
//                   xi_sum += A .* (alpha_t' (beta_{t+1} .* p_{t+1})) / c_{t+1}  :703-884
//   phi_norm    = sum_t (log c_t + max_t)                             :939-951
// in the MEX's operation and summation order.  The cluster parameters (shared by
// all lanes) are staged in LDS; the forward sweep keeps alpha in registers and
// parks it in the gamma output, the backward sweep turns it into gamma in place;
// c_t and max_t go to a [maxT][N] scratch pair.  Memory: the [t][n][k] outputs
// are written by consecutive lanes at the same t, so a wavefront's stores are
// contiguous runs of K doubles per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "vbhem_estep.h"
#include "vbhem_internal.h"
#include "vbhmm_fb.h"

namespace vbhem {
namespace {

constexpr int kFbmThreads = 128;
constexpr int kFbmMaxDim = 8;

struct FbmArgs {
  int N, K, dim, maxT;
  const int *offsets;
  const double *x, *m, *W, *v, *beta, *lLT, *pz1, *A;
  double cden;
  double *logrho, *gamma, *xi, *phi;
  double *cs, *mxs;  // scratch [maxT][N]: c_t, max_t
};

template <int KM>
__global__ __launch_bounds__(kFbmThreads) void vbhmm_fb_kernel(const FbmArgs p) {
  __shared__ double sA[KM * KM], sm[KM * kFbmMaxDim], sW[KM * kFbmMaxDim * kFbmMaxDim];
  __shared__ double sdb[KM], sv[KM], sll[KM], spz[KM];
  const int K = p.K, dim = p.dim;
  for (int x = threadIdx.x; x < K * K; x += kFbmThreads) sA[x] = p.A[x];
  for (int x = threadIdx.x; x < K * dim; x += kFbmThreads) sm[x] = p.m[x];
  for (int x = threadIdx.x; x < K * dim * dim; x += kFbmThreads) sW[x] = p.W[x];
  for (int k = threadIdx.x; k < K; k += kFbmThreads) {
    sdb[k] = dim / p.beta[k];
    sv[k] = p.v[k];
    sll[k] = p.lLT[k];
    spz[k] = p.pz1[k];
  }
  __syncthreads();
  const int n = blockIdx.x * kFbmThreads + threadIdx.x;
  if (n >= p.N) return;
  const size_t NK = (size_t)p.N * K;
  const int T = p.offsets[n + 1] - p.offsets[n];
  const double *xn = p.x + (size_t)p.offsets[n] * dim;
  double *xs = p.xi + (size_t)n * K * K;
  for (int q = 0; q < K * K; ++q) xs[q] = 0.0;
  // zeros past the end of the sequence (the MEX's zero-initialised outputs)
  for (int t = T; t < p.maxT; ++t)
    for (int k = 0; k < K; ++k) {
      p.logrho[(size_t)t * NK + (size_t)n * K + k] = 0.0;
      p.gamma[(size_t)t * NK + (size_t)n * K + k] = 0.0;
    }
  if (T < 1) {
    p.phi[n] = 0.0;
    return;
  }
  double al[KM], px[KM];
  double phi = 0.0;
  // ---- emission log-likelihoods + scaled forward sweep ----
  for (int t = 0; t < T; ++t) {
    double lr[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k < K) {
        double diff[kFbmMaxDim], tmp = 0.0;
        for (int a = 0; a < dim; ++a) diff[a] = xn[t * dim + a] - sm[k * dim + a];
        for (int a = 0; a < dim; ++a) {
          double w = 0.0;  // (W(:,a,k) . diff), mex.c:371-383
          for (int b = 0; b < dim; ++b) w += sW[(k * dim + b) * dim + a] * diff[b];
          w *= diff[a];
          tmp += w;
        }
        const double delta = sdb[k] + sv[k] * tmp;
        lr[k] = 0.5 * (sll[k] - delta) - p.cden;
        p.logrho[(size_t)t * NK + (size_t)n * K + k] = lr[k];
      }
    }
    double mx = lr[0];
#pragma unroll
    for (int k = 1; k < KM; ++k)
      if (k < K && lr[k] > mx) mx = lr[k];
#pragma unroll
    for (int k = 0; k < KM; ++k) px[k] = k < K ? exp(lr[k] - mx) : 0.0;
    double D[KM];
    if (t == 0) {
#pragma unroll
      for (int k = 0; k < KM; ++k) D[k] = k < K ? spz[k] * px[k] : 0.0;
    } else {
#pragma unroll
      for (int j = 0; j < KM; ++j) {
        double tmp = 0.0;
#pragma unroll
        for (int i = 0; i < KM; ++i)
          if (i < K && j < K) tmp += al[i] * sA[i * K + j];
        D[j] = tmp * px[j];
      }
    }
    double c = 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) c += k < K ? D[k] : 0.0;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      al[k] = k < K ? D[k] / c : 0.0;
      if (k < K) p.gamma[(size_t)t * NK + (size_t)n * K + k] = al[k];  // alpha_t, parked
    }
    p.cs[(size_t)t * p.N + n] = c;
    p.mxs[(size_t)t * p.N + n] = mx;
    phi += log(c) + mx;
  }
  p.phi[n] = phi;
  // ---- scaled backward sweep: gamma = alpha .* beta, xi_sum ----
  double be[KM];
#pragma unroll
  for (int k = 0; k < KM; ++k) be[k] = 1.0;  // gamma(T-1) = alpha(T-1) .* 1: already in place
  for (int t = T - 2; t >= 0; --t) {
    const double c1 = p.cs[(size_t)(t + 1) * p.N + n];
    const double mx1 = p.mxs[(size_t)(t + 1) * p.N + n];
    double bpi[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k)
      bpi[k] = k < K ? be[k] * exp(p.logrho[(size_t)(t + 1) * NK + (size_t)n * K + k] - mx1) : 0.0;
#pragma unroll
    for (int i = 0; i < KM; ++i) {
      double tmp = 0.0;
#pragma unroll
      for (int j = 0; j < KM; ++j)
        if (i < K && j < K) tmp += bpi[j] * sA[i * K + j];
      be[i] = i < K ? tmp / c1 : 0.0;
    }
    double *g = p.gamma + (size_t)t * NK + (size_t)n * K;
    double a[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      a[k] = k < K ? g[k] : 0.0;
      if (k < K) g[k] = a[k] * be[k];
    }
#pragma unroll
    for (int j = 0; j < KM; ++j)
#pragma unroll
      for (int i = 0; i < KM; ++i)
        if (i < K && j < K) xs[i * K + j] += sA[i * K + j] * a[i] * bpi[j] / c1;
  }
}

template <int KM>
hipError_t launch_fbm(const FbmArgs &a, hipStream_t st) {
  const unsigned grid = (unsigned)((a.N + kFbmThreads - 1) / kFbmThreads);
  hipLaunchKernelGGL(vbhmm_fb_kernel<KM>, dim3(grid), dim3(kFbmThreads), 0, st, a);
  return hipGetLastError();
}

int check_fbm(const vbhmm_seqs_t *s, const vbhmm_params_t *q, bool need_ptrs) {
  if (!s || !q) return set_error(VBHEM_ERR_ARG, "null sequences or parameters");
  if (s->N < 0 || s->dim < 1 || s->maxT < 0 || q->K < 1 || q->dim != s->dim)
    return set_error(VBHEM_ERR_ARG, "invalid sizes (need N>=0, dim>=1, maxT>=0, K>=1, equal dim)");
  if (q->K > 16 || s->dim > kFbmMaxDim)
    return set_error(VBHEM_ERR_UNSUPPORTED, "vbhmm_fb: K <= 16 and dim <= 8 supported");
  if (need_ptrs && s->N > 0 &&
      (!s->offsets || !s->x || !q->m || !q->W || !q->v || !q->beta || !q->logLambdaTilde ||
       !q->pz1 || !q->A))
    return set_error(VBHEM_ERR_ARG, "null input array");
  return VBHEM_OK;
}

}  // namespace
}  // namespace vbhem

extern "C" {

size_t vbhmm_fb_workspace_bytes(const vbhmm_seqs_t *s, int K) {
  if (!s || s->N < 0 || s->maxT < 0 || K < 1) return 0;
  return std::max<size_t>(256, (size_t)2 * s->maxT * s->N * sizeof(double) + 256);
}

int vbhmm_fb(const vbhmm_seqs_t *s, const vbhmm_params_t *q, double *logrho_dev, double *gamma_dev,
             double *xi_sum_dev, double *phi_norm_dev, void *workspace_dev, size_t workspace_bytes,
             void *stream) {
  using namespace vbhem;
  int rc = check_fbm(s, q, true);
  if (rc != VBHEM_OK) return rc;
  if (s->N == 0) return VBHEM_OK;
  if (!logrho_dev || !gamma_dev || !xi_sum_dev || !phi_norm_dev)
    return set_error(VBHEM_ERR_ARG, "null output array");
  const size_t need = vbhmm_fb_workspace_bytes(s, q->K);
  if (!workspace_dev || workspace_bytes < need)
    return set_error(VBHEM_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  FbmArgs a{};
  a.N = s->N; a.K = q->K; a.dim = s->dim; a.maxT = s->maxT;
  a.offsets = s->offsets; a.x = s->x;
  a.m = q->m; a.W = q->W; a.v = q->v; a.beta = q->beta; a.lLT = q->logLambdaTilde;
  a.pz1 = q->pz1; a.A = q->A; a.cden = q->const_denominator;
  a.logrho = logrho_dev; a.gamma = gamma_dev; a.xi = xi_sum_dev; a.phi = phi_norm_dev;
  a.cs = static_cast<double *>(workspace_dev);
  a.mxs = a.cs + (size_t)s->maxT * s->N;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = q->K <= 4 ? launch_fbm<4>(a, st) : q->K <= 8 ? launch_fbm<8>(a, st)
                                                             : launch_fbm<16>(a, st);
  if (e != hipSuccess) return set_error(VBHEM_ERR_HIP, std::string("vbhmm_fb_kernel: ") + hipGetErrorString(e));
  return VBHEM_OK;
}

int vbhmm_fb_host(int device, const vbhmm_seqs_t *sh, const vbhmm_params_t *qh, double *logrho,
                  double *gamma, double *xi_sum, double *phi_norm) {
  using namespace vbhem;
  int rc = check_fbm(sh, qh, true);
  if (rc != VBHEM_OK) return rc;
  if (sh->N == 0) return VBHEM_OK;
  if (sh->offsets[0] != 0) return set_error(VBHEM_ERR_ARG, "offsets[0] must be 0");
  for (int n = 0; n < sh->N; ++n) {
    const int len = sh->offsets[n + 1] - sh->offsets[n];
    if (len < 0 || len > sh->maxT)
      return set_error(VBHEM_ERR_ARG, "sequence lengths must be in [0, maxT]");
  }
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return set_error(VBHEM_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  const size_t N = sh->N, K = qh->K, dim = sh->dim, T = sh->maxT, nx = (size_t)sh->offsets[N];
  const size_t n_in[] = {nx * dim, K * dim, K * dim * dim, K, K, K, K, K * K};
  const double *h_in[] = {sh->x, qh->m, qh->W, qh->v, qh->beta, qh->logLambdaTilde, qh->pz1, qh->A};
  const size_t n_out[] = {T * N * K, T * N * K, N * K * K, N};
  double *h_out[] = {logrho, gamma, xi_sum, phi_norm};
  double *d_in[8] = {nullptr}, *d_out[4] = {nullptr};
  int *d_off = nullptr;
  void *ws = nullptr;
  const size_t wsb = vbhmm_fb_workspace_bytes(sh, qh->K);
  rc = VBHEM_OK;
  auto hf = [&rc](hipError_t err, const char *where) {
    if (err != hipSuccess && rc == VBHEM_OK)
      rc = set_error(VBHEM_ERR_HIP, std::string(where) + ": " + hipGetErrorString(err));
  };
  for (int k = 0; k < 8 && rc == VBHEM_OK; ++k) {
    hf(hipMalloc(&d_in[k], std::max<size_t>(1, n_in[k]) * sizeof(double)), "hipMalloc(in)");
    if (rc == VBHEM_OK && n_in[k])
      hf(hipMemcpy(d_in[k], h_in[k], n_in[k] * sizeof(double), hipMemcpyHostToDevice), "upload");
  }
  for (int k = 0; k < 4 && rc == VBHEM_OK; ++k)
    hf(hipMalloc(&d_out[k], std::max<size_t>(1, n_out[k]) * sizeof(double)), "hipMalloc(out)");
  if (rc == VBHEM_OK) hf(hipMalloc(&d_off, (N + 1) * sizeof(int)), "hipMalloc(offsets)");
  if (rc == VBHEM_OK)
    hf(hipMemcpy(d_off, sh->offsets, (N + 1) * sizeof(int), hipMemcpyHostToDevice), "upload");
  if (rc == VBHEM_OK) hf(hipMalloc(&ws, wsb), "hipMalloc(workspace)");
  if (rc == VBHEM_OK) {
    vbhmm_seqs_t sd = *sh;
    sd.offsets = d_off; sd.x = d_in[0];
    vbhmm_params_t qd = *qh;
    qd.m = d_in[1]; qd.W = d_in[2]; qd.v = d_in[3]; qd.beta = d_in[4];
    qd.logLambdaTilde = d_in[5]; qd.pz1 = d_in[6]; qd.A = d_in[7];
    rc = vbhmm_fb(&sd, &qd, d_out[0], d_out[1], d_out[2], d_out[3], ws, wsb, nullptr);
  }
  if (rc == VBHEM_OK) hf(hipDeviceSynchronize(), "kernel execution");
  for (int k = 0; k < 4 && rc == VBHEM_OK; ++k)
    if (n_out[k]) hf(hipMemcpy(h_out[k], d_out[k], n_out[k] * sizeof(double), hipMemcpyDeviceToHost), "download");
  for (auto *ptr : d_in) (void)hipFree(ptr);
  for (auto *ptr : d_out) (void)hipFree(ptr);
  (void)hipFree(d_off);
  (void)hipFree(ws);
  return rc;
}

}  // extern "C"

// vbhem_h3m.hip -- hmms_to_h3m_hem.m:42-140 on the device (include/vbhem_estep.h,
// vbhem_hmms_to_h3m): the N learned VB-HMMs, packed and zero-padded to SB states,
// into the base set h3m_b the E-step consumes.  One thread per (base, state) row:
//   use_post = 1 (vbhem_h3m_cluster.m:237, the default):
//     prior(s)  = exp(psi(alpha_s) - psi(sum alpha))                  (:46-50)
//     A(s, t)   = exp(psi(epsilon_st) - psi(sum_t epsilon_st))        (:52-58)
//     covars(s) = cov_s (beta_s + 1) / beta_s                         (:82, 88)
//   use_post = 0: prior, A and covars as given;
//   diag mode: the covariances' diagonals (:86-89);
//   an empty entry (nstates 0): a one-state dummy HMM (prior 1, A 1, unit covariance)
//   with weight 0 (:113-133); every other base weight 1 / (number of non-empty).
// Sub-stochastic prior / A are never renormalised.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vbhem_estep.h"
#include "vbhem_internal.h"

namespace vbhem {
namespace {

// digamma for x > 0: recurrence to x >= 8, then ln x - 1/(2x) - sum B_2k / (2k x^2k)
// (the host loop's psi, vbhem_em.hip)
__device__ double psi_dev(double x) {
  if (!(x > 0.0 && x < INFINITY)) return x == INFINITY ? x : __builtin_nan("");
  double acc = 0.0;
  while (x < 8.0) {
    acc -= 1.0 / x;
    x += 1.0;
  }
  const double r = 1.0 / x, r2 = r * r;
  const double series =
      r2 * (1.0 / 12 - r2 * (1.0 / 120 - r2 * (1.0 / 252 - r2 * (1.0 / 240 - r2 * (1.0 / 132 -
      r2 * (691.0 / 32760 - r2 * (1.0 / 12)))))));
  return acc + log(x) - 0.5 * r - series;
}

struct H3mArgs {
  int N, SB, d, covmode, use_post;
  const int *nstates;
  const double *alpha, *epsilon, *beta, *prior_in, *trans_in, *centres_in, *covars_in;
  double *prior, *A, *centres, *covars, *omega;
  int *count;  // [1]: the number of non-empty entries
};

constexpr int kH3mThreads = 256;

// count of non-empty entries: one block, fixed-order tree (bit-reproducible)
__global__ __launch_bounds__(kH3mThreads) void h3m_count_kernel(H3mArgs p) {
  __shared__ int part[kH3mThreads];
  int n = 0;
  for (int i = threadIdx.x; i < p.N; i += kH3mThreads) n += p.nstates[i] > 0;
  part[threadIdx.x] = n;
  __syncthreads();
  for (int o = kH3mThreads / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) p.count[0] = part[0];
}

__global__ __launch_bounds__(kH3mThreads) void hmms_to_h3m_kernel(H3mArgs p) {
  const long long row = (long long)blockIdx.x * kH3mThreads + threadIdx.x;
  if (row >= (long long)p.N * p.SB) return;
  const int i = (int)(row / p.SB), s = (int)(row - (long long)i * p.SB);
  const int SB = p.SB, d = p.d;
  const bool full = p.covmode == kCovFull;
  const int ns = p.nstates[i];
  const size_t is = (size_t)i * SB + s;
  double *Ar = p.A + is * SB, *cen = p.centres + is * d;
  double *cov = p.covars + is * (full ? (size_t)d * d : (size_t)d);
  const double *cin = p.covars_in + is * (size_t)d * d;
  if (s == 0) {
    const int cnt = p.count[0];
    p.omega[i] = ns > 0 ? 1.0 / (double)cnt : 0.0;
  }
  if (ns <= 0 || s >= ns) {
    // padding rows (and the empty entry's dummy state 0): zero, except the dummy
    const bool dummy = ns <= 0 && s == 0;
    p.prior[is] = dummy ? 1.0 : 0.0;
    for (int t = 0; t < SB; ++t) Ar[t] = dummy && t == 0 ? 1.0 : 0.0;
    for (int a = 0; a < d; ++a) cen[a] = 0.0;
    if (full) {
      for (int a = 0; a < d; ++a)
        for (int b2 = 0; b2 < d; ++b2) cov[a * d + b2] = dummy && a == b2 ? 1.0 : 0.0;
    } else {
      for (int a = 0; a < d; ++a) cov[a] = dummy ? 1.0 : 0.0;
    }
    return;
  }
  double infl = 1.0;
  if (p.use_post) {
    const double *al = p.alpha + (size_t)i * SB, *ep = p.epsilon + is * SB;
    double sa = 0.0, se = 0.0;
    for (int t = 0; t < ns; ++t) {
      sa += al[t];
      se += ep[t];
    }
    p.prior[is] = exp(psi_dev(al[s]) - psi_dev(sa));
    const double pse = psi_dev(se);
    for (int t = 0; t < SB; ++t) Ar[t] = t < ns ? exp(psi_dev(ep[t]) - pse) : 0.0;
    const double be = p.beta[is];
    infl = (be + 1.0) / be;
  } else {
    p.prior[is] = p.prior_in[is];
    const double *tr = p.trans_in + is * SB;
    for (int t = 0; t < SB; ++t) Ar[t] = t < ns ? tr[t] : 0.0;
  }
  for (int a = 0; a < d; ++a) cen[a] = p.centres_in[is * d + a];
  if (full) {
    for (int a = 0; a < d * d; ++a) cov[a] = infl * cin[a];
  } else {
    for (int a = 0; a < d; ++a) cov[a] = infl * cin[a * d + a];
  }
}

}  // namespace
}  // namespace vbhem

extern "C" int vbhem_hmms_to_h3m(int N, int SB, int d, int covmode, int use_post, const int *nstates,
                                 const double *alpha, const double *epsilon, const double *beta,
                                 const double *prior_in, const double *trans_in,
                                 const double *centres_in, const double *covars_in, double *prior,
                                 double *A, double *centres, double *covars, double *omega,
                                 void *workspace, void *stream) {
  using namespace vbhem;
  if (N < 1 || SB < 1 || d < 1 || (covmode != VBHEM_COV_DIAG && covmode != VBHEM_COV_FULL) ||
      !nstates || !centres_in || !covars_in || !prior || !A || !centres || !covars || !omega ||
      !workspace || (use_post && (!alpha || !epsilon || !beta)) || (!use_post && (!prior_in || !trans_in)))
    return set_error(VBHEM_ERR_ARG, "vbhem_hmms_to_h3m: bad arguments");
  H3mArgs a{N, SB, d, covmode, use_post, nstates, alpha, epsilon, beta, prior_in, trans_in,
            centres_in, covars_in, prior, A, centres, covars, omega, static_cast<int *>(workspace)};
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(h3m_count_kernel, dim3(1), dim3(kH3mThreads), 0, st, a);
  const long long rows = (long long)N * SB;
  hipLaunchKernelGGL(hmms_to_h3m_kernel, dim3((unsigned)((rows + kH3mThreads - 1) / kH3mThreads)),
                     dim3(kH3mThreads), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? VBHEM_OK : set_error(VBHEM_ERR_HIP, hipGetErrorString(e));
}

// vbhem_em_dev.hip -- the per-iteration host math of the EM loop, on the device.
//
// vbhem_h3m_c_step_fc.m runs, between two E-steps, the lower bound (vbhemh3m_lb.m:
// 64-186), the M-step (vbhem_compute_Statistics.m:57-82, vbhem_mstep_component.m:
// 42-70, :396) and the next iteration's psi prelude (:118-165, 180-191, 271-273).
// vbhem_em.hip has them in C++ on the host; here the same arithmetic runs as two
// small kernels on the E-step's stream, so an EM iteration never leaves the GPU:
// the packed statistics are read where the statistics kernel (and the all-reduce)
// left them, and the prelude writes the next E-step's cluster constants in place.
// Only the bound (one double) goes to the host, for the convergence test.
//
//   em_step_kernel<DP>   one block per cluster k, one thread per state s:
//                        [M-step of (k, s)] + prelude of (k, s) (logLambdaTilde, c,
//                        P = v W, m, the logATilde row), logPiTilde and logOmega
//   em_bound_kernel<DP>  one block: every (k, s) term of the bound, reduced in a
//                        fixed order (deterministic), written to host memory
//
// d x d determinants and inverses use LU with partial pivoting (as MATLAB's
// det / inv and vbhem_em.hip) on register arrays padded to DP in {2, 4, 8, 16} with
// an identity block (exact: the padding neither changes the determinant nor the
// inverse of the leading block, and never wins a pivot search).  psi is the host
// routine's recurrence + asymptotic series; lgamma is the device libm's.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vbhem_em_dev.h"

namespace vbhem {

namespace {

constexpr double kPiD = 3.14159265358979323846;
constexpr double kLn2D = 0.69314718055994530942;

__device__ double psi_dev(double x) {
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

// sum_{q=1..d} psi((v + 1 - q) / 2): two chains, psi(x - 1) = psi(x) - 1/(x - 1)
__device__ double psi_sum_half_dev(double v, int d) {
  double acc = 0.0;
  for (int c = 0; c < 2 && c < d; ++c) {
    double x = 0.5 * (v - c), p = psi_dev(x);
    for (int q = c; q < d; q += 2) {
      acc += p;
      x -= 1.0;
      p -= 1.0 / x;
    }
  }
  return acc;
}

// sum_{q=1..d} lgamma((v + 1 - q) / 2): two chains, lgamma(x - 1) = lgamma(x) - log(x - 1)
__device__ double lgamma_sum_half_dev(double v, int d) {
  double acc = 0.0;
  for (int c = 0; c < 2 && c < d; ++c) {
    double x = 0.5 * (v - c), g = lgamma(x);
    for (int q = c; q < d; q += 2) {
      acc += g;
      x -= 1.0;
      if (q + 2 < d) g -= log(x);
    }
  }
  return acc;
}

// LU with partial pivoting in registers (compile-time indices, row swaps as
// selects); returns det.  a is overwritten by the factors, perm[k] = pivot row.
template <int DP>
__device__ __forceinline__ double lu_reg(double (&a)[DP][DP], int (&perm)[DP]) {
  double det = 1.0;
#pragma unroll
  for (int k = 0; k < DP; ++k) {
    int p = k;
    double best = fabs(a[k][k]);
#pragma unroll
    for (int r = k + 1; r < DP; ++r)
      if (fabs(a[r][k]) > best) {
        best = fabs(a[r][k]);
        p = r;
      }
    perm[k] = p;
    if (p != k) det = -det;
#pragma unroll
    for (int r = k + 1; r < DP; ++r) {
      const bool sw = r == p;
#pragma unroll
      for (int c = 0; c < DP; ++c) {
        const double t = a[k][c];
        a[k][c] = sw ? a[r][c] : t;
        a[r][c] = sw ? t : a[r][c];
      }
    }
    const double pk = a[k][k];
    det *= pk;
    if (pk != 0.0) {
#pragma unroll
      for (int r = k + 1; r < DP; ++r) {
        const double f = a[r][k] / pk;
        a[r][k] = f;
#pragma unroll
        for (int c = k + 1; c < DP; ++c) a[r][c] -= f * a[k][c];
      }
    }
  }
  return det;
}

// d x d (row-major, stride d) -> DP x DP registers, identity padding
template <int DP>
__device__ __forceinline__ void load_pad(double (&a)[DP][DP], const double *m, int d) {
#pragma unroll
  for (int r = 0; r < DP; ++r)
#pragma unroll
    for (int c = 0; c < DP; ++c)
      a[r][c] = (r < d && c < d) ? m[r * d + c] : (r == c ? 1.0 : 0.0);
}

template <int DP>
__device__ double det_pad(const double *m, int d) {
  double a[DP][DP];
  int perm[DP];
  load_pad<DP>(a, m, d);
  return lu_reg<DP>(a, perm);
}

// inverse of the padded matrix in registers (a overwritten), columns solved in turn
template <int DP>
__device__ __forceinline__ void inv_reg(double (&a)[DP][DP], double (&out)[DP][DP]) {
  int perm[DP];
  lu_reg<DP>(a, perm);
#pragma unroll
  for (int col = 0; col < DP; ++col) {
    double x[DP];
#pragma unroll
    for (int r = 0; r < DP; ++r) x[r] = r == col ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < DP; ++k) {
#pragma unroll
      for (int r = k + 1; r < DP; ++r) {
        const bool sw = r == perm[k];
        const double t = x[k];
        x[k] = sw ? x[r] : t;
        x[r] = sw ? t : x[r];
      }
    }
#pragma unroll
    for (int r = 0; r < DP; ++r)
#pragma unroll
      for (int c = 0; c < r; ++c) x[r] -= a[r][c] * x[c];
#pragma unroll
    for (int r = DP - 1; r >= 0; --r) {
#pragma unroll
      for (int c = r + 1; c < DP; ++c) x[r] -= a[r][c] * x[c];
      x[r] /= a[r][r];
    }
#pragma unroll
    for (int r = 0; r < DP; ++r) out[r][col] = x[r];
  }
}

// packed statistics (include/vbhem_estep.h): Nj | N1 | M | Lt1 Lt7 | U
struct StatsView {
  const double *Nj, *N1, *M, *U;
  double Lt1, Lt7;
  __device__ StatsView(const double *v, int K, int S, int NU) {
    size_t o = 0;
    Nj = v + o; o += K;
    N1 = v + o; o += (size_t)K * S;
    M = v + o; o += (size_t)K * S * S;
    Lt1 = v[o];
    Lt7 = v[o + 1];
    o += 2;
    U = v + o;
    (void)NU;
  }
};

constexpr int kStepThreads = 64;   // >= S (S <= 64 on this path)
constexpr int kBoundThreads = 256;

template <int DP>
__global__ __launch_bounds__(kStepThreads) void em_step_kernel(const EmDevArgs a, int do_mstep) {
  __shared__ double red[kStepThreads];
  const int k = blockIdx.x, s = threadIdx.x;
  const int K = a.K, S = a.S, d = a.d;
  const bool full = a.covmode == 1;
  const int dd = full ? d * d : d;
  const size_t ks = (size_t)k * S + s;
  const bool on = s < S;
  double eta_ks = 0.0, alpha_k = 0.0;
  double sumA = 0.0;  // sum_k alpha (thread 0)
  if (do_mstep) {
    const StatsView st(a.stats, K, S, a.NU);
    if (on) {
      // vbhem_compute_Statistics.m:57-82
      const double *u = st.U + ks * a.NU;
      const double Nr = u[0] + 1e-50;
      double y[DP], SC[DP][DP];
#pragma unroll
      for (int x = 0; x < DP; ++x) y[x] = x < d ? u[1 + x] / Nr : 0.0;
#pragma unroll
      for (int x = 0; x < DP; ++x)
#pragma unroll
        for (int z = 0; z < DP; ++z) SC[x][z] = 0.0;
      if (full) {
        // packed upper triangle: entry (x, z), x <= z, at 1 + d + x d - x (x - 1) / 2 + (z - x)
#pragma unroll
        for (int x = 0; x < DP; ++x)
#pragma unroll
          for (int z = 0; z < DP; ++z)
            if (x < d && z >= x && z < d) {
              const double ue = u[1 + d + x * d - x * (x - 1) / 2 + (z - x)] / Nr;
              SC[x][z] = ue - y[x] * y[z];
              SC[z][x] = ue - y[z] * y[x];
            }
      } else {
#pragma unroll
        for (int x = 0; x < DP; ++x)
          if (x < d) SC[x][x] = u[1 + d + x] / Nr - y[x] * y[x];
      }
      // vbhem_mstep_component.m:42-70
      const double l0 = a.lambda0;
      const double lam = l0 + Nr, v = a.v0 + Nr + 1.0, mult1 = l0 * Nr / (l0 + Nr);
      a.lam_o[ks] = lam;
      a.v_o[ks] = v;
      double Mt[DP][DP], tW[DP][DP];
#pragma unroll
      for (int x = 0; x < DP; ++x) {
        if (x < d) a.m_o[ks * d + x] = (l0 * a.m0[x] + Nr * y[x]) / (l0 + Nr);
#pragma unroll
        for (int z = 0; z < DP; ++z)
          Mt[x][z] = (x < d && z < d)
                         ? a.W0inv[x * d + z] + Nr * SC[x][z] +
                               mult1 * (y[x] - a.m0[x]) * (y[z] - a.m0[z])
                         : (x == z ? 1.0 : 0.0);
      }
      inv_reg<DP>(Mt, tW);
      double *W = a.W_o + ks * dd;
#pragma unroll
      for (int x = 0; x < DP; ++x) {
        if (full) {
#pragma unroll
          for (int z = 0; z < DP; ++z)
            if (x < d && z < d) W[x * d + z] = (tW[x][z] + tW[z][x]) / 2;
        } else if (x < d) {
          W[x] = (tW[x][x] + tW[x][x]) / 2;
        }
      }
      eta_ks = a.eta0 + st.N1[ks];
      a.eta_o[ks] = eta_ks;
      for (int s2 = 0; s2 < S; ++s2)
        a.eps_o[ks * S + s2] = a.epsilon0 + (S > 1 ? st.M[ks * S + s2] : 1e-12);
    }
    alpha_k = a.alpha0 + (st.Nj[k] + 1e-50);
    if (s == 0) {
      a.alpha_o[k] = alpha_k;
      for (int j = 0; j < K; ++j) sumA += a.alpha0 + (st.Nj[j] + 1e-50);
    }
  } else {
    if (on) eta_ks = a.eta[ks];
    alpha_k = a.alpha[k];
    if (s == 0)
      for (int j = 0; j < K; ++j) sumA += a.alpha[j];
  }
  // every write of this thread's posterior entries is its own: read back below
  const double *pv = do_mstep ? a.v_o : a.v, *plam = do_mstep ? a.lam_o : a.lam;
  const double *pm = do_mstep ? a.m_o : a.m, *pW = do_mstep ? a.W_o : a.W;
  const double *peps = do_mstep ? a.eps_o : a.eps;
  if (on) {
    // psi prelude (step_fc.m:118-165, 180-191)
    const double v = pv[ks];
    const double t1 = psi_sum_half_dev(v, d);
    const double *W = pW + ks * dd;
    double logdet = 0.0;
    if (full) {
      logdet = log(det_pad<DP>(W, d));
    } else {
      for (int x = 0; x < d; ++x) logdet += log(W[x]);
    }
    const double lLT = t1 + d * kLn2D + logdet;
    a.lLT[ks] = lLT;
    a.c[ks] = -lLT + d / plam[ks];
    for (int x = 0; x < dd; ++x) a.P[ks * dd + x] = v * W[x];
    for (int x = 0; x < d; ++x) a.cm[ks * d + x] = pm[ks * d + x];
    const double *eps = peps + ks * S;
    double es = 0.0;
    for (int s2 = 0; s2 < S; ++s2) es += eps[s2];
    const double pes = psi_dev(es);
    for (int s2 = 0; s2 < S; ++s2) a.logA[ks * S + s2] = psi_dev(eps[s2]) - pes;
  }
  red[s] = eta_ks;
  __syncthreads();
  if (s == 0) {
    double ets = 0.0;
    for (int x = 0; x < S; ++x) ets += red[x];
    red[0] = ets;
    a.logOmega[k] = psi_dev(alpha_k) - psi_dev(sumA);
  }
  __syncthreads();
  if (on) a.logPi[ks] = psi_dev(eta_ks) - psi_dev(red[0]);
}

// fixed-order block reduction of NQ partial sums (blockDim = kBoundThreads)
template <int NQ>
__device__ void block_sum(double (&q)[NQ], double *lds) {
  const int t = threadIdx.x;
#pragma unroll
  for (int x = 0; x < NQ; ++x) lds[x * kBoundThreads + t] = q[x];
  __syncthreads();
  for (int off = kBoundThreads / 2; off > 0; off >>= 1) {
    if (t < off)
#pragma unroll
      for (int x = 0; x < NQ; ++x) lds[x * kBoundThreads + t] += lds[x * kBoundThreads + t + off];
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < NQ; ++x) q[x] = lds[x * kBoundThreads];
}

// vbhemh3m_lb.m:64-186 (value), the same terms as vbhem_em_lower_bound
template <int DP>
__global__ __launch_bounds__(kBoundThreads) void em_bound_kernel(const EmDevArgs a, double *L_out) {
  constexpr int NQ = 13;
  __shared__ double lds[NQ * kBoundThreads];
  const int K = a.K, S = a.S, d = a.d, t = threadIdx.x;
  const bool full = a.covmode == 1;
  const int dd = full ? d * d : d;
  const StatsView st(a.stats, K, S, a.NU);
  const double l0 = a.lambda0, const2 = d * log(l0 / (2 * kPiD));
  // partial sums: 0 Lt51, 1 sum lLT, 2 sum v trW, 3 lt10a, 4 H, 5 Lt9, 6 sum logPi,
  // 7 sum logA, 8 Lt2, 9 sum logOmega, 10 Lt8b, 11 sum lgamma(alpha), 12 sum alpha
  double q[NQ];
#pragma unroll
  for (int x = 0; x < NQ; ++x) q[x] = 0.0;
  for (int ks = t; ks < K * S; ks += kBoundThreads) {
    const int k = ks / S, s = ks - k * S;
    const double v = a.v[ks], lam = a.lam[ks], lLT = a.lLT[ks];
    const double *W = a.W + (size_t)ks * dd;
    double detW;
    if (full) {
      detW = det_pad<DP>(W, d);
    } else {
      detW = 1.0;
      for (int x = 0; x < d; ++x) detW *= W[x];
    }
    const double sg = lgamma_sum_half_dev(v, d);
    const double logBk = -(v / 2) * log(detW) - (v * d / 2) * kLn2D -
                         (d * (d - 1) / 4.0) * log(kPiD) - sg;
    q[4] += -logBk - 0.5 * (v - d - 1) * lLT + 0.5 * v * d;
    double mWm = 0.0, trW = 0.0;
    const double *mk = a.m + (size_t)ks * d;
    for (int x = 0; x < d; ++x)
      for (int z = 0; z < d; ++z) {
        const double wxz = full ? W[x * d + z] : (x == z ? W[x] : 0.0);
        const double wzx = full ? W[z * d + x] : (x == z ? W[x] : 0.0);
        mWm += (mk[x] - a.m0[x]) * wxz * (mk[z] - a.m0[z]);
        trW += a.W0inv[x * d + z] * wzx;
      }
    q[0] += const2 + lLT - d * l0 / lam - l0 * v * mWm;
    q[1] += lLT;
    q[2] += v * trW;
    q[3] += lLT + d * log(lam / (2 * kPiD));
    // Lt9: the epsilon row s of cluster k, eta entry s (and lgamma(sum eta) at s = 0)
    const double *er = a.eps + (size_t)ks * S;
    double ps = 0.0, lgp = 0.0, pt = 0.0, sla = 0.0;
    for (int s2 = 0; s2 < S; ++s2) {
      ps += er[s2];
      lgp += lgamma(er[s2]);
      pt += (er[s2] - 1) * a.logA[(size_t)ks * S + s2];
      sla += a.logA[(size_t)ks * S + s2];
    }
    q[5] += lgamma(ps) - lgp + pt;
    const double e = a.eta[ks];
    q[5] += -lgamma(e) + (e - 1) * a.logPi[ks];
    if (s == 0) {
      double es = 0.0;
      for (int s2 = 0; s2 < S; ++s2) es += a.eta[(size_t)k * S + s2];
      q[5] += lgamma(es);
    }
    q[6] += a.logPi[ks];
    q[7] += sla;
  }
  for (int k = t; k < K; k += kBoundThreads) {
    const double lo = a.logOmega[k], al = a.alpha[k];
    q[8] += (st.Nj[k] + 1e-50) * lo;
    q[9] += lo;
    q[10] += (al - 1) * lo;
    q[11] += lgamma(al);
    q[12] += al;
  }
  block_sum<NQ>(q, lds);
  if (t == 0) {
    const double a0 = a.alpha0, e0 = a.eta0, ep0 = a.epsilon0, v0 = a.v0;
    const double Lt3 = K * a.logCeta0 + (e0 - 1) * q[6];
    const double Lt4 = (double)K * S * a.logCepsilon0 + (ep0 - 1) * q[7];
    const double Lt5 = 0.5 * q[0] + (double)K * S * a.logB0 + 0.5 * (v0 - d - 1) * q[1] - 0.5 * q[2];
    const double Lt6 = a.logCalpha0 + (a0 - 1) * q[9];
    const double Lt8 = (lgamma(q[12]) - q[11]) + q[10];
    const double Lt10 = 0.5 * q[3] - 0.5 * d * S * K - q[4];
    *L_out = st.Lt1 + q[8] + Lt3 + Lt4 + Lt5 + Lt6 - st.Lt7 - Lt8 - q[5] - Lt10;
  }
}

template <int DP>
hipError_t launch_em_dev(const EmDevArgs &a, int mode, double *L_out, hipStream_t st) {
  if (mode == kEmBound) {
    hipLaunchKernelGGL(em_bound_kernel<DP>, dim3(1), dim3(kBoundThreads), 0, st, a, L_out);
  } else {
    hipLaunchKernelGGL(em_step_kernel<DP>, dim3(a.K), dim3(kStepThreads), 0, st, a,
                       mode == kEmMstepPrelude ? 1 : 0);
  }
  return hipGetLastError();
}

}  // namespace

bool em_dev_supported(int d, int S) { return d >= 1 && d <= kEmDevMaxD && S >= 1 && S <= kStepThreads; }

hipError_t launch_em_dev(const EmDevArgs &a, int mode, double *L_out, hipStream_t st) {
  if (!em_dev_supported(a.d, a.S)) return hipErrorInvalidValue;
  if (a.d <= 2) return launch_em_dev<2>(a, mode, L_out, st);
  if (a.d <= 4) return launch_em_dev<4>(a, mode, L_out, st);
  if (a.d <= 8) return launch_em_dev<8>(a, mode, L_out, st);
  return launch_em_dev<16>(a, mode, L_out, st);
}

}  // namespace vbhem

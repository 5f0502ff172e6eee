// vbhem_kernels.hip -- MI355X (gfx950) kernels for the VBHEM-H3M E-step.
//
// Hot path = the per-(base HMM i, cluster HMM j) hierarchical backward/forward
// recursion of src/vbhem/vbhem_hmm_bwd_fwd_mex.c (K1..K5, mex.c:715-1469),
// followed by the responsibilities (vbhem_h3m_c_step_fc.m:271-283) and the
// Z-weighted statistic reduction (vbhem_compute_Statistics.m:33-55).
//
// Kernels
//   fb_pairs_kernel<D>  one chain per wavefront slice: lane = (cluster state a,
//                       base state b) of one pair; several pairs per block share
//                       staged base/cluster parameters in LDS.  K1 emission,
//                       backward recursion with a factorised log-sum-exp, the
//                       termination, the forward recursion.  fp64 throughout.
//   fb_exact_kernel     reference-order fallback (stores Theta, S^2*Sb exps per
//                       step) for pairs whose factorised normaliser left its
//                       safe range (only with pathological hyperparameters).
//   pair_emit_kernel    K5 per pair (MEX-equivalent emit_pr/mu/Mu outputs).
//   (the fused epilogue -- responsibilities and statistics -- is in vbhem_stats.hip)
//
// Factorised backward step (exact algebra):
//   l(rho,sig,b) = logA(rho,sig) + v(sig,b),  v = E + L
//   exp(l) = A'(rho,sig) * G(sig,b) * exp(amax(rho) + M(b)),
//     A' = exp(logA - amax(rho)),  G = exp(v - M(b)),  M(b) = max_sig v(sig,b)
//   s(rho,b)   = M(b) + amax(rho) + log Z(rho,b),  Z = sum_sig A'(rho,sig) G(sig,b)
//   Theta(rho,sig,b) = A'(rho,sig) G(sig,b) / Z(rho,b)
// so a step costs S*Sb exps and S*Sb logs instead of the reference's S*S*Sb
// exps; the forward step needs no transcendental at all.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdint>

#include "vbhem_internal.h"
#include "vbhem_exact.h"

namespace vbhem {


constexpr double kLog2Pi = 1.8378770664093454835606594728112353;  // log(2*pi)
constexpr double kZMin = 1e-200;  // below: fall back to the exact reference order

__device__ __forceinline__ int packed_index(int a, int b, int d) {
  // upper-triangular (a <= b), row-major
  return a * d - (a * (a - 1)) / 2 + (b - a);
}

// ---------------------------------------------------------------------------
// K1: expected log-likelihood of base state b's Gaussian under cluster state a
//   E = -1/2 ( d log 2pi + c + sum_{a,b} P_ab (Sigma_ab + x_a x_b) ),  x = mu - m
// (mex.c:796-843 full, :744-759 diag).  P symmetric (P = v*W, W symmetrised at
// vbhem_mstep_component.m:62,68); Cs holds Sigma_aa on the diagonal and
// Sigma_ab + Sigma_ba off it, so an asymmetric Sigma is still exact.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ double emission_full(int d, const double *__restrict__ mrow,
                                                const double *__restrict__ Pp, double c,
                                                const double *__restrict__ mu,
                                                const double *__restrict__ Cs) {
  double ell = 0.0;
  if constexpr (D > 0) {
    double x[D];
#pragma unroll
    for (int q = 0; q < D; ++q) x[q] = mu[q] - mrow[q];
    int k = 0;
#pragma unroll
    for (int q = 0; q < D; ++q) {
      ell = fma(Pp[k], fma(x[q], x[q], Cs[k]), ell);
      ++k;
#pragma unroll
      for (int r = q + 1; r < D; ++r) {
        ell = fma(Pp[k], fma(2.0 * x[q], x[r], Cs[k]), ell);
        ++k;
      }
    }
  } else {
    int k = 0;
    for (int q = 0; q < d; ++q) {
      const double xq = mu[q] - mrow[q];
      ell = fma(Pp[k], fma(xq, xq, Cs[k]), ell);
      ++k;
      for (int r = q + 1; r < d; ++r) {
        const double xr = mu[r] - mrow[r];
        ell = fma(Pp[k], fma(2.0 * xq, xr, Cs[k]), ell);
        ++k;
      }
    }
  }
  return -0.5 * (d * kLog2Pi + c + ell);
}

template <int D>
__device__ __forceinline__ double emission_diag(int d, const double *__restrict__ mrow,
                                                const double *__restrict__ P, double c,
                                                const double *__restrict__ mu,
                                                const double *__restrict__ C) {
  double ell = 0.0;
  const int dd = D > 0 ? D : d;
#pragma unroll
  for (int q = 0; q < (D > 0 ? D : 1); ++q) {
    if constexpr (D > 0) {
      const double x = mu[q] - mrow[q];
      ell = fma(P[q], fma(x, x, C[q]), ell);
    }
  }
  if constexpr (D == 0) {
    for (int q = 0; q < dd; ++q) {
      const double x = mu[q] - mrow[q];
      ell = fma(P[q], fma(x, x, C[q]), ell);
    }
  }
  return -0.5 * (d * kLog2Pi + c + ell);
}

// ---------------------------------------------------------------------------
// fb_pairs_kernel: K1..K4 for BI bases x BJ clusters per block.
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(512) void fb_pairs_kernel(const FbArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  const int nthr = blockDim.x;
  const int S = p.S, SB = p.SB, NE = p.NE, RS = p.RS, AS = p.AS, ABS = p.ABS, T = p.T;
  const int d = D > 0 ? D : p.d;
  const int blk = blockIdx.x;
  const int ib = blk / p.njb, jb = blk % p.njb;
  const int i0 = p.i_begin + ib * p.BI, j0 = jb * p.BJ;
  const int PPB = p.BI * p.BJ;

  double *At = lds + p.off_At;      // [BJ][S][AS]   A' = exp(logA - rowmax)
  double *amax = lds + p.off_amax;  // [BJ][S]
  double *lpi = lds + p.off_lpi;    // [BJ][S]
  double *Ab = lds + p.off_Ab;      // [BI][SB][ABS]
  double *pib = lds + p.off_pib;    // [BI][SB]
  int *pflag = reinterpret_cast<int *>(lds + p.off_flag);  // [PPB]
  double *reg = lds + p.off_reg;    // union: K1 staging | per-pair scratch

  // ---- stage cluster constants ------------------------------------------
  for (int x = tid; x < p.BJ * S; x += nthr) {
    const int bj = x / S, r = x - (x / S) * S, j = j0 + bj;
    double mx = -INFINITY, lp = 0.0;
    if (j < p.K) {
      const double *la = p.logA + ((size_t)j * S + r) * S;
      mx = la[0];
      for (int s = 1; s < S; ++s) mx = fmax(mx, la[s]);
      for (int s = 0; s < S; ++s) At[(bj * S + r) * AS + s] = exp(la[s] - mx);
      lp = p.logPi[(size_t)j * S + r];
    } else {
      for (int s = 0; s < S; ++s) At[(bj * S + r) * AS + s] = 0.0;
    }
    amax[x] = mx;
    lpi[x] = lp;
  }
  // ---- stage base transition / prior ------------------------------------
  for (int x = tid; x < p.BI * SB * SB; x += nthr) {
    const int bi = x / (SB * SB), rem = x - bi * SB * SB, g = rem / SB, be = rem - g * SB;
    const int i = i0 + bi;
    Ab[(bi * SB + g) * ABS + be] = (i < p.i_end) ? p.A[((size_t)i * SB + g) * SB + be] : 0.0;
  }
  for (int x = tid; x < p.BI * SB; x += nthr) {
    const int bi = x / SB, be = x - bi * SB, i = i0 + bi;
    pib[x] = (i < p.i_end) ? p.prior[(size_t)i * SB + be] : 0.0;
  }
  for (int x = tid; x < PPB; x += nthr) pflag[x] = 0;
  // ---- stage K1 operands (packed) ----------------------------------------
  double *k1m = reg + p.off_k1m;    // [BJ][S][MS]
  double *k1P = reg + p.off_k1P;    // [BJ][S][PS]  packed P
  double *k1c = reg + p.off_k1c;    // [BJ][S]
  double *k1mu = reg + p.off_k1mu;  // [BI][SB][MS]
  double *k1C = reg + p.off_k1C;    // [BI][SB][PS] packed Sigma (sym-folded)
  const int np = p.np, MS = p.MS, PS = p.PS;
  for (int x = tid; x < p.BJ * S; x += nthr) {
    const int bj = x / S, s = x - bj * S, j = j0 + bj;
    const bool ok = j < p.K;
    for (int q = 0; q < d; ++q) k1m[x * MS + q] = ok ? p.m[((size_t)j * S + s) * d + q] : 0.0;
    k1c[x] = ok ? p.c[(size_t)j * S + s] : 0.0;
    if (p.covmode == kCovFull) {
      const double *Pj = p.P + ((size_t)j * S + s) * d * d;
      for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b)
          k1P[x * PS + packed_index(a, b, d)] = ok ? Pj[a * d + b] : 0.0;
    } else {
      for (int q = 0; q < d; ++q) k1P[x * PS + q] = ok ? p.P[((size_t)j * S + s) * d + q] : 0.0;
    }
  }
  for (int x = tid; x < p.BI * SB; x += nthr) {
    const int bi = x / SB, be = x - bi * SB, i = i0 + bi;
    const bool ok = i < p.i_end;
    for (int q = 0; q < d; ++q) k1mu[x * MS + q] = ok ? p.centres[((size_t)i * SB + be) * d + q] : 0.0;
    if (p.covmode == kCovFull) {
      const double *Ci = p.covars + ((size_t)i * SB + be) * d * d;
      for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b)
          k1C[x * PS + packed_index(a, b, d)] =
              ok ? (a == b ? Ci[a * d + a] : Ci[a * d + b] + Ci[b * d + a]) : 0.0;
    } else {
      for (int q = 0; q < d; ++q) k1C[x * PS + q] = ok ? p.covars[((size_t)i * SB + be) * d + q] : 0.0;
    }
  }
  (void)np;
  __syncthreads();

  // ---- lane role -----------------------------------------------------------
  const int q = tid / NE;
  const int e = tid - q * NE;
  const int a = e / SB;
  const int b = e - a * SB;
  const bool lane_ok = q < PPB;
  const int bi = lane_ok ? q / p.BJ : 0, bj = lane_ok ? q - (q / p.BJ) * p.BJ : 0;
  const int i = i0 + bi, j = j0 + bj;
  const bool active = lane_ok && (i < p.i_end) && (j < p.K);
  const size_t pair = (size_t)i * p.K + j;              // global (LL, flags)
  const size_t lp = (size_t)(i - p.i_buf0) * p.K + j;   // local (nu1, xi, tnu)

  double E = 0.0;
  if (lane_ok) {
    const int cs = bj * S + a, bs = bi * SB + b;
    if (p.covmode == kCovFull)
      E = emission_full<D>(d, k1m + cs * MS, k1P + cs * PS, k1c[cs], k1mu + bs * MS, k1C + bs * PS);
    else
      E = emission_diag<D>(d, k1m + cs * MS, k1P + cs * PS, k1c[cs], k1mu + bs * MS, k1C + bs * PS);
    if (p.smooth != 1.0) E = E / p.smooth;
  }
  __syncthreads();  // K1 staging region is reused below

  double *pr = reg + (size_t)(lane_ok ? q : 0) * p.pair_stride;
  double *Gst = pr;                                   // [(T-1)][S][RS]
  double *Zi = Gst + (size_t)(T - 1) * S * RS;        // [(T-1)][NE]
  double *X1 = Zi + (size_t)(T - 1) * NE;             // [2][S][RS]  (ping-pong)
  double *X2 = X1 + 2 * S * RS;                       // [S][RS]
  double *H = X2 + S * RS;                            // [S*S]
  double *Y = H + S * S;                              // [SB]
  const double *Atj = At + bj * S * AS;
  const double *amaxj = amax + bj * S;
  const double *lpij = lpi + bj * S;
  const double *Abi = Ab + bi * SB * ABS;
  const double *pibi = pib + bi * SB;

  // ---- K2: backward recursion (mex.c:915-1015) ------------------------------
  double L = 0.0;
  bool bad = false;
  for (int t = T - 1; t >= 1; --t) {
    double *Gt = Gst + (size_t)(t - 1) * S * RS;
    const double v = E + L;
    if (lane_ok) X1[a * RS + b] = v;
    __syncthreads();
    double Mb = 0.0;
    if (lane_ok) {
      Mb = X1[b];
      for (int s = 1; s < S; ++s) Mb = fmax(Mb, X1[s * RS + b]);
      Gt[a * RS + b] = exp(v - Mb);
    }
    __syncthreads();
    if (lane_ok) {
      const double *arow = Atj + a * AS;
      double Z = 0.0;
      for (int s = 0; s < S; ++s) Z = fma(arow[s], Gt[s * RS + b], Z);
      bad |= !(Z >= kZMin);
      Zi[(size_t)(t - 1) * NE + e] = 1.0 / Z;
      X2[a * RS + b] = Mb + amaxj[a] + log(Z);
    }
    __syncthreads();
    if (lane_ok) {
      // L(rho=a, gamma=b) = sum_beta Ab(b, beta) * s(a, beta)
      const double *arow = Abi + b * ABS;
      const double *srow = X2 + a * RS;
      double Ln = 0.0;
      for (int be = 0; be < SB; ++be) Ln = fma(arow[be], srow[be], Ln);
      L = Ln;
    }
  }

  // ---- K3: termination (mex.c:1020-1080) ------------------------------------
  const double v1 = lane_ok ? lpij[a] + E + L : 0.0;
  if (lane_ok) X1[a * RS + b] = v1;
  __syncthreads();
  double M1 = 0.0;
  if (lane_ok) {
    M1 = X1[b];
    for (int s = 1; s < S; ++s) M1 = fmax(M1, X1[s * RS + b]);
    X2[a * RS + b] = exp(v1 - M1);
  }
  __syncthreads();
  double nu = 0.0;
  if (lane_ok) {
    double Zs = 0.0;
    for (int s = 0; s < S; ++s) Zs += X2[s * RS + b];
    const double s1 = M1 + log(Zs);
    nu = pibi[b] * exp(v1 - s1);                // nu_1 = prior .* Theta_1
    if (a == 0) Y[b] = pibi[b] * s1;            // LL_elbo terms
  }
  __syncthreads();
  double *Xc = X1, *Xn = X1 + S * RS;
  if (lane_ok) {
    Xc[a * RS + b] = nu;
    for (int o = e; o < S * S; o += NE) H[o] = 0.0;
  }
  __syncthreads();
  if (active) {
    if (e == 0) {
      double ll = 0.0;
      for (int be = 0; be < SB; ++be) ll += Y[be];
      p.LL[pair] = ll;
    }
    if (b == 0) {
      double n1 = 0.0;
      for (int be = 0; be < SB; ++be) n1 += Xc[a * RS + be];
      p.nu1[lp * S + a] = n1;
    }
  }

  // ---- K4: forward recursion (mex.c:1178-1298) ------------------------------
  double tnu = nu;
  for (int t = 1; t < T; ++t) {
    const double *Gt = Gst + (size_t)(t - 1) * S * RS;
    if (lane_ok) {
      // f(rho=a, gamma=b) = sum_beta nu(a, beta) Ab(beta, b);  g = f / Z_t
      const double *nrow = Xc + a * RS;
      double f = 0.0;
      for (int be = 0; be < SB; ++be) f = fma(nrow[be], Abi[be * ABS + b], f);
      X2[a * RS + b] = f * Zi[(size_t)(t - 1) * NE + e];
    }
    __syncthreads();
    if (lane_ok) {
      // nu(sig=a, gamma=b) = G_t(a,b) * sum_rho A'(rho,a) g(rho,b)
      double acc = 0.0;
      for (int r = 0; r < S; ++r) acc = fma(Atj[r * AS + a], X2[r * RS + b], acc);
      nu = Gt[a * RS + b] * acc;
      tnu += nu;
      // h(rho,sig) += sum_gamma g(rho,gamma) G_t(sig,gamma)
      for (int o = e; o < S * S; o += NE) {
        const int ro = o / S, so = o - ro * S;
        const double *grow = X2 + ro * RS, *Grow = Gt + so * RS;
        double h = 0.0;
        for (int be = 0; be < SB; ++be) h = fma(grow[be], Grow[be], h);
        H[o] += h;
      }
      Xn[a * RS + b] = nu;
    }
    __syncthreads();
    double *tmp = Xc;
    Xc = Xn;
    Xn = tmp;
  }

  // ---- outputs ---------------------------------------------------------------
  if (active) {
    p.tnu[(lp * S + a) * SB + b] = tnu;
    for (int o = e; o < S * S; o += NE) {
      const int ro = o / S, so = o - ro * S;
      p.xi[lp * S * S + o] = Atj[ro * AS + so] * H[o];
    }
    if (bad) {  // underflow, or non-finite inputs (NaN propagates through exp/log here)
      bool nf = !isfinite(E);
      for (int s = 0; s < S; ++s) nf |= isnan(Atj[a * AS + s]) || isnan(amaxj[s]);
      atomicOr(&pflag[q], kFlagBad | (nf ? kFlagNonFinite : 0));
    }
  }
  __syncthreads();
  if (active && e == 0 && pflag[q] == kFlagBad) {
    const int slot = atomicAdd(p.flag_count, 1);
    atomicAdd(p.flag_count + 1, 1);
    p.flag_list[slot] = (int)pair;
  }
}

// ---------------------------------------------------------------------------
// fb_exact_kernel: reference-order recursion for flagged pairs, ONE WAVEFRONT per
// pair (exact_pair_wave: the element loops of mex.c:715-1298 over the lanes, every
// sum in the reference's order; Theta in the wave's global scratch slot, the pair's
// small arrays in the wave's LDS region), wavefronts grid-striding over the list.
// kExactBlocks blocks of kExactBlock threads: one scratch slot per wavefront.  The
// blocks consume the pass's flag counter; the last block to finish resets it (and the
// blocks-done counter) to zero, so the next pass needs no memset of its own
// (flag_count[1] keeps the total).  Every block reads the count before it signals
// completion, so the reset can never race a read.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kExactBlock) __attribute__((amdgpu_waves_per_eu(4)))
void fb_exact_kernel(const FbArgs p, double *scratch, size_t scratch_stride, int from_fold) {
  extern __shared__ double xlds[];
  const int cnt = __atomic_load_n(p.flag_count, __ATOMIC_RELAXED);
  // nothing flagged (the usual case): every block reads 0 -- nobody writes the
  // counter while it is 0 -- so all leave at once, with no reset to do
  if (cnt == 0) return;
  // from_fold: resp_kernel took the backward pass's entries [0, flag_count[3])
  const int x0 = from_fold ? p.flag_count[3] : 0;
  const int wpb = kExactBlock / 64, wave = threadIdx.x >> 6;
  const int gw = blockIdx.x * wpb + wave, nw = gridDim.x * wpb;
  double *w = scratch + (size_t)gw * scratch_stride;
  if (exact_wave_in_lds(p.S, p.SB)) {
    double *lw = xlds + (size_t)wave * exact_wave_lds(p.S, p.SB);
    for (int idx = x0 + gw; idx < cnt; idx += nw) exact_pair_wave<false>(p, p.flag_list[idx], w, lw);
  } else {
    for (int idx = x0 + gw; idx < cnt; idx += nw) exact_pair_wave<true>(p, p.flag_list[idx], w, nullptr);
  }
  __syncthreads();  // every thread of this block has read the count
  if (threadIdx.x == 0) {
    const int done = atomicAdd(p.flag_count + 2, 1);
    if (done == (int)gridDim.x - 1) {  // last block: everyone has read the count
      atomicExch(p.flag_count, 0);
      atomicExch(p.flag_count + 2, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// pair_emit_kernel: K5 per pair (mex.c:1348-1469), one thread per (pair, sigma).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void pair_emit_kernel(EmitArgs p) {
  const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)(p.i_end - p.i_begin) * p.K * p.S;
  if (x >= total) return;
  const int S = p.S, SB = p.SB, d = p.d;
  const size_t pl = x / S;             // local pair index
  const int s = (int)(x - pl * S);
  const size_t pair = (size_t)p.i_begin * p.K + pl;
  const int i = (int)(pair / p.K);
  const double *tn = p.tnu + (pair * S + s) * SB;
  const double *mu = p.centres + (size_t)i * SB * d;
  double pr = 0.0;
  for (int be = 0; be < SB; ++be) pr += tn[be];
  p.emit_pr[pair * S + s] = pr;
  for (int q = 0; q < d; ++q) {
    double acc = 0.0;
    for (int be = 0; be < SB; ++be) acc += tn[be] * mu[be * d + q];
    p.emit_mu[(pair * S + s) * d + q] = acc;
  }
  if (p.covmode == kCovFull) {
    const double *C = p.covars + (size_t)i * SB * d * d;
    double *out = p.emit_Mu + (pair * S + s) * d * d;
    for (int q = 0; q < d; ++q)
      for (int r = 0; r < d; ++r) {
        double acc = 0.0;
        for (int be = 0; be < SB; ++be)
          acc += tn[be] * (mu[be * d + q] * mu[be * d + r] + C[(be * d + q) * d + r]);
        out[q * d + r] = acc;
      }
  } else {
    const double *C = p.covars + (size_t)i * SB * d;
    double *out = p.emit_Mu + (pair * S + s) * d;
    for (int q = 0; q < d; ++q) {
      double acc = 0.0;
      for (int be = 0; be < SB; ++be) acc += tn[be] * (mu[be * d + q] * mu[be * d + q] + C[be * d + q]);
      out[q] = acc;
    }
  }
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
template <int D>
static hipError_t launch_fb_d(const FbArgs &a, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&fb_pairs_kernel<D>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fb_pairs_kernel<D>, grid, block, lds, st, a);
  return hipGetLastError();
}

hipError_t launch_fb(const FbArgs &a, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
  switch (a.d) {
    case 1: return launch_fb_d<1>(a, grid, block, lds, st);
    case 2: return launch_fb_d<2>(a, grid, block, lds, st);
    case 3: return launch_fb_d<3>(a, grid, block, lds, st);
    case 4: return launch_fb_d<4>(a, grid, block, lds, st);
    case 5: return launch_fb_d<5>(a, grid, block, lds, st);
    case 6: return launch_fb_d<6>(a, grid, block, lds, st);
    case 8: return launch_fb_d<8>(a, grid, block, lds, st);
    case 12: return launch_fb_d<12>(a, grid, block, lds, st);
    case 16: return launch_fb_d<16>(a, grid, block, lds, st);
    default: return launch_fb_d<0>(a, grid, block, lds, st);
  }
}

hipError_t launch_fb_exact(const FbArgs &a, double *scratch, size_t stride, int nslots,
                           hipStream_t st, bool from_fold) {
  // the scratch holds kExactSlots slots, one per wavefront (vbhem_capi.hip)
  if (nslots != kExactSlots) return hipErrorInvalidValue;
  const size_t lds = exact_wave_in_lds(a.S, a.SB)
                         ? (size_t)(kExactBlock / 64) * exact_wave_lds(a.S, a.SB) * sizeof(double)
                         : 0;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&fb_exact_kernel), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fb_exact_kernel, dim3(kExactBlocks), dim3(kExactBlock), lds, st, a, scratch,
                     stride, (int)from_fold);
  return hipGetLastError();
}

hipError_t launch_emit(const EmitArgs &a, hipStream_t st) {
  const size_t total = (size_t)(a.i_end - a.i_begin) * a.K * a.S;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(pair_emit_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace vbhem

// vbhem_stats.hip -- the fused E-step epilogue: responsibilities and the gated,
// Z-weighted statistic sums of one EM iteration (gfx950).
//
//   resp_kernel        hat_Z / Z = hat_Z * tilde_N per base (vbhem_h3m_c_step_fc.m:271-283)
//                      and the per-chunk partial sums Nj = sum_i Z (:282),
//                      Lt1 = sum Z .* L_elbo, Lt7 = sum hat_Z .* log(hat_Z)
//                      (vbhemh3m_lb.m:90, 107).
//   stats_kernel<..>   streaming split-K reduction over this chunk's bases
//                      (vbhem_compute_Statistics.m:33-55, gate Z > 1e-8):
//                        N1[j][s]    += g Z(i,j) sum_nu_1(i,j,s)
//                        M[j][s][r]  += g Z(i,j) sum_xi(i,j,s,r)
//                        U[(j,s)][c] += sum_b (g Z(i,j) sum_t_nu(i,j,s,b)) u(i,b,c)
//                      with u = [1, mu, packed Sigma + mu mu'] -- the emission
//                      moments of mex.c:1348-1469 contracted over the base states
//                      and the bases at once: a (K*S) x (N*Sb) x NU GEMM on
//                      v_mfma_f64_16x16x4f64, K-dim streamed in batches of NBB bases.
//   stats_final_kernel fixed-order sum of the per-chunk slabs.
//
// Grid: x = chunk of consecutive bases, y = group of JG clusters (rows j*S+s),
// so no tile is loaded twice; every block keeps its whole (JG*S) x NU output
// block in MFMA accumulators and its N1/M entries in registers.
// All sums run in a fixed order (no atomics): bit-reproducible.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "vbhem_internal.h"

namespace vbhem {

namespace {

typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// x / D for 0 <= x < 2^22 and small D, via a float reciprocal (exact: the
// +0.5 offset keeps the quotient 0.5/D away from an integer).
__device__ __forceinline__ int qdiv(int x, float inv) { return (int)(((float)x + 0.5f) * inv); }

__device__ __forceinline__ void chunk_range(int nb, int i_begin, int chunk, int nchunk, int &b0,
                                            int &b1) {
  const int per = (nb + nchunk - 1) / nchunk;
  b0 = i_begin + chunk * per;
  b1 = min(i_begin + nb, b0 + per);
}

}  // namespace

// ---------------------------------------------------------------------------
// resp_kernel: one wavefront per base (lanes over clusters j).
// ---------------------------------------------------------------------------
constexpr int kRespThreads = 256;

__global__ __launch_bounds__(kRespThreads) void resp_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kRespThreads / 64;
  const int K = p.K;
  double *accNj = lds;                 // [NW][K]
  double *accLt = accNj + NW * K;      // [NW][2]
  for (int x = tid; x < NW * K + 2 * NW; x += kRespThreads) accNj[x] = 0.0;
  __syncthreads();
  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  double l1 = 0.0, l7 = 0.0;
  for (int i = b0 + wave; i < b1; i += NW) {
    // log_Z = tilde_N .* (logOmega + L_elbo) is rounded before the shift, as in
    // step_fc.m:275-276 (an fma-contracted shift would let the winning entry
    // exceed 1 by ~ulp(log_Z)).
#pragma clang fp contract(off)
    const double tn = p.tildeN[i];
    const double *LL = p.LL + (size_t)i * K;
    double mx = -INFINITY;
    for (int j = lane; j < K; j += 64) mx = fmax(mx, tn * (p.logOmega[j] + LL[j]));
    mx = wave_max(mx);
    double sm = 0.0;
    for (int j = lane; j < K; j += 64) sm += exp(tn * (p.logOmega[j] + LL[j]) - mx);
    sm = wave_sum(sm);
    const double lse = mx + log(sm);
    for (int j = lane; j < K; j += 64) {
      const double ll = LL[j];
      const double hz = exp(tn * (p.logOmega[j] + ll) - lse) + 1e-50;
      const double Z = hz * tn;
      p.hatZ[(size_t)i * K + j] = hz;
      p.Z[(size_t)(i - p.i_buf0) * K + j] = Z;
      accNj[wave * K + j] += Z;
      l1 += Z * ll;
      l7 += hz * log(hz);
    }
  }
  l1 = wave_sum(l1);
  l7 = wave_sum(l7);
  if (lane == 0) {
    accLt[2 * wave] = l1;
    accLt[2 * wave + 1] = l7;
  }
  __syncthreads();
  double *slab = p.slabs + (size_t)blockIdx.x * p.slab_len;
  for (int j = tid; j < K; j += kRespThreads) {
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += accNj[w * K + j];
    slab[j] += s;
  }
  if (tid < 2) {
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += accLt[2 * w + tid];
    slab[(size_t)K + (size_t)K * p.S + (size_t)K * p.S * p.S + tid] += s;
  }
}

// ---------------------------------------------------------------------------
// stats_kernel<TPW, MAXM>: TPW = max MFMA tiles per wave, MAXM = max M entries
// per thread (registers).
// ---------------------------------------------------------------------------
constexpr int kStatsThreads = 512;
constexpr int kStatsWaves = kStatsThreads / 64;

template <int TPW, int MAXM>
__global__ __launch_bounds__(kStatsThreads) void stats_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = p.K, S = p.S, SB = p.SB, SBp = p.SBp, d = p.d, NU = p.NU, NBB = p.NBB;
  const int AST = p.AST, UST = p.UST;
  const int j0 = blockIdx.y * p.JG, j1 = min(K, j0 + p.JG), JGc = j1 - j0;
  const int RG = JGc * S, SS = S * S;
  const int MT = (RG + 15) / 16, NTL = (NU + 15) / 16, ntiles = MT * NTL;
  const bool full = p.covmode == kCovFull;

  double *As = lds;                                   // [RG][AST]   g Z sum_t_nu
  double *Us = As + (size_t)RG * AST;                 // [NBB*SBp][UST] base moments
  double *gzs = Us + (size_t)NBB * SBp * UST;         // [NBB][JGc]
  int *tab = reinterpret_cast<int *>(gzs + (size_t)NBB * JGc);  // [NU] packed (a,b)

  for (int x = tid; x < RG * AST + NBB * SBp * UST; x += kStatsThreads) As[x] = 0.0;
  for (int c = tid; c < NU; c += kStatsThreads) {
    int a = -1, b = -1;
    if (c >= 1 && c <= d) {
      a = c - 1;
    } else if (c > d) {
      if (full) {
        int k = c - 1 - d;
        a = 0;
        while (k >= d - a) { k -= d - a; ++a; }
        b = a + k;
      } else {
        a = b = c - 1 - d;
      }
    }
    tab[c] = (a + 1) | ((b + 1) << 16);
  }

  const float invNU = 1.0f / (float)NU, invSB = 1.0f / (float)SB, invS = 1.0f / (float)S;
  const float invSS = 1.0f / (float)SS, invJG = 1.0f / (float)JGc;
  const float invRSB = 1.0f / (float)(RG * SB);

  double4_t acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = (double4_t){0.0, 0.0, 0.0, 0.0};
  double accM[MAXM];
  int jM[MAXM];
#pragma unroll
  for (int e = 0; e < MAXM; ++e) {
    accM[e] = 0.0;
    jM[e] = qdiv(tid + e * kStatsThreads, invSS);
  }
  double accN1 = 0.0;
  const int jN1 = qdiv(tid, invS);

  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  const double *__restrict__ tnu = p.tnu;
  const double *__restrict__ xi = p.xi;
  const double *__restrict__ nu1 = p.nu1;
  const double *__restrict__ cen = p.centres;
  const double *__restrict__ cov = p.covars;
  const size_t dC = full ? (size_t)d * d : (size_t)d;
  __syncthreads();

  for (int ib = b0; ib < b1; ib += NBB) {
    const int nq = min(NBB, b1 - ib);
    // -- gated Z of the batch, and the base moments u (independent of Z) -------
    for (int x = tid; x < NBB * JGc; x += kStatsThreads) {
      const int q = qdiv(x, invJG), jj = x - q * JGc;
      double z = 0.0;
      if (q < nq) z = p.Z[(size_t)(ib + q - p.i_buf0) * K + j0 + jj];
      gzs[x] = (z > 1e-8) ? z : 0.0;
    }
    for (int x = tid; x < NBB * SB * NU; x += kStatsThreads) {
      const int row = qdiv(x, invNU), c = x - row * NU;
      const int q = qdiv(row, invSB), be = row - q * SB;
      double u = 0.0;
      if (q < nq) {
        const int i = ib + q;
        const int t = tab[c], a = (t & 0xffff) - 1, b = (t >> 16) - 1;
        const double *mu = cen + ((size_t)i * SB + be) * d;
        if (a < 0) {
          u = 1.0;
        } else if (b < 0) {
          u = mu[a];
        } else {
          const double *C = cov + ((size_t)i * SB + be) * dC;
          u = (full ? C[a * d + b] : C[a]) + mu[a] * mu[b];
        }
      }
      Us[(q * SBp + be) * UST + c] = u;
    }
    __syncthreads();
    // -- A = g Z sum_t_nu (rows r = (j - j0)*S + s, cols q*SBp + beta) ---------
#pragma unroll 4
    for (int x = tid; x < NBB * RG * SB; x += kStatsThreads) {
      const int q = qdiv(x, invRSB), rem = x - q * RG * SB;
      const int r = qdiv(rem, invSB), be = rem - r * SB;
      double v = 0.0;
      if (q < nq) {
        const size_t pr = (size_t)(ib + q - p.i_buf0) * K * S + (size_t)j0 * S + r;
        v = gzs[q * JGc + qdiv(r, invS)] * tnu[pr * SB + be];
      }
      As[r * AST + q * SBp + be] = v;
    }
    // -- N1 / M partial sums (registers) ---------------------------------------
    for (int q = 0; q < nq; ++q) {
      const size_t ib_rel = (size_t)(ib + q - p.i_buf0);
      if (tid < RG) accN1 += gzs[q * JGc + jN1] * nu1[ib_rel * K * S + (size_t)j0 * S + tid];
      const double *xq = xi + ib_rel * K * SS + (size_t)j0 * SS;
#pragma unroll
      for (int e = 0; e < MAXM; ++e) {
        const int x = tid + e * kStatsThreads;
        if (x < JGc * SS) accM[e] += gzs[q * JGc + jM[e]] * xq[x];
      }
    }
    __syncthreads();
    // -- MFMA: acc[tile] += A[16 rows, 4 k] x U[4 k, 16 cols] -------------------
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int tile = wave + t * kStatsWaves;
      if (tile < ntiles) {
        const int mt = tile % MT, nt = tile / MT;
        const int row = mt * 16 + (lane & 15);
        const int col = nt * 16 + (lane & 15);
        const double *arow = As + (size_t)(row < RG ? row : 0) * AST;
        const double amask = row < RG ? 1.0 : 0.0;
        for (int ks = 0; ks < NBB * SBp; ks += 4) {
          const int k = ks + (lane >> 4);
          const double av = amask * arow[k];
          const double bv = Us[k * UST + col];
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }

  // -- slab (this chunk) += partials ------------------------------------------
  double *slab = p.slabs + (size_t)blockIdx.x * p.slab_len;
  if (tid < RG) slab[K + (size_t)j0 * S + tid] += accN1;
  double *slabM = slab + K + (size_t)K * S + (size_t)j0 * SS;
#pragma unroll
  for (int e = 0; e < MAXM; ++e) {
    const int x = tid + e * kStatsThreads;
    if (x < JGc * SS) slabM[x] += accM[e];
  }
  double *slabU = slab + K + (size_t)K * S + (size_t)K * SS + 2;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = wave + t * kStatsWaves;
    if (tile < ntiles) {
      const int mt = tile % MT, nt = tile / MT;
      const int col = nt * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + (lane >> 4) + 4 * r;
        if (row < RG && col < NU) slabU[((size_t)j0 * S + row) * NU + col] += acc[t][r];
      }
    }
  }
  (void)invS;
}

// 256 threads = 32 columns x 8 slab partitions: partition p sums slabs
// p, p+8, p+16, ... (coalesced 256-B rows), then the 8 partials are added in
// fixed order -- deterministic, and ~slab_len/32 blocks fill the chip.
constexpr int kFinalCols = 32, kFinalParts = 8;
__global__ __launch_bounds__(256) void stats_final_kernel(const double *slabs, int nslab,
                                                          int slab_len, double *out) {
  __shared__ double part[kFinalParts][kFinalCols];
  const int c = threadIdx.x % kFinalCols, pp = threadIdx.x / kFinalCols;
  const int x = blockIdx.x * kFinalCols + c;
  double acc = 0.0;
  if (x < slab_len)
    for (int k = pp; k < nslab; k += kFinalParts) acc += slabs[(size_t)k * slab_len + x];
  part[pp][c] = acc;
  __syncthreads();
  if (pp == 0 && x < slab_len) {
    double s = part[0][c];
#pragma unroll
    for (int q = 1; q < kFinalParts; ++q) s += part[q][c];
    out[x] = s;
  }
}

// ---------------------------------------------------------------------------
// planning + launch
// ---------------------------------------------------------------------------
namespace {
constexpr size_t kStatsLdsTarget = 64 * 1024;  // two 512-thread blocks per CU
constexpr int kMaxTPW = 16, kMaxM = 16;

size_t stats_lds_bytes(int RG, int AST, int NBB, int SBp, int UST, int JG, int NU) {
  return ((size_t)RG * AST + (size_t)NBB * SBp * UST + (size_t)NBB * JG) * sizeof(double) +
         (size_t)NU * sizeof(int);
}
}  // namespace

bool plan_stats(StatsArgs &a, size_t &lds, int &ngroups) {
  const int K = a.K, S = a.S;
  a.SBp = (a.SB + 3) / 4 * 4;
  const int NTL = (a.NU + 15) / 16;
  a.UST = NTL * 16;
  // clusters per row group: at most 128 rows, balanced over the groups
  int jg = std::max(1, 128 / S);
  ngroups = (K + jg - 1) / jg;
  jg = (K + ngroups - 1) / ngroups;
  a.JG = jg;
  const int RG = jg * S;
  const int ntiles = ((RG + 15) / 16) * NTL;
  if ((ntiles + kStatsWaves - 1) / kStatsWaves > kMaxTPW) return false;
  if ((jg * S * S + kStatsThreads - 1) / kStatsThreads > kMaxM) return false;
  if (RG > kStatsThreads) return false;
  int nbb = 8;
  for (; nbb >= 1; --nbb) {
    a.NBB = nbb;
    a.AST = nbb * a.SBp + 1;
    lds = stats_lds_bytes(RG, a.AST, nbb, a.SBp, a.UST, jg, a.NU);
    if (lds <= kStatsLdsTarget) break;
  }
  if (nbb < 1) {
    a.NBB = 1;
    a.AST = a.SBp + 1;
    lds = stats_lds_bytes(RG, a.AST, 1, a.SBp, a.UST, jg, a.NU);
    if (lds > 160 * 1024) return false;
  }
  return true;
}

template <int TPW, int MAXM>
static hipError_t launch_stats_t(const StatsArgs &a, int nchunk, int ngroups, size_t lds,
                                 hipStream_t st) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&stats_kernel<TPW, MAXM>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((stats_kernel<TPW, MAXM>), dim3(nchunk, ngroups), dim3(kStatsThreads), lds, st,
                     a);
  return hipGetLastError();
}

hipError_t launch_resp(const StatsArgs &a, int nchunk, hipStream_t st) {
  const size_t lds = ((size_t)(kRespThreads / 64) * (a.K + 2)) * sizeof(double);
  hipLaunchKernelGGL(resp_kernel, dim3(nchunk), dim3(kRespThreads), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_stats(const StatsArgs &a, int nchunk, int ngroups, size_t lds, hipStream_t st) {
  const int RG = a.JG * a.S;
  const int ntiles = ((RG + 15) / 16) * ((a.NU + 15) / 16);
  const int tpw = (ntiles + kStatsWaves - 1) / kStatsWaves;
  const int m = (a.JG * a.S * a.S + kStatsThreads - 1) / kStatsThreads;
  if (tpw <= 4 && m <= 4) return launch_stats_t<4, 4>(a, nchunk, ngroups, lds, st);
  if (tpw <= 8 && m <= 4) return launch_stats_t<8, 4>(a, nchunk, ngroups, lds, st);
  if (tpw <= 8) return launch_stats_t<8, 16>(a, nchunk, ngroups, lds, st);
  return launch_stats_t<16, 16>(a, nchunk, ngroups, lds, st);
}

hipError_t launch_stats_final(const double *slabs, int nslab, int slab_len, double *out,
                              hipStream_t st) {
  hipLaunchKernelGGL(stats_final_kernel, dim3((slab_len + kFinalCols - 1) / kFinalCols), dim3(256),
                     0, st, slabs, nslab, slab_len, out);
  return hipGetLastError();
}

}  // namespace vbhem

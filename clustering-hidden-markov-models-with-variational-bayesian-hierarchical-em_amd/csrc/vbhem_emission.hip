// vbhem_emission.hip -- K1, the expected emission log-likelihood of every
// (base state beta, cluster state sigma) of every (base i, cluster j) pair
// (mex.c:715-865), as one fp64 GEMM on v_mfma_f64_16x16x4f64:
//
//   E[(i,b),(j,s)] = -1/2 ( d log 2pi + c_s + <P_s, Sigma_b> + (mu_b - m_s)' P_s (mu_b - m_s) )
//                  = -1/2 ( bias_s + sum_e W[e][(j,s)] * U[e][(i,b)] )
//
// with every mean shifted by the same vector z (the average cluster mean; the
// quadratic form is shift-invariant, the shift keeps the expanded terms small):
//   full: U = [ Sigma_ab + Sigma_ba + 2 mu'_a mu'_b (a<b) | Sigma_aa + mu'_a^2 (a=b) , mu'_a ]
//         W = [ P_ab (packed upper, symmetrised)                              , -2 (P m')_a ]
//         bias = d log 2pi + c + m'' P m'
//   diag: U = [ Sigma_a + mu'_a^2 , mu'_a ],  W = [ P_a , -2 P_a m'_a ],  bias = d log 2pi + c + sum P_a m'_a^2
// (mu' = mu - z, m' = m - z; KD = d(d+1)/2 + d full, 2d diag).
//
// emission_prep_kernel builds W, bias and z once per call (K*S columns);
// emission_kernel streams the base set: every wavefront walks tiles of 16
// consecutive columns (i,b), builds its MFMA B operand U directly in registers
// from the covariances and means, and multiplies by W (LDS-resident when it
// fits, else read from L2) for all K*S rows.  Output layout E[(j,s)][(i - i_buf0) * Sb + b] (cluster-
// major rows): the MFMA tile stores 128-B row segments and fb_split_kernel's
// lanes (consecutive bases x base states) read contiguous 256-B runs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>

#include "vbhem_internal.h"
#include "vbhem_math.h"

namespace vbhem {

namespace {
typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void packed_ab(int e, int d, int &a, int &b) {
  a = 0;
  int k = e;
  while (k >= d - a) {
    k -= d - a;
    ++a;
  }
  b = a + k;
}
}  // namespace

// ---------------------------------------------------------------------------
// prep: z (mean of all cluster means), bias[K*S], W[KD][K*S]; one block per
// cluster row r = (j, s), threads over the packed entries (every block forms z
// in the same fixed order, block 0 publishes it).  Two per-call jobs ride along
// so they cost no launch of their own: row r's A' = exp(logA - rowmax) for the
// backward pass (p.Atg, gated schedule) and, in block 0, zeroing the fallback
// counters (p.zero_ints).
// ---------------------------------------------------------------------------
constexpr int kPrepThreads = 64;

__global__ __launch_bounds__(kPrepThreads) void emission_prep_kernel(EmissionArgs p) {
  __shared__ double zs[64], pm[64], zp[kPrepThreads];
  const int tid = threadIdx.x, d = p.d, KS = p.K * p.S, r = blockIdx.x;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  if (r == 0)
    for (int x = tid; x < p.n_zero; x += kPrepThreads) p.zero_ints[x] = 0;
  if (p.Atg && tid < p.S && r < KS) {
    const double *la = p.logA + (size_t)r * p.S;
    double mx = la[0];
    for (int s2 = 1; s2 < p.S; ++s2) mx = fmax(mx, la[s2]);
    p.Atg[(size_t)r * p.S + tid] = exp_nonpos(la[tid] - mx);
  }
  // z: coordinate a = tid % d, the rows q = part, part + NP, ... summed by thread
  // (a, part), then the NP parts of each coordinate in order (d <= 64).  Only
  // finite means count: a diverged cluster (NaN constants, e.g. one trial of a
  // batched launch) must not poison the shift, and so every other cluster's E.
  const int NP = kPrepThreads / d, part = tid / d, a0 = tid - part * d;
  if (p.zfix) {  // the shift the prepared operand U was built with
    for (int a = tid; a < d; a += kPrepThreads) {
      zs[a] = p.zfix[a];
      if (r == 0) p.shift[a] = zs[a];
    }
  } else if (part < NP) {
    double s = 0.0, n = 0.0;
    for (int q = part; q < KS; q += NP) {
      const double v = p.m[(size_t)q * d + a0];
      if (isfinite(v)) {
        s += v;
        n += 1.0;
      }
    }
    zp[tid] = s;
    pm[tid] = n;
  }
  __syncthreads();
  for (int a = tid; a < d && !p.zfix; a += kPrepThreads) {
    double s = 0.0, n = 0.0;
    for (int q = 0; q < NP; ++q) {
      s += zp[q * d + a];
      n += pm[q * d + a];
    }
    zs[a] = n > 0.0 ? s / n : 0.0;
    if (r == 0) p.shift[a] = zs[a];
  }
  __syncthreads();  // zs published; pm is reused below
  // W' = -W/2 and bias' = -bias/2 (exact scalings), so E = bias' + sum W' U;
  // rows r >= K*S and k-rows e >= KD are the zero padding of the [kdp][ksp] layout
  const int KSP = p.ksp;
  double *Wc = p.W + r;  // column r, row stride ksp
  if (r >= KS) {
    for (int e = tid; e < p.kdp; e += kPrepThreads) Wc[(size_t)e * KSP] = 0.0;
    if (tid == 0) p.bias[r] = 0.0;
    return;
  }
  for (int e = p.KD + tid; e < p.kdp; e += kPrepThreads) Wc[(size_t)e * KSP] = 0.0;
  const double *mr = p.m + (size_t)r * d;
  if (full) {
    const double *P = p.P + (size_t)r * d * d;
    for (int a = tid; a < d; a += kPrepThreads) {
      const double v = em_pm_full(P, mr, zs, a, d);  // (P_sym m')_a
      pm[a] = v;
      Wc[(size_t)(NPF + a) * KSP] = v;  // -(1/2)(-2 v)
    }
    for (int e = tid; e < NPF; e += kPrepThreads) {
      int a, b;
      packed_ab(e, d, a, b);
      Wc[(size_t)e * KSP] = em_w_full(P, a, b, d);
    }
    __syncthreads();
    if (tid == 0) {
      double q = 0.0;
      for (int a = 0; a < d; ++a) q = fma(mr[a] - zs[a], pm[a], q);
      p.bias[r] = em_bias(d, p.c[r], q);
    }
  } else {
    const double *P = p.P + (size_t)r * d;
    for (int a = tid; a < d; a += kPrepThreads) {
      const double ma = mr[a] - zs[a];
      Wc[(size_t)a * KSP] = -0.5 * P[a];
      Wc[(size_t)(d + a) * KSP] = P[a] * ma;  // -(1/2)(-2 P m')
    }
    if (tid == 0) {
      double q = 0.0;
      for (int a = 0; a < d; ++a) {
        const double ma = mr[a] - zs[a];
        q = fma(P[a] * ma, ma, q);
      }
      p.bias[r] = em_bias(d, p.c[r], q);
    }
  }
}

// ---------------------------------------------------------------------------
// The GEMM E[(j,s)][col] = bias'[(j,s)] + sum_e W'[e][(j,s)] U[e][col] on
// v_mfma_f64_16x16x4f64: operand A = W' (16 rows x 4 k), operand B = U (4 k x 16
// columns), C = 16 rows x 16 columns, lane l holding C[4v + (l>>4)][l & 15].
// Every wavefront independently walks tiles of 16 columns (i,b); rows are
// processed in chunks of 8 row tiles (32 fp64 accumulators per lane), all 8
// always issued (W' is zero-padded to a multiple of 128 rows).
// ---------------------------------------------------------------------------
constexpr int kEmRowChunk = 8;
constexpr int kEmRawChunk = 4;  // raw kernel: 4 row tiles per chunk (register budget)
// doubles per wave: 16 cols x (d*d <= 64, d <= 8), rows padded to an odd stride
// (dd + 1, d + 1) so the 16 lanes of a k-group read 16 different bank pairs
constexpr int kEmRawSlot = 16 * 65 + 16 * 9;

constexpr int kEmMaxThreads = 512;

// emission_raw_kernel<KQ, WL, SM> (d <= 8): the tile's raw covariances and means
// are loaded with coalesced 16-B loads, prefetched one tile ahead in registers,
// and committed to the wave's private LDS slot; each lane then forms its whole
// B operand U[4t + (l>>4)][l & 15], t < KQ, in registers from a per-lane operand
// descriptor (u = raw[oA] + raw[oB] + f mu'_a mu'_b + g mu'_a).  The k-loop is
// W' reads (LDS when WL, else L2) + MFMAs only; accumulators start at bias'.
// KQ = k-steps (compile time: no k-loop branches); SM: E /= smooth (VHEM).
template <int KQ, bool WL, bool SM>
__global__ __launch_bounds__(kEmMaxThreads) void emission_raw_kernel(EmissionArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NTH = blockDim.x, NW = NTH / 64;
  const int d = p.d, SB = p.SB, KS = p.K * p.S, KSP = p.ksp;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  const int dd = full ? d * d : d;
  const int ncols = (p.i_end - p.i_begin) * SB;
  const int nctile = (ncols + 15) / 16;
  double *bl = lds;                                    // [ksp] bias'
  double *Wl = bl + KSP;                               // [4 KQ][ksp] (WL)
  double *slots = Wl + (WL ? (size_t)4 * KQ * KSP : 0);
  double *slot = slots + wave * kEmRawSlot;
  double *zsh = slots + NW * kEmRawSlot;               // [d] the shift z
  const int dds = dd | 1, ds = d | 1;                  // odd row strides
  double *rawc = slot;                                 // [16][dds], [dd] = 0
  double *mus = slot + 16 * dds;                       // [16][ds] (shifted by z)
  for (int a = tid; a < d; a += NTH) zsh[a] = p.shift[a];
  for (int x = tid; x < KSP; x += NTH) bl[x] = p.bias[x];
  if (WL)
    for (int x = tid; x < 4 * KQ * KSP; x += NTH) Wl[x] = p.W[x];
  const int kl = lane >> 4, cl = lane & 15;
  // this lane's operand descriptors, k-rows e = 4t + kl (e >= KD: u = 0)
  int desc[KQ];
#pragma unroll
  for (int t = 0; t < KQ; ++t) {
    const int e = 4 * t + kl;
    int a = 0, b = 0, kind = 4;
    if (e < NPF) {
      a = b = e;
      if (full) packed_ab(e, d, a, b);
      kind = full ? (a == b ? 0 : 1) : 2;
    } else if (e < NPF + d) {
      a = b = e - NPF;
      kind = 3;
    }
    const int z = dd;  // the zero slot of a padded covariance row
    const int oA = kind == 0 ? a * d + a : kind == 1 ? a * d + b : kind == 2 ? a : z;
    const int oB = kind == 1 ? b * d + a : z;
    const int f = kind == 1 ? 2 : (kind == 3 || kind == 4) ? 0 : 1, g = kind == 3 ? 1 : 0;
    desc[t] = oA | (oB << 7) | (a << 14) | (b << 18) | (f << 22) | (g << 24);
  }
  __syncthreads();
  const size_t ldE = (size_t)p.e_ld;
  const int wstride = gridDim.x * NW;
  int ct = blockIdx.x * NW + wave;

  // register prefetch of a tile's raw covariances (16 cols x dd <= 1024 doubles) and
  // means (16 x d <= 128): 8 + 1 double2 per lane, fully coalesced
  constexpr int kPre = 8;
  double2 pre_c[kPre], pre_m;
  auto prefetch = [&](int t) {
    const int c0 = t * 16;
    const int ccount = min(16, ncols - c0);
    const size_t g0 = (size_t)p.i_begin * SB + c0;
    const double2 *src = reinterpret_cast<const double2 *>(p.covars + g0 * dd);
    const int n2 = ccount * dd / 2;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {  // clamped, unconditional loads (no branch + wait)
      const int x = lane + 64 * k;
      const double2 v = src[x < n2 ? x : 0];
      pre_c[k] = (x < n2) ? v : make_double2(0.0, 0.0);
    }
    const double2 *ms = reinterpret_cast<const double2 *>(p.centres + g0 * d);
    const int nm2 = ccount * d / 2;
    const double2 vm = ms[lane < nm2 ? lane : 0];
    pre_m = lane < nm2 ? vm : make_double2(0.0, 0.0);
  };
  if (ct < nctile) prefetch(ct);
  const double *Wsrc = WL ? Wl : p.W;

  for (; ct < nctile; ct += wstride) {
    const int c0 = ct * 16;
    const int ccount = min(16, ncols - c0);
    const bool cv = cl < ccount;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // previous tile's LDS reads done
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int x = lane + 64 * k;  // elements 2x, 2x+1 of the tile's [16][dd] block
      if (x < 8 * dd) {
        const int c = (2 * x) / dd, o = 2 * x - c * dd;  // dd even: the pair stays in a row
        rawc[c * dds + o] = pre_c[k].x;
        rawc[c * dds + o + 1] = pre_c[k].y;
      }
    }
    if (lane < 16) rawc[lane * dds + dd] = 0.0;  // the zero slot of every column
    if (lane < 8 * d) {
      const int c = (2 * lane) / d, o = 2 * lane - c * d;
      mus[c * ds + o] = pre_m.x - zsh[o];
      mus[c * ds + o + 1] = pre_m.y - zsh[o + 1];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (ct + wstride < nctile) prefetch(ct + wstride);  // next tile, overlaps the MFMAs
    double ub[KQ];
#pragma unroll
    for (int t = 0; t < KQ; ++t) {
      const int tb = desc[t];
      const int oA = tb & 127, oB = (tb >> 7) & 127, a = (tb >> 14) & 15, b = (tb >> 18) & 15;
      const double f = (double)((tb >> 22) & 3), g = (double)((tb >> 24) & 1);
      const double ma = mus[cl * ds + a], mb = mus[cl * ds + b];
      const double caa = rawc[cl * dds + oA] + rawc[cl * dds + oB];
      const double u = fma(f * ma, mb, fma(g, ma, caa));
      ub[t] = cv ? u : 0.0;
    }
    double *Ec = p.E + (size_t)(p.i_begin - p.i_buf0) * SB + c0 + cl;  // this lane's column
    // row stride laundered per tile: otherwise the 32 loop-invariant row offsets
    // (64-bit) are hoisted out of the tile loop and the kernel spills
    size_t ldT = ldE;
    int kspT = KSP;
    asm volatile("" : "+s"(ldT), "+s"(kspT));
    for (int r0 = 0; r0 < KSP; r0 += 16 * kEmRawChunk) {
      double4_t acc[kEmRawChunk];
      const double *br = bl + r0 + kl;
      asm volatile("" : "+v"(br));
#pragma unroll
      for (int q = 0; q < kEmRawChunk; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[q][v] = br[q * 16 + 4 * v];
      double wc[kEmRawChunk], wn[kEmRawChunk];
      const double *Wr = Wsrc + (size_t)kl * kspT + r0 + cl;
      asm volatile("" : "+v"(Wr));
#pragma unroll
      for (int q = 0; q < kEmRawChunk; ++q) wc[q] = Wr[q * 16];
#pragma unroll
      for (int t = 0; t < KQ; ++t) {
        if (t + 1 < KQ) {
#pragma unroll
          for (int q = 0; q < kEmRawChunk; ++q) wn[q] = Wr[(size_t)4 * (t + 1) * kspT + q * 16];
        }
#pragma unroll
        for (int q = 0; q < kEmRawChunk; ++q)
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(wc[q], ub[t], acc[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < kEmRawChunk; ++q) wc[q] = wn[q];
      }
      if (cv) {
#pragma unroll
        for (int q = 0; q < kEmRawChunk; ++q)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int row = r0 + q * 16 + kl + 4 * v;
            if (row < KS) Ec[(size_t)row * ldT] = SM ? acc[q][v] / p.smooth : acc[q][v];
          }
      }
    }
  }
}

// emission_gen_kernel<WL> (d > 8): operand B formed per k-step from the column's
// covariances and means read through L1/L2.
template <bool WL>
__global__ __launch_bounds__(kEmMaxThreads) void emission_gen_kernel(EmissionArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NTH = blockDim.x, NW = NTH / 64;
  const int d = p.d, SB = p.SB, KS = p.K * p.S, KD = p.KD, KSP = p.ksp;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  const int dd = full ? d * d : d;
  const int KQ = p.kdp / 4;
  const int ncols = (p.i_end - p.i_begin) * SB;
  const int nctile = (ncols + 15) / 16;
  int *tab = reinterpret_cast<int *>(lds);                 // [KD] packed operand descriptor
  double *Wl = lds + (KD + 1) / 2 + 1;                     // [kdp][ksp] (WL)
  if (WL)
    for (int x = tid; x < p.kdp * KSP; x += NTH) Wl[x] = p.W[x];
  for (int e = tid; e < KD; e += NTH) {
    int a, b, kind;
    if (e < NPF) {
      a = b = e;
      if (full) packed_ab(e, d, a, b);
      kind = full ? (a == b ? 0 : 1) : 2;
    } else {
      a = b = e - NPF;
      kind = 3;
    }
    tab[e] = a | (b << 8) | (kind << 16);
  }
  __syncthreads();
  const int kl = lane >> 4, cl = lane & 15;
  const size_t ldE = (size_t)p.e_ld;
  const int wstride = gridDim.x * NW;
  const double *Wsrc = WL ? Wl : p.W;
  for (int ct = blockIdx.x * NW + wave; ct < nctile; ct += wstride) {
    const int c0 = ct * 16;
    const int ccount = min(16, ncols - c0);
    const int col = c0 + cl;
    const bool cv = cl < ccount;
    const size_t g0 = (size_t)p.i_begin * SB + c0;
    const double *Cg = p.covars + (g0 + (cv ? cl : 0)) * dd;
    const double *Mg = p.centres + (g0 + (cv ? cl : 0)) * d;
    const size_t cbuf = (size_t)(p.i_begin - p.i_buf0) * SB + col;
    for (int r0 = 0; r0 < KSP; r0 += 16 * kEmRowChunk) {
      double4_t acc[kEmRowChunk];
#pragma unroll
      for (int q = 0; q < kEmRowChunk; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[q][v] = p.bias[r0 + q * 16 + kl + 4 * v];
      double wc[kEmRowChunk], wn[kEmRowChunk];
      const double *Wr = Wsrc + (size_t)kl * KSP + r0 + cl;
#pragma unroll
      for (int q = 0; q < kEmRowChunk; ++q) wc[q] = Wr[q * 16];
      for (int t = 0; t < KQ; ++t) {
        if (t + 1 < KQ) {
#pragma unroll
          for (int q = 0; q < kEmRowChunk; ++q) wn[q] = Wr[(size_t)4 * (t + 1) * KSP + q * 16];
        }
        const int e = 4 * t + kl;
        double u = 0.0;
        if (e < KD) {
          const int tb = tab[e];
          const int a = tb & 0xff, b = (tb >> 8) & 0xff, kind = tb >> 16;
          const double ma = Mg[a] - p.shift[a], mb = Mg[b] - p.shift[b];
          double caa = kind <= 1 ? Cg[a * d + b] : (kind == 2 ? Cg[a] : 0.0);
          if (kind == 1) caa += Cg[b * d + a];
          u = kind == 3 ? ma : (kind == 1 ? fma(2.0 * ma, mb, caa) : fma(ma, ma, caa));
          u = cv ? u : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kEmRowChunk; ++q)
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(wc[q], u, acc[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < kEmRowChunk; ++q) wc[q] = wn[q];
      }
      if (cv) {
#pragma unroll
        for (int q = 0; q < kEmRowChunk; ++q)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int row = r0 + q * 16 + kl + 4 * v;
            if (row < KS) {
              const double ev = acc[q][v];
              p.E[(size_t)row * ldE + cbuf] = p.smooth != 1.0 ? ev / p.smooth : ev;
            }
          }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The prepared operand U (vbhem_prepare_base, or per call for the bases a call
// processes) and the GEMM on it.
//
// u_shift_kernel: z = mean of the centres of every valid base state (i, b < nstates[i])
//   of [0, N): phase 0 -- block q sums a fixed contiguous column range; phase 1 -- one
//   block adds the partials in block order (fixed order: bit-reproducible).
// u_prep_kernel: one block per column tile writes the tile's kq * 64 doubles in MFMA
//   B-operand lane order (vbhem_internal.h, kUHead):
//   full: u(e, col) = Sigma_ab + Sigma_ba + 2 mu'_a mu'_b (a < b) | Sigma_aa + mu'_a^2 (e < NPF),
//         mu'_(e - NPF) (e < NPF + d);   diag: Sigma_e + mu'_e^2 | mu'_(e - d);   mu' = mu - z.
// emission_u_kernel<KQB, RC>: E = bias' + W'^T U, persistent over rounds of one 16-column
//   tile per wavefront: the tile's U (kq <= KQB doubles per lane) is loaded once into
//   registers (coalesced: 512 B per k-step); W' is staged in LDS in A-operand lane order,
//   RC row tiles (16 rows each) per chunk -- once per block when every row fits one chunk
//   (K*S <= 128 at kq <= 12), else chunk by chunk per round; accumulators start at bias'.
//   Nothing of the base set is recomputed per cluster row chunk, W' is never read from L2
//   per k-step (the raw/generic kernels' costs at d > 8).
// ---------------------------------------------------------------------------
constexpr int kUShiftBlocks = 256;
constexpr int kUThreads = 256;

__global__ __launch_bounds__(kUThreads) void u_shift_kernel(UPrepArgs p, int phase, int nblk) {
  __shared__ double sp[kUThreads], sn[kUThreads];
  const int tid = threadIdx.x, d = p.d;
  const int P = kUThreads / d, part = tid / d, a = tid - part * d;
  double *partial = p.U + kUHead;  // [nblk][d + 1] (the tile area, rewritten later)
  double s = 0.0, n = 0.0;
  if (phase == 0) {
    const long long ncol = (long long)p.N * p.SB;
    const long long per = (ncol + gridDim.x - 1) / gridDim.x;
    const long long c0 = (long long)blockIdx.x * per, c1 = min(ncol, c0 + per);
    if (part < P) {
      for (long long col = c0 + part; col < c1; col += P) {
        const int i = (int)(col / p.SB), b = (int)(col - (long long)i * p.SB);
        const int ns = p.nstates ? p.nstates[i] : p.SB;
        if (b < ns) {
          s += p.centres[col * d + a];
          n += 1.0;
        }
      }
    }
  } else if (part < P) {
    for (int q = part; q < nblk; q += P) {
      s += partial[(size_t)q * (d + 1) + a];
      n += (a == 0) ? partial[(size_t)q * (d + 1) + d] : 0.0;
    }
  }
  sp[tid] = s;
  sn[tid] = n;
  __syncthreads();
  if (tid < d) {
    double ss = 0.0, nn = 0.0;
    for (int q = 0; q < P; ++q) {
      ss += sp[q * d + tid];
      nn += sn[q * d + (phase == 0 ? tid : 0)];
    }
    if (phase == 0) {
      partial[(size_t)blockIdx.x * (d + 1) + tid] = ss;
      if (tid == 0) partial[(size_t)blockIdx.x * (d + 1) + d] = nn;
    } else {
      p.U[tid] = nn > 0.0 ? ss / nn : 0.0;
    }
  }
  if (phase == 1)
    for (int x = d + tid; x < kUHead; x += kUThreads) p.U[x] = 0.0;
}

__global__ __launch_bounds__(kUThreads) void u_prep_kernel(UPrepArgs p) {
  __shared__ double zs[kUHead];
  const int tid = threadIdx.x, d = p.d, SB = p.SB, kq = p.kdp / 4;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  const int dd = full ? d * d : d;
  const double *z = p.z ? p.z : p.U;
  for (int a = tid; a < d; a += kUThreads) zs[a] = z[a];
  __syncthreads();
  const long long tile = blockIdx.x;
  const long long c_begin = (long long)p.i_begin * SB, c_end = (long long)p.i_end * SB;
  double *Ut = p.U + kUHead + (size_t)tile * kq * 64;
  for (int x = tid; x < kq * 64; x += kUThreads) {
    const int t = x >> 6, l = x & 63, kl = l >> 4, cl = l & 15;
    const int e = 4 * t + kl;
    const long long col = p.u_col0 + tile * 16 + cl;
    double u = 0.0;
    if (col >= c_begin && col < c_end) {
      const double *C = p.covars + (size_t)col * dd;
      const double *mu = p.centres + (size_t)col * d;
      if (e < NPF) {
        int a = e, b = e;
        if (full) packed_ab(e, d, a, b);
        const double ma = mu[a] - zs[a], mb = mu[b] - zs[b];
        if (!full) u = fma(ma, ma, C[a]);
        else if (a == b) u = fma(ma, ma, C[a * d + a]);
        else u = fma(2.0 * ma, mb, C[a * d + b] + C[b * d + a]);
      } else if (e < NPF + d) {
        u = mu[e - NPF] - zs[e - NPF];
      }
    }
    Ut[x] = u;
  }
}

// us_build_kernel: the statistics copy Us (vbhem_internal.h), one thread per entry
// (grid-stride), the same moment arithmetic as u_prep_kernel.
__global__ __launch_bounds__(kUThreads) void us_build_kernel(UPrepArgs p, double *Us) {
  __shared__ double zs[kUHead];
  const int tid = threadIdx.x, d = p.d, SB = p.SB;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d, NU = 1 + d + NPF;
  const int SBP = us_sbp(SB), NUP = us_nup(NU);
  const int dd = full ? d * d : d;
  for (int a = tid; a < d; a += kUThreads) zs[a] = p.U[a];
  __syncthreads();
  const long long n = (long long)p.N * SBP * NUP;
  for (long long x = (long long)blockIdx.x * kUThreads + tid; x < n; x += (long long)gridDim.x * kUThreads) {
    const long long i = x / (SBP * NUP);
    const int r = (int)(x - i * (SBP * NUP)), ft = r / (SBP * 16), q = r - ft * SBP * 16;
    const int b = q >> 4, f = 16 * ft + (q & 15);
    double u = 0.0;
    if (b < SB && f < NU) {
      const long long col = i * SB + b;
      const double *mu = p.centres + (size_t)col * d;
      if (f == 0) {
        u = 1.0;
      } else if (f <= d) {
        u = mu[f - 1] - zs[f - 1];
      } else {
        const double *C = p.covars + (size_t)col * dd;
        const int e = f - 1 - d;
        int a = e, bb = e;
        if (full) packed_ab(e, d, a, bb);
        const double ma = mu[a] - zs[a], mb = mu[bb] - zs[bb];
        if (!full) u = fma(ma, ma, C[a]);
        else if (a == bb) u = fma(ma, ma, C[a * d + a]);
        else u = fma(2.0 * ma, mb, C[a * d + bb] + C[bb * d + a]);
      }
    }
    Us[x] = u;
  }
}

#ifndef UNWAVE_MAXT
#define UNWAVE_MAXT 512  // launch bound of emission_u_kernel (threads per block)
#endif
typedef unsigned int em_u2 __attribute__((ext_vector_type(2)));

// BST (the PF path): E stores as buffer stores, a lane outside the tile carrying an
// out-of-range offset instead of a branch, and the next round's U loads branch-free
// (clamped), so the wait for those loads counts the stores issued after them exactly
// instead of draining every store of the round at a join (E < 4 GB: the launcher)
template <int KQB, int RC, int NTW, bool EXACT, bool PF = false, int SPL = 1, bool BST = false>
__global__ __launch_bounds__(UNWAVE_MAXT) void emission_u_kernel(EmissionArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NT = blockDim.x, NW = NT >> 6;
  const int kq = EXACT ? KQB : p.kdp / 4, KS = p.K * p.S, SB = p.SB;
  const int nrt = p.ksp / 16, nchunk = nrt / RC;
  double *Wl = lds;                            // [kq][RC][64] W' chunk, A-operand lane order
  double *bl = Wl + (size_t)kq * RC * 64;      // [RC * 16] bias' of the chunk
  const long long c_begin = (long long)p.i_begin * SB, c_end = (long long)p.i_end * SB;
  const long long t_first = (c_begin - p.u_col0) / 16;
  const long long t_last = (c_end - p.u_col0 + 15) / 16;
  const long long per_round = (long long)gridDim.x * NW * NTW;
  const long long rounds = (t_last - t_first + per_round - 1) / per_round;
  const int kl = lane >> 4, cl = lane & 15;
  const size_t ldE = (size_t)p.e_ld;
  const double sm = p.smooth;
  const bool vhem = __builtin_amdgcn_readfirstlane((int)(sm != 1.0)) != 0;
  // E entry of row ub + kl at the lane's byte offset bofs (< 4 GB within a base group):
  // a wave-uniform row base plus a 32-bit lane offset (chunked path: fewer VALU address
  // operations per store than a 64-bit row x stride product)
  auto e_at = [&](int ub, unsigned bofs) -> double & {
    const char *rb = reinterpret_cast<const char *>(p.E) + (size_t)ub * ldE * sizeof(double);
    return *reinterpret_cast<double *>(const_cast<char *>(rb) + bofs);
  };
  typedef __attribute__((address_space(3))) void *lds_ptr;
  typedef __attribute__((address_space(1))) void *glb_ptr;
  auto stage = [&](int ch) {
    __syncthreads();  // the previous chunk's reads are done
    // W' chunk straight from L2 into LDS (global_load_lds_dwordx4: lane j lands at
    // block + 16 j), 1 KB = two A-operand rows per wave instruction, no register
    // round trip and one wait for the whole chunk
    const int nblk = kq * RC / 2;
    for (int b = wave; b < nblk; b += NW) {
      const int x = b * 128 + 2 * lane;
      const int t = x / (RC * 64), rem = x - t * (RC * 64), rt = rem >> 6, l = rem & 63;
      const int row = (ch * RC + rt) * 16 + (l & 15), e = 4 * t + (l >> 4);
      __builtin_amdgcn_global_load_lds((glb_ptr)(p.W + (size_t)e * p.ksp + row),
                                       (lds_ptr)(Wl + (size_t)b * 128), 16, 0, 0);
    }
    for (int x = tid; x < RC * 16; x += NT) bl[x] = p.bias[ch * RC * 16 + x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  if (nchunk == 1) stage(0);
  if constexpr (PF) {  // NTW == 1, W' in one chunk (the launcher checks)
    {
      // W' resident for the whole kernel: the next round's tile of U is loaded while
      // this round's MFMAs run (one item per wave, double-buffered in registers).  An
      // item is a 16-column tile's RC / SPL row tiles: SPL = 2 for small base counts
      // (a 12,500-base shard: 6,250 tiles on 3,072 waves ran as 3 rounds for 2.03 of
      // work; as 12,500 half-tiles, 5 rounds for 4.07), each half reading the tile's U
      constexpr int RCI = RC / SPL;
      const long long nitem = (t_last - t_first) * SPL;
      const long long rounds_i = (nitem + per_round - 1) / per_round;
      auto item_at = [&](long long r) { return r * per_round + (long long)blockIdx.x * NW + wave; };
      auto load_u = [&](long long r, double (&u)[KQB]) {
        const long long it = item_at(r);
        const long long tile = t_first + (it < nitem ? it / SPL : 0);
        const double *Ut = p.U + kUHead + (size_t)tile * kq * 64 + lane;
        if constexpr (BST) {
          // (t past kq: a repeat of the last slice, never used)
#pragma unroll
          for (int t = 0; t < KQB; ++t) u[t] = Ut[(size_t)min(t, kq - 1) * 64];
        } else {
#pragma unroll
          for (int t = 0; t < KQB; ++t) u[t] = t < kq ? Ut[(size_t)t * 64] : 0.0;
        }
      };
      __amdgpu_buffer_rsrc_t re;
      if constexpr (BST)
        re = __builtin_amdgcn_make_buffer_rsrc(p.E, (short)0, (int)(unsigned)((size_t)KS * ldE * 8), 0x00020000);
      double u[KQB], un[KQB];
      if (rounds_i > 0) load_u(0, u);
#pragma unroll 1
      for (long long r = 0; r < rounds_i; ++r) {
        const long long it = item_at(r);
        const long long tile = t_first + it / SPL;
        const int q0 = SPL == 1 ? 0 : (int)(it % SPL) * RCI;
        const long long col = p.u_col0 + tile * 16 + cl;
        const bool cv = it < nitem && col >= c_begin && col < c_end;
        double *Ec = p.E + (cv ? col - (long long)p.i_buf0 * SB : 0);
        if constexpr (BST) load_u(r + 1, un);  // (past the last round: a repeat, unused)
        else if (r + 1 < rounds_i) load_u(r + 1, un);
        // W' is loop-invariant: an opaque offset keeps its LDS reads in the loop
        // (hoisted, 88 values would take 176 VGPRs)
        int woff = lane + q0 * 64, boff = kl + q0 * 16;
        asm volatile("" : "+v"(woff), "+v"(boff));
        double4_t acc[RCI];
#pragma unroll
        for (int q = 0; q < RCI; ++q)
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[q][v] = bl[q * 16 + boff + 4 * v];
#pragma unroll
        for (int t = 0; t < KQB; ++t) {
          if (t < kq) {
#pragma unroll
            for (int q = 0; q < RCI; ++q)
              acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(Wl[(t * RC + q) * 64 + woff], u[t], acc[q],
                                                            0, 0, 0);
          }
        }
        if constexpr (BST) {
          const unsigned cofs = (unsigned)(cv ? col - (long long)p.i_buf0 * SB : 0) * 8u;
          auto put = [&](int row, double x) {
            const unsigned off = (cv && row < KS) ? cofs + (unsigned)row * (unsigned)ldE * 8u : 0xfffffff8u;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(em_u2, x), re, (int)off, 0, 0);
          };
          // the VHEM division behind a uniform branch (both sides: the same stores)
          if (vhem) {
#pragma unroll
            for (int q = 0; q < RCI; ++q)
#pragma unroll
              for (int v = 0; v < 4; ++v) put((q0 + q) * 16 + kl + 4 * v, acc[q][v] / sm);
          } else {
#pragma unroll
            for (int q = 0; q < RCI; ++q)
#pragma unroll
              for (int v = 0; v < 4; ++v) put((q0 + q) * 16 + kl + 4 * v, acc[q][v]);
          }
        } else if (cv) {
          // the VHEM division (hem_hmm_bwd_fwd_mex.c:848-860) behind a uniform branch:
          // written as a select, the full fp64 division ran for every stored value
          if (vhem) {
#pragma unroll
            for (int q = 0; q < RCI; ++q)
#pragma unroll
              for (int v = 0; v < 4; ++v) {
                const int row = (q0 + q) * 16 + kl + 4 * v;
                if (row < KS) Ec[(size_t)row * ldE] = acc[q][v] / sm;
              }
          } else {
#pragma unroll
            for (int q = 0; q < RCI; ++q)
#pragma unroll
              for (int v = 0; v < 4; ++v) {
                const int row = (q0 + q) * 16 + kl + 4 * v;
                if (row < KS) Ec[(size_t)row * ldE] = acc[q][v];
              }
          }
        }
#pragma unroll
        for (int t = 0; t < KQB; ++t) u[t] = un[t];
      }
    }
  } else {
  for (long long r = 0; r < rounds; ++r) {
    // NTW column tiles per wave: each staged W' chunk feeds NTW * RC MFMAs per k-step
    double u[NTW][KQB];
    unsigned lofs[NTW];  // 32-bit lane byte offsets of the stores (e_at)
    bool cv[NTW];
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const long long tile = t_first + r * per_round + ((long long)blockIdx.x * NW + wave) * NTW + n;
      const bool tv = tile < t_last;
      const double *Ut = p.U + kUHead + (size_t)(tv ? tile : t_first) * kq * 64 + lane;
#pragma unroll
      for (int t = 0; t < KQB; ++t) {  // kq is uniform: a scalar branch, no load past the tile
        if (t < kq) u[n][t] = Ut[(size_t)t * 64];
        else u[n][t] = 0.0;
      }
      const long long col = p.u_col0 + tile * 16 + cl;
      cv[n] = tv && col >= c_begin && col < c_end;
      lofs[n] = ((unsigned)(cv[n] ? col - (long long)p.i_buf0 * SB : 0) + (unsigned)kl * (unsigned)ldE) * 8u;
    }
    for (int ch = 0; ch < nchunk; ++ch) {
      if (nchunk > 1) stage(ch);
      double4_t acc[NTW][RC];
#pragma unroll
      for (int q = 0; q < RC; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const double b = bl[q * 16 + kl + 4 * v];
#pragma unroll
          for (int n = 0; n < NTW; ++n) acc[n][q][v] = b;
        }
#pragma unroll
      for (int t = 0; t < KQB; ++t) {
        if (t < kq) {
#pragma unroll
          for (int q = 0; q < RC; ++q) {
            const double w = Wl[(t * RC + q) * 64 + lane];
#pragma unroll
            for (int n = 0; n < NTW; ++n)
              acc[n][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, u[n][t], acc[n][q], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int n = 0; n < NTW; ++n) {
        if (!cv[n]) continue;
        if (vhem) {  // (uniform: see above)
#pragma unroll
          for (int q = 0; q < RC; ++q)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int ub = (ch * RC + q) * 16 + 4 * v;
              if (ub + kl < KS) e_at(ub, lofs[n]) = acc[n][q][v] / sm;
            }
        } else {
#pragma unroll
          for (int q = 0; q < RC; ++q)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int ub = (ch * RC + q) * 16 + 4 * v;
              if (ub + kl < KS) e_at(ub, lofs[n]) = acc[n][q][v];
            }
        }
      }
    }
  }
  }
}

// emission_db_kernel<KQ, RC, NTW>: the chunked path (W' restaged per RC-row-tile chunk,
// C5's K S = 384 rows) with the chunks double-buffered in LDS and E written by buffer
// stores.  emission_u_kernel's chunked loop waits for everything in flight before it
// stages a chunk (s_waitcnt vmcnt(0)): the previous chunk's E stores included, which
// sat on the critical path (a timing build without the stores ran 1.65 vs 1.85 ms per
// C5 group).  Here chunk ch + 1's LDS-DMA is issued right after the
// barrier that opens chunk ch, and the wait before chunk ch + 1 counts only the E
// stores issued after that DMA -- every lane issues exactly NTW RC 4 of them per
// chunk (buffer stores; a column past the base range or a padding row carries an
// out-of-range offset and is dropped), so vmcnt(NTW RC 4) is exact.  Each chunk's
// buffer holds its W' row tiles in A-operand lane order and its RC 16 biases.  Same
// accumulation order as emission_u_kernel: the same E bits (checked bit for bit on
// C5, scripts/cmp_libs.py).  Measured (round 6, C5 N = 1500): 1.757 ms per emission
// launch against 1.864 for the chunked path (VBHEM_EM_NODB=1).
template <int KQ, int RC, int NTW>
__global__ __launch_bounds__(256) void emission_db_kernel(EmissionArgs p) {
  constexpr int CW = KQ * RC * 64;       // W' doubles per chunk
  constexpr int CB = CW + RC * 16;       // + its biases
  constexpr int NST = NTW * RC * 4;      // E stores per lane and chunk
  // the two chunk buffers as two LDS objects, the chunk loop unrolled by two so each
  // half reads one and fills the other: the compiler's LDS-DMA tracking can then see
  // that the DMA in flight does not write what the half reads (with one array indexed
  // by a runtime buffer number it waited for the DMA -- vmcnt(0) -- before the first
  // MFMA of every chunk)
  __shared__ __attribute__((aligned(16))) double buf0[CB];
  __shared__ __attribute__((aligned(16))) double buf1[CB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int NW = blockDim.x >> 6;
  const int KS = p.K * p.S, SB = p.SB;
  const int nchunk = p.ksp / 16 / RC;   // even (the launcher checks)
  const long long c_begin = (long long)p.i_begin * SB, c_end = (long long)p.i_end * SB;
  const long long t_first = (c_begin - p.u_col0) / 16;
  const long long t_last = (c_end - p.u_col0 + 15) / 16;
  const long long per_round = (long long)gridDim.x * NW * NTW;
  const long long rounds = (t_last - t_first + per_round - 1) / per_round;
  const int kl = lane >> 4, cl = lane & 15;
  const unsigned ldE8 = (unsigned)p.e_ld * 8u;
  typedef __attribute__((address_space(3))) void *lds_ptr;
  // chunk ch into dst: W' (two A-operand rows of 16 bytes per lane and wave
  // instruction) and, from wave 0's first lanes, its RC 16 biases
  // (written as inline asm: the builtin makes the compiler's LDS-DMA tracking wait for
  // the DMA in flight -- vmcnt(0) -- before the reads of the other buffer in one of the
  // two halves; the asm is invisible to it, and the waits above are explicit.  M0 takes
  // the wave's LDS destination, one wait state before the load reads it; nothing else
  // in this kernel uses M0, so it is not declared clobbered -- the compiler reserves it
  // and warns)
  auto dma = [&](int ch, double *dst) {
    constexpr int nblk = KQ * RC / 2;
    const unsigned base = (unsigned)(size_t)(lds_ptr)dst;
    for (int b = wave; b < nblk; b += NW) {
      const int x = b * 128 + 2 * lane;
      const int t = x / (RC * 64), rem = x - t * (RC * 64), rt = rem >> 6, l = rem & 63;
      const int row = (ch * RC + rt) * 16 + (l & 15), e = 4 * t + (l >> 4);
      const double *g = p.W + (size_t)e * p.ksp + row;
      const unsigned la = __builtin_amdgcn_readfirstlane(base + (unsigned)b * 1024u);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                   ::"v"(g), "s"(la) : "memory");
    }
    if (wave == 0 && lane < RC * 16 / 2) {
      const double *g = p.bias + ch * RC * 16 + 2 * lane;
      const unsigned la = __builtin_amdgcn_readfirstlane(base + (unsigned)CW * 8u);
      asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                   ::"v"(g), "s"(la) : "memory");
    }
  };
  const __amdgpu_buffer_rsrc_t re =
      __builtin_amdgcn_make_buffer_rsrc(p.E, (short)0, (int)(unsigned)((size_t)KS * p.e_ld * 8), 0x00020000);
  double u[NTW][KQ];
  unsigned cofs[NTW];
  bool cv[NTW];
  // one chunk: wait for its DMA, barrier, the next chunk's DMA into the other buffer,
  // the MFMAs from this one, the E stores
  auto chunk = [&](int ch, bool first, const double *Wl, double *other, int nch, bool more) {
    if (first) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the U tiles came after
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    // every wave's share landed and every wave's reads of the other buffer are done:
    // an execution barrier without __syncthreads' release fence, which would wait for
    // the E stores still in flight (vmcnt(0)) -- what this kernel avoids
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (more) dma(nch, other);
    const double *bl = Wl + CW;
    double4_t acc[NTW][RC];
#pragma unroll
    for (int q = 0; q < RC; ++q)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const double bv = bl[q * 16 + kl + 4 * v];
#pragma unroll
        for (int n = 0; n < NTW; ++n) acc[n][q][v] = bv;
      }
#pragma unroll
    for (int t = 0; t < KQ; ++t) {
#pragma unroll
      for (int q = 0; q < RC; ++q) {
        const double w = Wl[(t * RC + q) * 64 + lane];
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[n][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, u[n][t], acc[n][q], 0, 0, 0);
      }
    }
#pragma unroll
    for (int n = 0; n < NTW; ++n)
#pragma unroll
      for (int q = 0; q < RC; ++q)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = (ch * RC + q) * 16 + kl + 4 * v;
          const unsigned off = (cv[n] && row < KS) ? cofs[n] + (unsigned)row * ldE8 : 0xfffffff8u;
          // element by element: the store of a bit-cast vector element from the MFMA
          // accumulator compiled to element 0 four times (hipcc 7.2, seen in the ISA)
          const double x = acc[n][q][v];
          em_u2 bits;
          bits.x = (unsigned)__double2loint(x);
          bits.y = (unsigned)__double2hiint(x);
          __builtin_amdgcn_raw_buffer_store_b64(bits, re, (int)off, 0, 0);
        }
  };
  if (rounds > 0) dma(0, buf0);
#pragma unroll 1
  for (long long r = 0; r < rounds; ++r) {
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const long long tile = t_first + r * per_round + ((long long)blockIdx.x * NW + wave) * NTW + n;
      const bool tv = tile < t_last;
      const double *Ut = p.U + kUHead + (size_t)(tv ? tile : t_first) * KQ * 64 + lane;
#pragma unroll
      for (int t = 0; t < KQ; ++t) u[n][t] = Ut[(size_t)t * 64];
      const long long col = p.u_col0 + tile * 16 + cl;
      cv[n] = tv && col >= c_begin && col < c_end;
      cofs[n] = (unsigned)(cv[n] ? col - (long long)p.i_buf0 * SB : 0) * 8u;
    }
    const bool last = r + 1 == rounds;
#pragma unroll 1
    for (int ch = 0; ch < nchunk; ch += 2) {
      chunk(ch, ch == 0, buf0, buf1, ch + 1, true);
      // (the round's last chunk fills buf0 with the next round's chunk 0)
      chunk(ch + 1, false, buf1, buf0, ch + 2 < nchunk ? ch + 2 : 0, ch + 2 < nchunk || !last);
    }
  }
}

template <int KQ, int RC, int NTW>
static hipError_t launch_db_fn(const EmissionArgs &a, hipStream_t st) {
  if (a.kdp / 4 != KQ || (a.ksp / 16) % (2 * RC) != 0) return hipErrorInvalidValue;
  auto *fn = &emission_db_kernel<KQ, RC, NTW>;
  const size_t lds = 0;  // (static: the two chunk buffers)
  const int per_cu = resident_per_cu(reinterpret_cast<const void *>(fn), 256, lds);
  const long long c_begin = (long long)a.i_begin * a.SB, c_end = (long long)a.i_end * a.SB;
  const long long ntile = (c_end - a.u_col0 + 15) / 16 - (c_begin - a.u_col0) / 16;
  const long long want = (ntile + 4 * NTW - 1) / (4 * NTW);
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(want, (long long)device_cus() * per_cu));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_u_prep(const UPrepArgs &a, hipStream_t st) {
  if (a.d < 1 || a.d > kUHead || a.u_col0 % 16 != 0) return hipErrorInvalidValue;
  const long long c_end = (long long)a.i_end * a.SB;
  const long long ntile = u_tiles(c_end - a.u_col0);
  if (!a.z) {  // partial sums parked in the tile area (u_prep_kernel rewrites it)
    const long long area = ntile * (a.kdp / 4) * 64;
    const int nblk = (int)std::max<long long>(1, std::min<long long>(kUShiftBlocks, area / (a.d + 1)));
    hipLaunchKernelGGL(u_shift_kernel, dim3(nblk), dim3(kUThreads), 0, st, a, 0, nblk);
    hipLaunchKernelGGL(u_shift_kernel, dim3(1), dim3(kUThreads), 0, st, a, 1, nblk);
  }
  if (ntile > 0 && a.i_end > a.i_begin)
    hipLaunchKernelGGL(u_prep_kernel, dim3((unsigned)ntile), dim3(kUThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_us_build(const UPrepArgs &a, double *Us, hipStream_t st) {
  if (a.d < 1 || a.d > kUHead || a.N < 0) return hipErrorInvalidValue;
  const long long n = (long long)us_doubles(a.N, a.SB, a.d, a.covmode);
  if (n == 0) return hipSuccess;
  const long long nb = std::min<long long>((n + kUThreads - 1) / kUThreads, 16384);
  hipLaunchKernelGGL(us_build_kernel, dim3((unsigned)nb), dim3(kUThreads), 0, st, a, Us);
  return hipGetLastError();
}

#ifndef UNTW
#define UNTW 2
#endif
#ifndef UNWAVE_CHUNKED
#define UNWAVE_CHUNKED 4
#endif
#ifndef UNWAVE_SINGLE
#define UNWAVE_SINGLE 4  // 133 VGPRs at kq <= 12: 3 waves per SIMD, 4-wave blocks use them all
#endif
// the buffer-store path addresses E with 32-bit byte offsets (the fused E-step's base
// groups keep E below 4 GB; a caller's own buffer may not)
static bool em_bst_ok(const EmissionArgs &a) {
  return (unsigned long long)a.K * a.S * (unsigned long long)a.e_ld * 8ull < 0xfffffff0ull;
}

bool plan_emission_u(EmissionArgs &a, size_t &lds) {
  const int kq = a.kdp / 4;
  if (kq > kUMaxKq) {
    a.urc = 0;
    return false;
  }
  a.ukqb = kq <= 4 ? 4 : kq <= 12 ? 12 : kUMaxKq;
  a.urc = kq <= 12 ? 8 : 4;   // ksp / 16 is a multiple of 8: RC divides it
  // chunked W' (restaged every round): 4-wave blocks, two per CU, so one block's
  // staging overlaps the other's MFMAs
  a.nwave = a.ksp / 16 > a.urc ? UNWAVE_CHUNKED : UNWAVE_SINGLE;
  lds = ((size_t)kq * a.urc * 64 + (size_t)a.urc * 16) * sizeof(double);
  return true;
}

template <int KQB, int RC, int NTW, bool EXACT = false, bool PF = false, int SPL = 1, bool BST = false>
static hipError_t launch_u_fn(const EmissionArgs &a, size_t lds, hipStream_t st) {
  if (EXACT && a.kdp / 4 != KQB) return hipErrorInvalidValue;
  if (PF && (NTW != 1 || a.ksp / 16 != RC)) return hipErrorInvalidValue;
  if (SPL != 1 && !PF) return hipErrorInvalidValue;
  if (BST && !PF) return hipErrorInvalidValue;
  if constexpr (PF && !BST)
    if (em_bst_ok(a) && !std::getenv("VBHEM_EM_NOBST"))  // (A/B switch)
      return launch_u_fn<KQB, RC, NTW, EXACT, PF, SPL, true>(a, lds, st);
  auto *fn = &emission_u_kernel<KQB, RC, NTW, EXACT, PF, SPL, BST>;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  const int cus = device_cus();
  const int per_cu = resident_per_cu(reinterpret_cast<const void *>(fn), a.nwave * 64, lds);
  const long long c_begin = (long long)a.i_begin * a.SB, c_end = (long long)a.i_end * a.SB;
  const long long ntile = (c_end - a.u_col0 + 15) / 16 - (c_begin - a.u_col0) / 16;
  const long long want = (ntile * SPL + (long long)a.nwave * NTW - 1) / ((long long)a.nwave * NTW);
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(want, (long long)cus * per_cu));
  hipLaunchKernelGGL(fn, dim3(grid), dim3(a.nwave * 64), lds, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
bool plan_emission(EmissionArgs &a, size_t &lds) {
  const bool full = a.covmode == kCovFull;
  const int d = a.d;
  if (d > 64) return false;
  a.KD = full ? d * (d + 1) / 2 + d : 2 * d;
  a.kdp = emission_kdp(d, a.covmode);
  a.ksp = emission_ksp(a.K * a.S);
  const int dd = full ? d * d : d;
  a.wfull = (dd <= 64 && d <= 8 && dd % 2 == 0 && d % 2 == 0);  // RAW: tile staged in LDS
  // 8 waves per block with W' in LDS when it fits one block per CU, else 4 waves
  // reading W' through L1/L2
  const size_t wbytes = (size_t)a.kdp * a.ksp * sizeof(double);
  if (a.wfull) {
    const size_t head = ((size_t)a.ksp + d) * sizeof(double);
    const size_t slot = (size_t)kEmRawSlot * sizeof(double);
    a.wlds = head + wbytes + 8 * slot <= 160 * 1024;
    a.nwave = a.wlds ? 8 : 4;
    lds = head + (a.wlds ? wbytes : 0) + (size_t)a.nwave * slot;
  } else {
    const size_t head = ((size_t)(a.KD + 1) / 2 + 1) * sizeof(double);
    a.wlds = head + wbytes <= 160 * 1024;
    a.nwave = a.wlds ? 8 : 4;
    lds = head + (a.wlds ? wbytes : 0);
  }
  a.CB = 16;
  return true;
}

hipError_t launch_emission_prep(const EmissionArgs &a, hipStream_t st) {
  hipLaunchKernelGGL(emission_prep_kernel, dim3(a.ksp), dim3(kPrepThreads), 0, st, a);
  return hipGetLastError();
}

template <typename F>
static hipError_t launch_emission_fn(F *fn, const EmissionArgs &a, size_t lds, hipStream_t st) {
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  const int cus = device_cus();
  const int per_cu = resident_per_cu(reinterpret_cast<const void *>(fn), a.nwave * 64, lds);
  const int ncols = (a.i_end - a.i_begin) * a.SB;
  const int nctile = (ncols + 15) / 16;
  // persistent: every resident block, every wave walks 16-column tiles
  const unsigned grid = (unsigned)std::min((nctile + a.nwave - 1) / a.nwave, cus * per_cu);
  hipLaunchKernelGGL(fn, dim3(grid), dim3(a.nwave * 64), lds, st, a);
  return hipGetLastError();
}

template <int KQ>
static hipError_t launch_raw_kq(const EmissionArgs &a, size_t lds, hipStream_t st) {
  const bool sm = a.smooth != 1.0;
  if (a.wlds) return sm ? launch_emission_fn(&emission_raw_kernel<KQ, true, true>, a, lds, st)
                        : launch_emission_fn(&emission_raw_kernel<KQ, true, false>, a, lds, st);
  return sm ? launch_emission_fn(&emission_raw_kernel<KQ, false, true>, a, lds, st)
            : launch_emission_fn(&emission_raw_kernel<KQ, false, false>, a, lds, st);
}

// the one-chunk GEMM in half-tiles when the tiles fill fewer than 4 rounds of the
// device's waves (the last, partial round then costs a smaller share); above that the
// doubled U reads cost more than the finer tail saves.  VBHEM_EM_SPLIT=0 / 1 forces it.
static bool use_row_split(const EmissionArgs &a) {
  if (const char *ev = std::getenv("VBHEM_EM_SPLIT")) return std::atoi(ev) != 0;
  const long long ntile = ((long long)(a.i_end - a.i_begin) * a.SB + 15) / 16;
  const long long waves = (long long)device_cus() * 3 * a.nwave;  // 3 blocks per CU
  return ntile < 4 * waves;
}

hipError_t launch_emission(const EmissionArgs &a, size_t lds, hipStream_t st) {
  const int ncols = (a.i_end - a.i_begin) * a.SB;
  if (ncols <= 0) return hipSuccess;
  if (a.U && a.urc) {
    // W' in one chunk (K S <= 128): the double-buffered variant
    const bool one = a.ksp / 16 == a.urc && !std::getenv("VBHEM_NO_UPF");
    if (a.ukqb == 4) return one ? launch_u_fn<4, 8, 1, false, true>(a, lds, st) : launch_u_fn<4, 8, 1>(a, lds, st);
    if (a.ukqb == 12) {
      if (one && use_row_split(a))  // small base counts (shards): half-tiles, a finer last round
        return launch_u_fn<12, 8, 1, false, true, 2>(a, lds, st);
      return one ? launch_u_fn<12, 8, 1, false, true>(a, lds, st) : launch_u_fn<12, 8, 1>(a, lds, st);
    }
    // W' restaged per chunk: two column tiles per wave halve the staging per column
    if (a.kdp / 4 == 38) {  // d = 16 full (C5)
      // double-buffered chunks with buffer stores (E below 4 GB; VBHEM_EM_NODB: A/B)
      if (em_bst_ok(a) && (a.ksp / 16) % 4 == 0 && !std::getenv("VBHEM_EM_NODB"))
        return launch_db_fn<38, 2, 2>(a, st);
      return launch_u_fn<38, 4, UNTW, true>(a, lds, st);
    }
    return launch_u_fn<kUMaxKq, 4, UNTW>(a, lds, st);
  }
  if (a.wfull) {
    // KD = d(d+1)/2 + d (full) or 2d (diag), d <= 8 even: k-steps 2, 4, 7, 11 (full),
    // 1, 2, 3, 4 (diag)
    switch (a.kdp / 4) {
      case 1: return launch_raw_kq<1>(a, lds, st);
      case 2: return launch_raw_kq<2>(a, lds, st);
      case 3: return launch_raw_kq<3>(a, lds, st);
      case 4: return launch_raw_kq<4>(a, lds, st);
      case 7: return launch_raw_kq<7>(a, lds, st);
      case 11: return launch_raw_kq<11>(a, lds, st);
      default: return hipErrorInvalidValue;
    }
  }
  return a.wlds ? launch_emission_fn(&emission_gen_kernel<true>, a, lds, st)
                : launch_emission_fn(&emission_gen_kernel<false>, a, lds, st);
}

}  // namespace vbhem

// vbhem_stats.hip -- the fused E-step epilogue: responsibilities and the gated,
// Z-weighted statistic sums of one EM iteration (gfx950).
//
//   resp_kernel        hat_Z / Z = hat_Z * tilde_N per base (vbhem_h3m_c_step_fc.m:271-283)
//                      and the per-chunk partial sums Nj = sum_i Z (:282),
//                      Lt1 = sum Z .* L_elbo, Lt7 = sum hat_Z .* log(hat_Z)
//                      (vbhemh3m_lb.m:90, 107).
//   nm_kernel          streaming weighted sums over this chunk's bases
//                      (vbhem_compute_Statistics.m:33-55, gate Z > 1e-8):
//                        N1[j][s]    += g Z(i,j) sum_nu_1(i,j,s)
//                        M[j][s][r]  += g Z(i,j) sum_xi(i,j,s,r)
//   stats_kernel<..>   split-K reduction
//                        U[(j,s)][c] += sum_b (g Z(i,j) sum_t_nu(i,j,s,b)) u(i,b,c)
//                      with u = [1, mu, packed Sigma + mu mu'] -- the emission
//                      moments of mex.c:1348-1469 contracted over the base states
//                      and the bases at once: a (K*S) x (N*Sb) x NU GEMM on
//                      v_mfma_f64_16x16x4f64, K-dim streamed in batches of NBB bases.
//   gate_list_kernel / stats_list_kernel / stats_list_u_kernel  the gated schedule's
//                      per-cluster lists of pairs with Z > 1e-8 and the sums over
//                      them only (the base moments gathered from the covariances,
//                      or read from the emission GEMM's prepared operand U).
//   stats_final_kernel fixed-order sum of the per-chunk slabs.
//
// Grid: x = chunk of consecutive bases, y = group of JG clusters (rows j*S+s),
// so no tile is loaded twice; every block keeps its whole (JG*S) x NU output
// block in MFMA accumulators and its N1/M entries in registers.
// All sums run in a fixed order (no atomics): bit-reproducible.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "vbhem_internal.h"
#include "vbhem_exact.h"

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

constexpr double kGateZ = 1e-8;  // vbhem_compute_Statistics.m:35  (Z_Ni(i) > 1e-8)

// ---------------------------------------------------------------------------
// resp_kernel: one wavefront per base (lanes over clusters j).
// ---------------------------------------------------------------------------
#ifndef VBHEM_RESP_THREADS
#define VBHEM_RESP_THREADS 512  // 8 waves per chunk block: 2x the bases in flight (C4 -10 us)
#endif
constexpr int kRespThreads = VBHEM_RESP_THREADS;
constexpr int kRespFoldWaves = 4;  // folded fallback: worker wavefronts per chunk block

__device__ __forceinline__ double group_max(double v, int G) {
  for (int off = G >> 1; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ double group_sum(double v, int G) {
  for (int off = G >> 1; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

#ifndef VBHEM_RESP_UNROLL
#define VBHEM_RESP_UNROLL 1   // base steps of a wave unrolled (build switch for A/B)
#endif

// G = lanes per base (power of two >= K, <= 64): 64/G bases per wavefront step.
// (4 waves per SIMD: two chunk blocks per CU; the folded fallback must not raise it)
#ifndef VBHEM_RESP_WPE
#define VBHEM_RESP_WPE 4
#endif
typedef unsigned int resp_u2 __attribute__((ext_vector_type(2)));

// KP: K when it is a power of two <= 64 (every lane of a base group holds a cluster:
// the group reductions unroll and the stores need no lane mask), else 0
template <int KP>
__global__ __launch_bounds__(kRespThreads) __attribute__((amdgpu_waves_per_eu(VBHEM_RESP_WPE))) void resp_kernel(
    const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kRespThreads / 64;
  const int K = KP ? KP : p.K;
  int G = KP ? KP : 1;
  if (!KP)
    while (G < K && G < 64) G <<= 1;
  const int BPW = 64 / G;            // bases per wave step
  const int sub = lane / G, gl = lane - sub * G;
  double *accNj = lds;               // [NW*BPW][K]
  double *accLt = accNj + NW * BPW * K;  // [NW][2]
  int *gcnt = reinterpret_cast<int *>(accLt + 2 * NW);  // [K] gated pairs of this chunk
  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  if (p.fold) {
    // the folded fallback (vbhem_internal.h, kFlagHead): the backward pass's flagged
    // pairs of this block's bases get their exact L_elbo (and other outputs) before any
    // of them is read; block 0 records where the gate-list pass's entries will start.
    // The block's scratch slots: xslots / gridDim of them (the host folds only when
    // gridDim <= xslots); the queue borrows the accumulators' LDS before they are set
    int *fc = p.fx.flag_count;
    const int cnt = __atomic_load_n(fc, __ATOMIC_RELAXED);
    if (blockIdx.x == 0 && tid == 0) fc[3] = cnt;
    if (cnt > 0) {  // block-uniform
      const int nw = min(kRespFoldWaves, max(1, p.xslots / (int)gridDim.x));
      int *q = reinterpret_cast<int *>(lds), *qn = q + kRespThreads;
      auto mine = [&](int pair) { const int i = pair / K; return i >= b0 && i < b1; };
      if (exact_wave_in_lds(p.fx.S, p.fx.SB))
        fold_exact<false>(p.fx, 0, cnt, mine, p.xscratch, p.xstride, (int)blockIdx.x * nw, nw, q, qn,
                          lds + fold_lds_bytes(kRespThreads, 0, 1, 1) / sizeof(double));
      else
        fold_exact<true>(p.fx, 0, cnt, mine, p.xscratch, p.xstride, (int)blockIdx.x * nw, nw, q, qn,
                         nullptr);
    }
  }
  for (int x = tid; x < NW * BPW * K + 2 * NW; x += kRespThreads) accNj[x] = 0.0;
  for (int x = tid; x < K; x += kRespThreads) gcnt[x] = 0;
  __syncthreads();
  double l1 = 0.0, l7 = 0.0;
  if constexpr (KP > 0) {
    // K = G: a lane per cluster, 64 / K bases per wave step.  Two bases' loads in
    // flight behind the one being computed (two named buffers, no register copies), and
    // the hat_Z / Z stores are buffer stores whose lanes past the chunk carry an
    // out-of-range offset (dropped by the hardware) instead of a branch: the compiler
    // then waits for a buffer's loads without also waiting for the stores issued after
    // them (a join after branched stores drains every store of the step)
    constexpr int BP = 64 / KP;
    const int stride = NW * BP;
    const double lo = p.logOmega[gl];
    const int nb = b1 - b0;
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
        p.hatZ + (size_t)b0 * KP, (short)0, nb * KP * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(
        p.Z + (size_t)(b0 - p.i_buf0) * KP, (short)0, nb * KP * 8, 0x00020000);
    auto step = [&](int ib, double tnb, double llb) {
#pragma clang fp contract(off)
      const bool iv = ib < b1;
      const double lz = tnb * (lo + llb);  // rounded before the shift (see below)
      double mx = lz;
#pragma unroll
      for (int off = KP >> 1; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
      double sm = exp(lz - mx);
#pragma unroll
      for (int off = KP >> 1; off >= 1; off >>= 1) sm += __shfl_xor(sm, off, 64);
      const double lse = mx + log(sm);
      const double hz = exp(lz - lse) + 1e-50;
      const double Z = hz * tnb;
      const int off = iv ? ((ib - b0) * KP + gl) * 8 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(resp_u2, hz), rh, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(resp_u2, Z), rz, off, 0, 0);
      // (no branch in the step: the lanes past the chunk add zeros)
      accNj[(wave * BP + sub) * KP + gl] += iv ? Z : 0.0;
      atomicAdd(&gcnt[gl], (iv && Z > kGateZ) ? 1 : 0);
      l1 += iv ? Z * llb : 0.0;
      l7 += iv ? hz * log(hz) : 0.0;
    };
    auto ld = [&](int ib, double &tnb, double &llb) {
      const int ii = ib < b1 ? ib : b0;
      tnb = p.tildeN[ii];
      llb = p.LL[(size_t)ii * KP + gl];
    };
    int i = b0 + wave * BP + sub;
    double tA, lA, tB, lB;
    ld(i, tA, lA);
    for (; i - sub < b1; i += 2 * stride) {
      ld(i + stride, tB, lB);
      step(i, tA, lA);
      ld(i + 2 * stride, tA, lA);
      step(i + stride, tB, lB);  // (past the chunk: every lane adds zeros, stores dropped)
    }
  } else if (K <= G) {
    // one cluster per lane: the next base's tilde_N and L_elbo are loaded while
    // this base's ẑ is computed (a C4 wave walks 6 bases of its chunk in turn)
    const int stride = NW * BPW;
    const double lo = gl < K ? p.logOmega[gl] : 0.0;
    int i = b0 + wave * BPW + sub;
    int ii = i < b1 ? i : b0;
    double tn = p.tildeN[ii];
    double ll = gl < K ? p.LL[(size_t)ii * K + gl] : 0.0;
    // one base step: hat_Z, Z and the sums of base ib (valid when ib < b1)
    auto step = [&](int ib, double tnb, double llb) {
#pragma clang fp contract(off)
      const bool iv = ib < b1;
      const double lz = tnb * (lo + llb);  // rounded before the shift (see below)
      double mx = gl < K ? lz : -INFINITY;
      mx = group_max(mx, G);
      double sm = gl < K ? exp(lz - mx) : 0.0;
      sm = group_sum(sm, G);
      const double lse = mx + log(sm);
      if (iv && gl < K) {
        const double hz = exp(lz - lse) + 1e-50;
        const double Z = hz * tnb;
        p.hatZ[(size_t)ib * K + gl] = hz;
        p.Z[(size_t)(ib - p.i_buf0) * K + gl] = Z;
        accNj[(wave * BPW + sub) * K + gl] += Z;
        if (Z > kGateZ) atomicAdd(&gcnt[gl], 1);
        l1 += Z * llb;
        l7 += hz * log(hz);
      }
    };
#if VBHEM_RESP_UNROLL == 2
    // two base steps per iteration: their chains (group max, exp, group sum, log)
    // interleave; the sums still take base i before base i + stride
    for (; i - sub < b1; i += 2 * stride) {
      const int i2 = i + stride, i2c = i2 < b1 ? i2 : b0;
      const int in = i + 2 * stride < b1 ? i + 2 * stride : b0;
      const double tn2 = p.tildeN[i2c];
      const double ll2 = gl < K ? p.LL[(size_t)i2c * K + gl] : 0.0;
      const double tn_n = p.tildeN[in];
      const double ll_n = gl < K ? p.LL[(size_t)in * K + gl] : 0.0;
      step(i, tn, ll);
      step(i2, tn2, ll2);
      tn = tn_n;
      ll = ll_n;
    }
#else
    for (; i - sub < b1; i += stride) {
      const int in = i + stride < b1 ? i + stride : b0;
      const double tn_n = p.tildeN[in];
      const double ll_n = gl < K ? p.LL[(size_t)in * K + gl] : 0.0;
      step(i, tn, ll);
      tn = tn_n;
      ll = ll_n;
    }
#endif
  } else
  for (int i = b0 + wave * BPW + sub; i - sub < b1; i += NW * BPW) {
    // log_Z = tilde_N .* (logOmega + L_elbo) is rounded before the shift, as in
    // step_fc.m:275-276 (an fma-contracted shift would let the winning entry
    // exceed 1 by ~ulp(log_Z)).
#pragma clang fp contract(off)
    const bool iv = i < b1;
    const int ii = iv ? i : b0;
    const double tn = p.tildeN[ii];
    const double *LL = p.LL + (size_t)ii * K;
    double mx = -INFINITY;
    for (int j = gl; j < K; j += G) mx = fmax(mx, tn * (p.logOmega[j] + LL[j]));
    mx = group_max(mx, G);
    double sm = 0.0;
    for (int j = gl; j < K; j += G) sm += exp(tn * (p.logOmega[j] + LL[j]) - mx);
    sm = group_sum(sm, G);
    const double lse = mx + log(sm);
    if (iv) {
      for (int j = gl; j < K; j += G) {
        const double ll = LL[j];
        const double hz = exp(tn * (p.logOmega[j] + ll) - lse) + 1e-50;
        const double Z = hz * tn;
        p.hatZ[(size_t)i * K + j] = hz;
        p.Z[(size_t)(i - p.i_buf0) * K + j] = Z;
        accNj[(wave * BPW + sub) * K + j] += Z;
        if (Z > kGateZ) atomicAdd(&gcnt[j], 1);
        l1 += Z * ll;
        l7 += hz * log(hz);
      }
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
    for (int w = 0; w < NW * BPW; ++w) s += accNj[w * K + j];
    slab[j] = p.assign ? s : slab[j] + s;
  }
  if (tid < 2) {
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += accLt[2 * w + tid];
    double &dst = slab[(size_t)K + (size_t)K * p.S + (size_t)K * p.S * p.S + tid];
    dst = p.assign ? s : dst + s;
  }
  if (p.gate_cnt)
    for (int j = tid; j < K; j += kRespThreads) p.gate_cnt[(size_t)blockIdx.x * K + j] = gcnt[j];
}

// ---------------------------------------------------------------------------
// resp_trials_kernel: resp_kernel for R = K / KT independent EM trials batched
// as one cluster set (trial r = clusters [r KT, (r+1) KT)).  hat_Z(i, .) is
// normalised within each trial (step_fc.m:275-281 per trial); Nj, Lt1, Lt7 go
// to trial r's section [r SL, (r+1) SL) of the slab.  K <= 256: a lane holds
// the clusters gl + s G, s < kRespSlots; per-trial sums are masked lane sums in
// a fixed order (deterministic).
// ---------------------------------------------------------------------------
constexpr int kRespSlots = 4;

__global__ __launch_bounds__(kRespThreads) void resp_trials_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kRespThreads / 64;
  const int K = p.K, KT = p.KT, R = K / KT, SL = p.SL, S = p.S;
  int G = 1;
  while (G < K && G < 64) G <<= 1;
  const int BPW = 64 / G;
  const int sub = lane / G, gl = lane - sub * G;
  double *accNj = lds;                        // [NW*BPW][K]
  double *accLt = accNj + NW * BPW * K;       // [NW][R][2]
  int *gcnt = reinterpret_cast<int *>(accLt + 2 * NW * R);  // [K]
  for (int x = tid; x < NW * BPW * K + 2 * NW * R; x += kRespThreads) accNj[x] = 0.0;
  for (int x = tid; x < K; x += kRespThreads) gcnt[x] = 0;
  __syncthreads();
  int tr[kRespSlots];  // trial of this lane's slot s (-1: no cluster)
#pragma unroll
  for (int s = 0; s < kRespSlots; ++s) {
    const int j = gl + s * G;
    tr[s] = j < K ? j / KT : -1;
  }
  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  double l1[kRespSlots], l7[kRespSlots];
#pragma unroll
  for (int s = 0; s < kRespSlots; ++s) l1[s] = l7[s] = 0.0;
  for (int i = b0 + wave * BPW + sub; i - sub < b1; i += NW * BPW) {
#pragma clang fp contract(off)
    const bool iv = i < b1;
    const int ii = iv ? i : b0;
    const double tn = p.tildeN[ii];
    const double *LL = p.LL + (size_t)ii * K;
    double lz[kRespSlots], lse[kRespSlots];
#pragma unroll
    for (int s = 0; s < kRespSlots; ++s) {
      const int j = tr[s] >= 0 ? gl + s * G : 0;
      lz[s] = tr[s] >= 0 ? tn * (p.logOmega[j] + LL[j]) : -INFINITY;
      lse[s] = 0.0;
    }
    for (int r = 0; r < R; ++r) {
      double mx = -INFINITY;
#pragma unroll
      for (int s = 0; s < kRespSlots; ++s) mx = tr[s] == r ? fmax(mx, lz[s]) : mx;
      mx = group_max(mx, G);
      double sm = 0.0;
#pragma unroll
      for (int s = 0; s < kRespSlots; ++s) sm += tr[s] == r ? exp(lz[s] - mx) : 0.0;
      sm = group_sum(sm, G);
      const double l = mx + log(sm);
#pragma unroll
      for (int s = 0; s < kRespSlots; ++s) lse[s] = tr[s] == r ? l : lse[s];
    }
    if (iv) {
#pragma unroll
      for (int s = 0; s < kRespSlots; ++s) {
        if (tr[s] < 0) continue;
        const int j = gl + s * G;
        const double hz = exp(lz[s] - lse[s]) + 1e-50;
        const double Z = hz * tn;
        p.hatZ[(size_t)i * K + j] = hz;
        p.Z[(size_t)(i - p.i_buf0) * K + j] = Z;
        accNj[(wave * BPW + sub) * K + j] += Z;
        if (Z > kGateZ) atomicAdd(&gcnt[j], 1);
        l1[s] += Z * LL[j];
        l7[s] += hz * log(hz);
      }
    }
  }
  for (int r = 0; r < R; ++r) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int s = 0; s < kRespSlots; ++s) {
      a += tr[s] == r ? l1[s] : 0.0;
      b += tr[s] == r ? l7[s] : 0.0;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      accLt[(wave * R + r) * 2] = a;
      accLt[(wave * R + r) * 2 + 1] = b;
    }
  }
  __syncthreads();
  double *slab = p.slabs + (size_t)blockIdx.x * p.slab_len;
  for (int j = tid; j < K; j += kRespThreads) {
    double s = 0.0;
    for (int w = 0; w < NW * BPW; ++w) s += accNj[w * K + j];
    const int r = j / KT;
    double &dst = slab[(size_t)r * SL + (j - r * KT)];
    dst = p.assign ? s : dst + s;
  }
  for (int x = tid; x < 2 * R; x += kRespThreads) {
    const int r = x >> 1, q = x & 1;
    double s = 0.0;
    for (int w = 0; w < NW; ++w) s += accLt[(w * R + r) * 2 + q];
    double &dst = slab[(size_t)r * SL + KT + (size_t)KT * S + (size_t)KT * S * S + q];
    dst = p.assign ? s : dst + s;
  }
  if (p.gate_cnt)
    for (int j = tid; j < K; j += kRespThreads) p.gate_cnt[(size_t)blockIdx.x * K + j] = gcnt[j];
}

// ---------------------------------------------------------------------------
// gate_list_kernel: the gated pairs as per-cluster lists of bases, ascending i
// (list[j][n], n < list_tot[j]).  Block = the resp_kernel chunk: its offset in
// cluster j's list is the gate count of the chunks before it; inside the chunk
// the bases are ranked by wave ballots (masks in LDS, one barrier per slice).
// Deterministic (no global atomics): the same list every call.
// ---------------------------------------------------------------------------
constexpr int kListThreads = 256;

__global__ __launch_bounds__(kListThreads) void gate_list_kernel(const StatsArgs p) {
  extern __shared__ int ish[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kListThreads / 64;
  const int K = p.K, nchunk = gridDim.x, me = blockIdx.x;
  int *before = ish;          // [K] this chunk's offset in every cluster's list
  int *total = ish + K;       // [K]
  int *wcnt = ish + 2 * K;    // [NW] (unused slot)
  // this chunk's offset (gate counts of chunks c < me) and cluster totals: thread
  // (r, j) sums chunks c = r, r + R, ...; then the R partials of each j in order
  int *pb = wcnt + NW;        // [R][K]
  int *pt = pb + kListThreads;  // [R][K]
  for (int j0 = 0; j0 < K; j0 += kListThreads) {
    const int KC = min(K - j0, kListThreads), R = kListThreads / KC;
    const int r = tid / KC, j = j0 + (tid - r * KC);
    if (r < R) {
      // 32 chunks' counts in flight per thread (clamped addresses, then masked sums): one
      // memory round trip for up to 32 R chunks instead of one per 8
      int sb = 0, stt = 0;
      for (int c0 = r; c0 < nchunk; c0 += 32 * R) {
        int v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          const int c = min(c0 + q * R, nchunk - 1);
          v[q] = p.gate_cnt[(size_t)c * K + j];
        }
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          const int c = c0 + q * R;
          stt += c < nchunk ? v[q] : 0;
          sb += c < me ? v[q] : 0;
        }
      }
      pb[tid] = sb;
      pt[tid] = stt;
    }
    __syncthreads();
    if (tid < KC) {
      int sb = 0, stt = 0;
      for (int q = 0; q < R; ++q) {
        sb += pb[q * KC + tid];
        stt += pt[q * KC + tid];
      }
      before[j0 + tid] = sb;
      total[j0 + tid] = stt;
    }
    __syncthreads();
  }
  if (me == 0)
    for (int j = tid; j < K; j += kListThreads) p.list_tot[j] = total[j];
  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, me, nchunk, b0, b1);
  // per 256-base slice: every wave ballots all K clusters into LDS masks (no
  // barrier per cluster), one barrier, then each thread places its base in the
  // lists that gate it in, after the bases of the lower waves and chunks
  unsigned long long *msk = reinterpret_cast<unsigned long long *>(
      ish + ((2 * K + NW + 2 * kListThreads + 1) & ~1));  // [NW][K], 8-byte aligned
  constexpr int kJB = 16;  // clusters whose Z are loaded together (one round trip, not K)
  for (int i0 = b0; i0 < b1; i0 += kListThreads) {
    const int i = i0 + tid;
    const bool iv = i < b1;
    const double *Zi = p.Z + (size_t)((iv ? i : b0) - p.i_buf0) * K;
    for (int j0 = 0; j0 < K; j0 += kJB) {
      double z[kJB];
#pragma unroll
      for (int q = 0; q < kJB; ++q) z[q] = j0 + q < K ? Zi[j0 + q] : 0.0;
#pragma unroll
      for (int q = 0; q < kJB; ++q) {
        const unsigned long long m = __ballot(iv && z[q] > kGateZ);
        if (lane == 0 && j0 + q < K) msk[wave * K + j0 + q] = m;
      }
    }
    __syncthreads();
    for (int j = 0; j < K; ++j) {
      const unsigned long long m = msk[wave * K + j];
      if ((m >> lane) & 1ull) {
        int off = before[j];
        for (int w = 0; w < wave; ++w) off += __popcll(msk[w * K + j]);
        p.list[(size_t)j * p.list_cap + off + __popcll(m & ((1ull << lane) - 1ull))] = i;
      }
    }
    __syncthreads();  // every thread has read before[] and the masks
    for (int j = tid; j < K; j += kListThreads) {
      int t = 0;
      for (int w = 0; w < NW; ++w) t += __popcll(msk[w * K + j]);
      before[j] += t;
    }
    __syncthreads();  // before[] updated before the next slice's masks overwrite these
  }
}

// ---------------------------------------------------------------------------
// stats_list_kernel<PER>: the gated sums over the gated-pair lists only.
// Block (c, j) = part c of cluster j's list (fixed split, ascending bases) ->
// slab c's cluster-j entries; PB pairs per batch staged in LDS as
//   [ Z sum_t_nu (S x SB) | Z sum_nu_1 (S) | Z sum_xi (S x S) | u (SB x NU) ],
// each thread owning PER outputs of  N1 (S) | M (S x S) | U (S x NU).
// ---------------------------------------------------------------------------
constexpr int kSlThreads = 256;

template <int PER>
__global__ __launch_bounds__(kSlThreads) void stats_list_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  const int K = p.K, S = p.S, SB = p.SB, d = p.d, NU = p.NU, PB = p.PB;
  const int j = blockIdx.y, c = blockIdx.x, nch = gridDim.x;
  const bool full = p.covmode == kCovFull;
  const int dd = full ? d * d : d;
  const int OT = S * SB, OM = OT + S, OU = OM + S * S;  // record: tnu | nu1 | xi | u
  const int RS = (OU + SB * NU + 1) / 2 * 2;  // record stride (doubles), = sl_record()
  const int NO = S + S * S + S * NU;
  double *rec = lds;                                            // [PB][RS]
  int *tab = reinterpret_cast<int *>(rec + (size_t)PB * RS);    // [NU] packed (a, b)
  double *sz = reinterpret_cast<double *>(tab + (NU + 1) / 2 * 2);  // [PB] Z of the batch
  int *sidx = reinterpret_cast<int *>(sz + PB);                   // [PB] bases of the batch
  for (int cc = tid; cc < NU; cc += kSlThreads) {
    int a = -1, b = -1;
    if (cc >= 1 && cc <= d) {
      a = cc - 1;
    } else if (cc > d) {
      if (full) {
        int k = cc - 1 - d;
        a = 0;
        while (k >= d - a) { k -= d - a; ++a; }
        b = a + k;
      } else {
        a = b = cc - 1 - d;
      }
    }
    tab[cc] = (a + 1) | ((b + 1) << 16);
  }
  const int tot = p.list_tot[j];
  const int n0 = (int)((long long)tot * c / nch), n1 = (int)((long long)tot * (c + 1) / nch);
  const int *lst = p.list + (size_t)j * p.list_cap;
  const float invNU = 1.0f / (float)NU, invOU = 1.0f / (float)OU, invUN = 1.0f / (float)(SB * NU);
  double *slab = p.slabs + (size_t)c * p.slab_len;
  // trial section of cluster j (R = K / KT trials; one section when KT = K)
  const int KT = p.KT, tr = j / KT, jt = j - tr * KT;
  double *tsl = slab + (size_t)tr * p.SL;
  for (int o0 = 0; o0 < NO; o0 += PER * kSlThreads) {
    double acc[PER];
#pragma unroll
    for (int e = 0; e < PER; ++e) acc[e] = 0.0;
    for (int n = n0; n < n1; n += PB) {
      const int np = min(PB, n1 - n);
      __syncthreads();  // tab ready / previous batch consumed
      // batch-wide staging: every element of every pair in flight at once
      if (tid < np) {
        const int i = lst[n + tid];
        const size_t lp = (size_t)(i - p.i_buf0) * K + j;
        sidx[tid] = i;
        sz[tid] = p.Z[lp];
      }
      __syncthreads();
      for (int x = tid; x < np * OU; x += kSlThreads) {
        const int pq = qdiv(x, invOU), e = x - pq * OU;
        const size_t lp = (size_t)(sidx[pq] - p.i_buf0) * K + j;
        double v;
        if (e < OT) v = p.tnu[lp * OT + e];
        else if (e < OM) v = p.nu1[lp * S + (e - OT)];
        else v = p.xi[lp * S * S + (e - OM)];
        rec[(size_t)pq * RS + e] = sz[pq] * v;
      }
      for (int x = tid; x < np * SB * NU; x += kSlThreads) {
        const int pq = qdiv(x, invUN), e = x - pq * SB * NU;
        const int bb = qdiv(e, invNU), cc = e - bb * NU;
        const int i = sidx[pq];
        const int t = tab[cc], a = (t & 0xffff) - 1, b2 = (t >> 16) - 1;
        const double *mu = p.centres + ((size_t)i * SB + bb) * d;
        const double *C = p.covars + ((size_t)i * SB + bb) * dd;
        double u;
        if (a < 0) u = 1.0;
        else if (b2 < 0) u = mu[a];
        else u = (full ? C[a * d + b2] : C[a]) + mu[a] * mu[b2];
        rec[(size_t)pq * RS + OU + e] = u;
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int o = o0 + tid + e * kSlThreads;
        if (o < S) {
          for (int pq = 0; pq < np; ++pq) acc[e] += rec[(size_t)pq * RS + OT + o];
        } else if (o < S + S * S) {
          for (int pq = 0; pq < np; ++pq) acc[e] += rec[(size_t)pq * RS + OM + (o - S)];
        } else if (o < NO) {
          const int oo = o - S - S * S;
          const int sg = qdiv(oo, invNU), cc = oo - sg * NU;
          for (int pq = 0; pq < np; ++pq) {
            const double *r = rec + (size_t)pq * RS;
            for (int bb = 0; bb < SB; ++bb) acc[e] = fma(r[sg * SB + bb], r[OU + bb * NU + cc], acc[e]);
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      const int o = o0 + tid + e * kSlThreads;
      double *dst = nullptr;
      if (o < S) {
        dst = tsl + KT + (size_t)jt * S + o;
      } else if (o < S + S * S) {
        dst = tsl + KT + (size_t)KT * S + (size_t)jt * S * S + (o - S);
      } else if (o < NO) {
        const int oo = o - S - S * S;
        dst = tsl + KT + (size_t)KT * S + (size_t)KT * S * S + 2 + (size_t)jt * S * NU + oo;
      }
      if (dst) *dst = p.assign ? acc[e] : *dst + acc[e];
    }
  }
}

// ---------------------------------------------------------------------------
// stats_kernel<TPW>: the emission-moment GEMM U (TPW = max MFMA tiles per
// wave).  Software-pipelined over batches of NBB (<= 4) bases: while batch b
// is contracted on the MFMA, the loads of batch b+1 (sum_t_nu, Z, covariances,
// means) are in flight into registers.  N1 / M are summed by nm_kernel.
// ---------------------------------------------------------------------------
constexpr int kStatsThreads = 512;
constexpr int kStatsWaves = kStatsThreads / 64;
constexpr int kStatsMaxNBB = 4;
constexpr int kStatsMaxA = 8;   // sum_t_nu values per thread per batch
constexpr int kStatsMaxR = 8;   // raw covariance / mean values per thread per batch

template <int TPW>
__global__ __launch_bounds__(kStatsThreads) void stats_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = p.K, S = p.S, SB = p.SB, SBp = p.SBp, d = p.d, NU = p.NU, NBB = p.NBB;
  const int AST = p.AST, UST = p.UST;
  const int j0 = blockIdx.y * p.JG, j1 = min(K, j0 + p.JG), JGc = j1 - j0;
  const int RG = JGc * S, SS = S * S;
  const int MT = (RG + 15) / 16, NTL = (NU + 15) / 16, ntiles = MT * NTL;
  const bool full = p.covmode == kCovFull;
  const int dd = full ? d * d : d;
  const int NA = NBB * RG * SB;          // A elements per batch
  const int NRC = NBB * SB * dd;         // raw covariance values per batch
  const int NR = NRC + NBB * SB * d;     // + means

  double *As = lds;                                   // [RG][AST]   g Z sum_t_nu
  double *Us = As + (size_t)RG * AST;                 // [NBB*SBp][UST] base moments
  double *raw = Us + (size_t)NBB * SBp * UST;         // [NBB*SB][dd] | [NBB*SB][d]
  double *gzs = raw + (size_t)NR;                     // [NBB][JGc]
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
  const float invJG = 1.0f / (float)JGc;
  const float invRSB = 1.0f / (float)(RG * SB);

  double4_t acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = (double4_t){0.0, 0.0, 0.0, 0.0};

  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  const double *__restrict__ tnu = p.tnu;

  // ---- register prefetch buffers ----
  double pa[kStatsMaxA], pr[kStatsMaxR], pz = 0.0;
  auto prefetch = [&](int ib) {
    const int nq = min(NBB, b1 - ib);
#pragma unroll
    for (int e = 0; e < kStatsMaxA; ++e) {
      const int x = tid + e * kStatsThreads;
      const int q = qdiv(x, invRSB), rem = x - q * RG * SB;
      pa[e] = (x < NA && q < nq) ? tnu[((size_t)(ib + q - p.i_buf0) * K * S + (size_t)j0 * S) * SB + rem]
                                 : 0.0;
    }
    const size_t gs = (size_t)ib * SB;
#pragma unroll
    for (int e = 0; e < kStatsMaxR; ++e) {
      const int x = tid + e * kStatsThreads;
      double v = 0.0;
      if (x < NRC) {
        if (x < nq * SB * dd) v = p.covars[gs * dd + x];
      } else if (x < NR) {
        const int y = x - NRC;
        if (y < nq * SB * d) v = p.centres[gs * d + y];
      }
      pr[e] = v;
    }
    if (tid < NBB * JGc) {
      const int q = qdiv(tid, invJG), jj = tid - q * JGc;
      pz = q < nq ? p.Z[(size_t)(ib + q - p.i_buf0) * K + j0 + jj] : 0.0;
    }
  };
  __syncthreads();
  if (b0 < b1) prefetch(b0);

  for (int ib = b0; ib < b1; ib += NBB) {
    const int nq = min(NBB, b1 - ib);
    // -- commit: gated Z and the raw base data of this batch -> LDS ------------------
    if (tid < NBB * JGc) gzs[tid] = (pz > kGateZ) ? pz : 0.0;
#pragma unroll
    for (int e = 0; e < kStatsMaxR; ++e) {
      const int x = tid + e * kStatsThreads;
      if (x < NR) raw[x] = pr[e];
    }
    __syncthreads();
    // -- A = g Z sum_t_nu and the base moments U -------------------------------------
#pragma unroll
    for (int e = 0; e < kStatsMaxA; ++e) {
      const int x = tid + e * kStatsThreads;
      if (x < NA) {
        const int q = qdiv(x, invRSB), rem = x - q * RG * SB;
        const int r = qdiv(rem, invSB), be = rem - r * SB;
        As[r * AST + q * SBp + be] = (q < nq) ? gzs[q * JGc + qdiv(r, invS)] * pa[e] : 0.0;
      }
    }
    for (int x = tid; x < NBB * SB * NU; x += kStatsThreads) {
      const int row = qdiv(x, invNU), c = x - row * NU;
      const int q = qdiv(row, invSB), be = row - q * SB;
      double u = 0.0;
      if (q < nq) {
        const int t = tab[c], a = (t & 0xffff) - 1, b = (t >> 16) - 1;
        const double *mu = raw + NRC + (size_t)row * d;
        if (a < 0) {
          u = 1.0;
        } else if (b < 0) {
          u = mu[a];
        } else {
          const double *C = raw + (size_t)row * dd;
          u = (full ? C[a * d + b] : C[a]) + mu[a] * mu[b];
        }
      }
      Us[(q * SBp + be) * UST + c] = u;
    }
    __syncthreads();
    // -- next batch's loads fly while this batch is contracted --------------------------
    if (ib + NBB < b1) prefetch(ib + NBB);
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
}

// ---------------------------------------------------------------------------
// nm_kernel: N1[j][s] += g Z(i,j) sum_nu_1(i,j,s) and M[j][s][r] += g Z(i,j)
// sum_xi(i,j,s,r) over this chunk's bases -- plain streaming weighted sums
// (each thread owns fixed outputs; 4 bases in flight per step).
// ---------------------------------------------------------------------------
constexpr int kNmThreads = 256;

// PER outputs per thread (K*S + K*S*S <= PER * 256), UNR bases per step in flight.
template <int PER, int UNR>
__global__ __launch_bounds__(kNmThreads) void nm_kernel(const StatsArgs p) {
  const int tid = threadIdx.x;
  const int K = p.K, S = p.S, KS = K * S, KSS = KS * S, NO = KS + KSS;
  int b0, b1;
  chunk_range(p.i_end - p.i_begin, p.i_begin, blockIdx.x, gridDim.x, b0, b1);
  double acc[PER];
  int jo[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    acc[e] = 0.0;
    const int x = tid + e * kNmThreads;
    jo[e] = x < KS ? x / S : (x < NO ? (x - KS) / (S * S) : 0);
  }
  for (int i = b0; i < b1; i += UNR) {
    double v[UNR][PER], z[UNR][PER];
    // branch-free: clamped addresses and unconditional loads (a conditional load
    // becomes a branch with its own vmcnt(0) wait and serialises the stream)
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool iv = i + u < b1;
      const size_t ir = (size_t)((iv ? i + u : i) - p.i_buf0);
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int x = tid + e * kNmThreads;
        const int xc = x < NO ? x : 0;
        const double *src = xc < KS ? p.nu1 + ir * KS + xc : p.xi + ir * KSS + (xc - KS);
        v[u][e] = *src;
        z[u][e] = p.Z[ir * K + jo[e]];
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const bool iv = i + u < b1;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int x = tid + e * kNmThreads;
        const double zz = z[u][e];
        z[u][e] = (iv && x < NO && zz > kGateZ) ? zz : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int e = 0; e < PER; ++e) acc[e] = fma(z[u][e], v[u][e], acc[e]);
  }
  double *slab = p.slabs + (size_t)blockIdx.x * p.slab_len + K;  // [N1 | M]
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int x = tid + e * kNmThreads;
    if (x < NO) slab[x] += acc[e];
  }
}

// 256 threads = 16 columns x 16 slab partitions: partition p sums slabs
// p, p+16, p+32, ... (128-B rows, four loads in flight per thread), then the 16
// partials are added in fixed order -- deterministic; ~slab_len/16 blocks (C4:
// 506) keep every CU's loads in flight (32-column blocks left it latency-bound).
constexpr int kFinalCols = 16, kFinalParts = 16;
__global__ __launch_bounds__(256) void stats_final_kernel(const double *slabs, int nslab_all,
                                                          int nslab_stats, int slab_len, int KT,
                                                          int S, int SL, double *out, int *fpre,
                                                          unsigned long long tag,
                                                          unsigned long long *done,
                                                          unsigned long long done_val) {
  __shared__ double part[kFinalParts][kFinalCols];
  // the call's last kernel closes the flag head (kFlagPre): the total kept, the counters
  // zeroed, the tag written -- the next call's in-kernel preparation finds them clean.
  // With a completion word, counter [2] (fb_exact_kernel's blocks-done, zero between
  // passes) counts this kernel's finished blocks instead: the last one resets it
  if (fpre && blockIdx.x == 0 && threadIdx.x == 0) {
    int *fc = fpre + kFlagPre;
    fpre[2] = fc[1];
    for (int c = 0; c < kFlagHead; ++c)
      if (!(done && c == 2)) fc[c] = 0;
    *reinterpret_cast<unsigned long long *>(fpre) = tag;
  }
  const int c = threadIdx.x % kFinalCols, pp = threadIdx.x / kFinalCols;
  const int x = blockIdx.x * kFinalCols + c;
  // resp_kernel's columns (Nj, Lt1, Lt7) have a partial in every chunk's slab; the
  // gated statistics' only in their kernel's parts
  const int xs = x % SL, lt = KT * (1 + S + S * S);
  const int nslab = (xs < KT || (xs >= lt && xs < lt + 2)) ? nslab_all : nslab_stats;
  double acc = 0.0;
  if (x < slab_len) {
    int k = pp;
    for (; k + 3 * kFinalParts < nslab; k += 4 * kFinalParts) {
      const double *q = slabs + (size_t)k * slab_len + x;
      const double v0 = q[0], v1 = q[(size_t)kFinalParts * slab_len],
                   v2 = q[(size_t)2 * kFinalParts * slab_len], v3 = q[(size_t)3 * kFinalParts * slab_len];
      acc += v0;
      acc += v1;
      acc += v2;
      acc += v3;
    }
    for (; k < nslab; k += kFinalParts) acc += slabs[(size_t)k * slab_len + x];
  }
  part[pp][c] = acc;
  __syncthreads();
  if (pp == 0 && x < slab_len) {
    double s = part[0][c];
#pragma unroll
    for (int q = 1; q < kFinalParts; ++q) s += part[q][c];
    // a lost flag-head handshake (kFlagLost, fb_bwd2_kernel): results untrusted
    if (fpre && __hip_atomic_load(fpre + kFlagLost, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    kFlagLostMark)
      s = __builtin_nan("");
    if (done)  // written through to the system (the host polls the word, not an event)
      __hip_atomic_store(reinterpret_cast<unsigned long long *>(out + x), __double_as_longlong(s),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      out[x] = s;
  }
  if (done && fpre) {
    // every store of this block acknowledged (written through at system scope: what a
    // system-scope release would wait for, without its L2 write-back), then one count
    // per block; the last block to count publishes the word after all of them
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    if (threadIdx.x == 0) {
      int *cnt = fpre + kFlagPre + 2;
      const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (int)gridDim.x - 1) {
        __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(done, done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// planning + launch
// ---------------------------------------------------------------------------
namespace {
constexpr size_t kStatsLdsTarget = 78 * 1024;  // two 512-thread blocks per CU
constexpr int kMaxTPW = 16;

size_t stats_lds_bytes(int RG, int AST, int NBB, int SBp, int UST, int JG, int NU, int SB, int d,
                       int dd) {
  return ((size_t)RG * AST + (size_t)NBB * SBp * UST + (size_t)NBB * SB * (dd + d) +
          (size_t)NBB * JG) * sizeof(double) +
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
  if (K * S + K * S * S > 24 * kNmThreads) return false;
  if (RG > kStatsThreads) return false;
  const int dd = a.covmode == kCovFull ? a.d * a.d : a.d;
  int nbb = kStatsMaxNBB;
  for (; nbb >= 1; --nbb) {
    const bool regs_ok = (nbb * RG * a.SB + kStatsThreads - 1) / kStatsThreads <= kStatsMaxA &&
                         (nbb * a.SB * (dd + a.d) + kStatsThreads - 1) / kStatsThreads <= kStatsMaxR;
    a.NBB = nbb;
    a.AST = nbb * a.SBp + 1;
    lds = stats_lds_bytes(RG, a.AST, nbb, a.SBp, a.UST, jg, a.NU, a.SB, a.d, dd);
    if (regs_ok && lds <= kStatsLdsTarget) break;
  }
  if (nbb < 1) return false;
  return true;
}

template <int TPW>
static hipError_t launch_stats_t(const StatsArgs &a, int nchunk, int ngroups, size_t lds,
                                 hipStream_t st) {
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&stats_kernel<TPW>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((stats_kernel<TPW>), dim3(nchunk, ngroups), dim3(kStatsThreads), lds, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int no = a.K * a.S + a.K * a.S * a.S;
  if (no <= 6 * kNmThreads)
    hipLaunchKernelGGL((nm_kernel<6, 4>), dim3(nchunk), dim3(kNmThreads), 0, st, a);
  else
    hipLaunchKernelGGL((nm_kernel<24, 1>), dim3(nchunk), dim3(kNmThreads), 0, st, a);
  return hipGetLastError();
}

size_t resp_lds(int K, int KT) {
  int G = 1;
  while (G < K && G < 64) G <<= 1;
  const size_t R = KT >= 1 && K % KT == 0 ? (size_t)(K / KT) : 1;
  // (at least the folded fallback's queue, which borrows this space first)
  return std::max(((size_t)(kRespThreads / 64) * ((64 / G) * (size_t)K + 2 * R)) * sizeof(double) +
                      (size_t)K * sizeof(int),
                  (size_t)(kRespThreads + 1) * sizeof(int));
}

template <int KP>
static hipError_t launch_resp_k(const StatsArgs &a, int nchunk, size_t lds, hipStream_t st) {
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&resp_kernel<KP>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(resp_kernel<KP>, dim3(nchunk), dim3(kRespThreads), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_resp(const StatsArgs &a, int nchunk, hipStream_t st) {
  // per-wave Nj accumulators of all K clusters in LDS (past 64 KB at K ~ 960: the
  // launch sets the dynamic-LDS attribute; the caller rejects K past a CU's LDS)
  size_t lds = resp_lds(a.K, a.KT);
  // the folded fallback borrows the accumulators' space first (queue + worker regions)
  if (a.fold) lds = std::max(lds, fold_lds_bytes(kRespThreads, kRespFoldWaves, a.fx.S, a.fx.SB));
  if (a.KT != a.K) {  // batched trials
    if (a.K > kRespSlots * 64 || a.KT < 1 || a.K % a.KT != 0) return hipErrorInvalidValue;
    hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&resp_trials_kernel), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(resp_trials_kernel, dim3(nchunk), dim3(kRespThreads), lds, st, a);
    return hipGetLastError();
  }
  switch (std::getenv("VBHEM_RESP_GENERIC") ? 0 : a.K) {  // (A/B: the generic kernel)
    case 4: return launch_resp_k<4>(a, nchunk, lds, st);
    case 8: return launch_resp_k<8>(a, nchunk, lds, st);
    case 16: return launch_resp_k<16>(a, nchunk, lds, st);
    case 32: return launch_resp_k<32>(a, nchunk, lds, st);
    case 64: return launch_resp_k<64>(a, nchunk, lds, st);
    default: return launch_resp_k<0>(a, nchunk, lds, st);
  }
}

hipError_t launch_stats(const StatsArgs &a, int nchunk, int ngroups, size_t lds, hipStream_t st) {
  const int RG = a.JG * a.S;
  const int ntiles = ((RG + 15) / 16) * ((a.NU + 15) / 16);
  const int tpw = (ntiles + kStatsWaves - 1) / kStatsWaves;
  if (tpw <= 4) return launch_stats_t<4>(a, nchunk, ngroups, lds, st);
  if (tpw <= 8) return launch_stats_t<8>(a, nchunk, ngroups, lds, st);
  return launch_stats_t<16>(a, nchunk, ngroups, lds, st);
}

// ---------------------------------------------------------------------------
// stats_list_u_kernel<FPL, SM>: stats_list_kernel on the emission GEMM's prepared
// operand U (vbhem_emission.hip: per base-state column the features
// [Sigma_ab + Sigma_ba + 2 mu'_a mu'_b (a < b) | Sigma_aa + mu'_a^2, mu'], mu' = mu - z),
// so the emission moments need no gather of the d x d covariances and no
// per-element rebuild.  Block (c, j) = part c of cluster j's list, as
// stats_list_kernel; wave w takes the part's pairs w, w + 4, ...:
//   lane f (+ 64 q) owns moment column f = 0 (ones) | 1 + a (mu_a) | 1 + d + k (packed
//   (a, b) of Sigma + mu mu') for every state s: acc[q][s] += sum_b Z tnu(s, b) u(b, f),
//   with Z tnu and the pair's U columns staged per pair in a wave-private LDS slab (U
//   read coalesced: lanes over (k-step, k, base state), SB contiguous columns per row);
//   sum_xi / sum_nu_1 accumulate lane-parallel from global memory.
// Waves reduce in fixed order (bit-reproducible), then every output is shifted back:
//   mu_a = m'_a + z_a N,  (Sigma + mu mu')_ab = Q'_ab + z_a m'_b + z_b m'_a + z_a z_b N
// (Q' = half the off-diagonal feature), N = sum Z tnu, m' = sum Z tnu mu'.
// ---------------------------------------------------------------------------
constexpr int kSuWaves = 4;

// the prepared-operand statistics' output phase: the block's reduced sums in red
// ([S][NU] | [S] | [S][S]) shifted back by z and written (or added) to slab c
__device__ __forceinline__ void su_output(const StatsArgs &p, const double *red, const double *zs,
                                          int c, int nch, int j, int tid) {
  const int S = p.S, NU = p.NU, d = p.d;
  const bool full = p.covmode == kCovFull;
  const int KT = p.KT, tr = j / KT, jt = j - tr * KT;
  double *tsl = p.slabs + (size_t)c * p.slab_len + (size_t)tr * p.SL;
  const int NO = S * NU + S + S * S;
  for (int o = tid; o < NO; o += 64 * kSuWaves) {
    double v;
    double *dst;
    if (o < S * NU) {
      const int s2 = o / NU, f = o - s2 * NU;
      const double *rs = red + (size_t)s2 * NU;
      const double N = rs[0];
      if (f == 0) {
        v = N;
      } else if (f <= d) {
        v = fma(zs[f - 1], N, rs[f]);
      } else {
        int a = f - 1 - d, b = a;
        if (full) {
          int k = a;
          a = 0;
          while (k >= d - a) { k -= d - a; ++a; }
          b = a + k;
        }
        const double q2 = (full && a != b) ? 0.5 * rs[f] : rs[f];
        v = q2 + (zs[a] * rs[1 + b] + zs[b] * rs[1 + a]) + zs[a] * zs[b] * N;
      }
      dst = tsl + KT + (size_t)KT * S + (size_t)KT * S * S + 2 + (size_t)jt * S * NU + o;
    } else if (o < S * NU + S) {
      v = red[o];
      dst = tsl + KT + (size_t)jt * S + (o - S * NU);
    } else {
      v = red[o];
      dst = tsl + KT + (size_t)KT * S + (size_t)jt * S * S + (o - S * NU - S);
    }
    *dst = p.assign ? v : *dst + v;
    if (p.assign)  // the slabs past this grid's chunks hold nothing of cluster j
      for (int cz = c + nch; cz < p.nzero; cz += nch) dst[(size_t)(cz - c) * p.slab_len] = 0.0;
  }
}


template <int FPL, int SM>
__global__ __launch_bounds__(64 * kSuWaves) void stats_list_u_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = p.K, S = p.S, SB = p.SB, d = p.d, NU = p.NU, kq = p.ukdp / 4;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  const int j = blockIdx.y, c = blockIdx.x, nch = gridDim.x;
  const int OT = S * SB, TS = (OT + 1) / 2 * 2, KP = p.ukdp + 1;
  const int WS = TS + (SB * KP + 1) / 2 * 2;
  double *tw = lds + (size_t)wave * WS;                 // [SB][S] Z tnu of the wave's pair
  double *uw = tw + TS;                                 // [SB][KP] its U columns
  double *red = lds + (size_t)kSuWaves * WS;           // [S][NU] | [S] | [S][S]
  double *zs = red + (size_t)S * NU + S + S * S;       // [d]
  for (int a = tid; a < d; a += 64 * kSuWaves) zs[a] = p.uz[a];
  // my moment columns: U feature (-1: the ones column), valid
  int ue[FPL];
  bool fv[FPL];
#pragma unroll
  for (int q = 0; q < FPL; ++q) {
    const int f = lane + 64 * q;
    fv[q] = f < NU;
    ue[q] = f == 0 ? -1 : f <= d ? NPF + f - 1 : f - 1 - d;
  }
  double acc[FPL][SM], accx[4], accn = 0.0;
#pragma unroll
  for (int q = 0; q < FPL; ++q)
#pragma unroll
    for (int s2 = 0; s2 < SM; ++s2) acc[q][s2] = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) accx[e] = 0.0;
  const int tot = p.list_tot[j];
  const int n0 = (int)((long long)tot * c / nch), n1 = (int)((long long)tot * (c + 1) / nch);
  const int *lst = p.list + (size_t)j * p.list_cap;
  const double *Ub0 = p.U + kUHead;
  for (int nb = n0 + wave; nb < n1; nb += 64 * kSuWaves) {
    // the bases of the next 64 pairs of this wave, one per lane
    const int nl = nb + lane * kSuWaves;
    const int il = nl < n1 ? lst[nl] : 0;
    const int np = min(64, (n1 - nb + kSuWaves - 1) / kSuWaves);
    for (int k = 0; k < np; ++k) {
      const int i = __builtin_amdgcn_readlane(il, k);
      const size_t lp = (size_t)(i - p.i_buf0) * K + j;
      const double z = p.Z[lp];
      // every load of the pair in flight before the first LDS write (a plain loop
      // waits on each load before its store)
      {
        double v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int x = lane + 64 * e;
          v[e] = x < OT ? p.tnu[lp * OT + x] : 0.0;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int x = lane + 64 * e;
          if (x < OT) {
            const int s2 = x / SB, b = x - s2 * SB;
            tw[b * S + s2] = z * v[e];
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int x = lane + 64 * e;
        if (x < S * S) accx[e] = fma(z, p.xi[lp * S * S + x], accx[e]);
      }
      if (lane < S) accn = fma(z, p.nu1[lp * S + lane], accn);
      const long long c0 = (long long)i * SB - p.u_col0;
      for (int x0 = lane; x0 < 4 * kq * SB; x0 += 64 * 8) {
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int x = x0 + 64 * e;
          const int t4 = x / SB, b = x - t4 * SB;  // t4 = 4 t + k: feature e
          const long long col = c0 + b;
          v[e] = x < 4 * kq * SB
                     ? Ub0[(size_t)(col >> 4) * kq * 64 + (t4 >> 2) * 64 + (t4 & 3) * 16 + (col & 15)]
                     : 0.0;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int x = x0 + 64 * e;
          const int t4 = x / SB, b = x - t4 * SB;
          if (x < 4 * kq * SB) uw[b * KP + t4] = v[e];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
      for (int b = 0; b < SM; ++b) {
        if (b < SB) {
          double uv[FPL];
#pragma unroll
          for (int q = 0; q < FPL; ++q)
            uv[q] = !fv[q] ? 0.0 : ue[q] < 0 ? 1.0 : uw[b * KP + ue[q]];
#pragma unroll
          for (int s2 = 0; s2 < SM; ++s2) {
            if (s2 < S) {
              const double tv = tw[b * S + s2];
#pragma unroll
              for (int q = 0; q < FPL; ++q) acc[q][s2] = fma(tv, uv[q], acc[q][s2]);
            }
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  // fixed-order reduction over the waves
  for (int w = 0; w < kSuWaves; ++w) {
    if (wave == w) {
#pragma unroll
      for (int q = 0; q < FPL; ++q)
#pragma unroll
        for (int s2 = 0; s2 < SM; ++s2) {
          const int f = lane + 64 * q;
          if (fv[q] && s2 < S) {
            double *r = red + (size_t)s2 * NU + f;
            *r = w == 0 ? acc[q][s2] : *r + acc[q][s2];
          }
        }
      if (lane < S) {
        double *r = red + (size_t)S * NU + lane;
        *r = w == 0 ? accn : *r + accn;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int x = lane + 64 * e;
        if (x < S * S) {
          double *r = red + (size_t)S * NU + S + x;
          *r = w == 0 ? accx[e] : *r + accx[e];
        }
      }
    }
    __syncthreads();
  }
  su_output(p, red, zs, c, nch, j, tid);
}

// ---------------------------------------------------------------------------
// stats_list_m_kernel<NTW, G, KSM, NXR, PD>: the gated sums on the MFMA pipe, from the
// statistics copy Us of the prepared operand.  For cluster j the emission moments are
//   acc[s][f] = sum over the gated pairs (i, j) and base states b of
//               (Z tnu)(s, b) * Us(i, b, f)
// i.e. one (16 x 4) x (4 x 16) v_mfma_f64_16x16x4f64 per k-slice of four base states
// and 16-feature tile: A = Z tnu (lane: state s = lane & 15, base state 4 kk + lane / 16;
// zero past S / SB; KSM = SBP / 4 k-slices), B = 16 consecutive features of four base
// states (one contiguous 512-byte segment of Us's tile-major block per load).  Block
// (c, j) = part c of cluster j's list, as stats_list_u_kernel.  Its 4 waves are G pair
// groups x 4 / G tile groups: wave w takes
// the part's pairs w % G, + G, ... and the feature tiles w / G + (4 / G) t, t < NTW,
// plus the sum_nu_1 | sum_xi entries lane + 64 (w / G + (4 / G) r).  The next PD - 1
// pairs' operands are in flight while a pair's MFMAs run (a register ring; the kernel is
// bound by memory latency, not by the MFMA pipe); no LDS in the loop.  The
// pair groups' sums are added in group order at the end (bit-reproducible).  Output
// as stats_list_u_kernel (shifted back by z).
// ---------------------------------------------------------------------------
constexpr int kSmWaves = 4;
static_assert(kSmWaves == kSuWaves, "su_output's thread stride");
typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int NTW, int G, int KSM, int NXR, int PD>
__global__ __launch_bounds__(64 * kSmWaves) void stats_list_m_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  constexpr int TG = kSmWaves / G;  // tile groups; NXR: sum_nu_1 | sum_xi chunks of 64 per wave
  // the wave index in an SGPR: the tile / pair-group tests below are scalar branches and
  // the loads' tile offsets scalar adds to the pair's base
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pg = wave % G, tg = wave / G;
  const int K = p.K, S = p.S, SB = p.SB, d = p.d, NU = p.NU;
  const int SBP = us_sbp(SB), NUP = us_nup(NU), ntile = NUP / 16;  // SBP = 4 KSM (launch)
  const int OT = S * SB, NX = S + S * S;
  // block -> (cluster j, part c of its list, parts nch): the gated pairs of all clusters
  // in parts of about P = total / (blocks - K) pairs, at most p.nzero (the slab count)
  // parts per cluster, at least one (an empty cluster's block writes its zeros)
  __shared__ int sm_map[3];
  if (wave == 0) {
    int total = 0;
    for (int x = lane; x < K; x += 64) total += p.list_tot[x];
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    const int nb = (int)gridDim.x, P = max(1, (total + max(1, nb - K) - 1) / max(1, nb - K));
    int pre = 0, jj = -1, cc = 0, np = 1;
    for (int x0 = 0; x0 < K && jj < 0; x0 += 64) {
      const int x = x0 + lane;
      int parts = 0;
      if (x < K) {
        const int t = p.list_tot[x], Pj = max(P, (t + p.nzero - 1) / p.nzero);
        parts = max(1, (t + Pj - 1) / Pj);
      }
      int inc = parts;  // inclusive prefix over the lanes
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
      }
      const int b0 = pre + inc - parts;  // this cluster's first block
      const bool hit = x < K && (int)blockIdx.x >= b0 && (int)blockIdx.x < b0 + parts;
      const unsigned long long m = __ballot(hit);
      if (m) {
        const int src = __builtin_ctzll(m);
        jj = __shfl(x, src, 64);
        cc = (int)blockIdx.x - __shfl(b0, src, 64);
        np = __shfl(parts, src, 64);
      }
      pre += __shfl(inc, 63, 64);
    }
    if (lane == 0) {
      sm_map[0] = jj;
      sm_map[1] = cc;
      sm_map[2] = np;
    }
  }
  __syncthreads();
  const int j = sm_map[0], c = sm_map[1], nch = sm_map[2];
  if (j < 0) return;  // past the last part (block-uniform)
  double *red = lds;                                  // [S][NU] | [S] | [S][S]
  double *zs = red + (size_t)S * NU + S + S * S;      // [d]
  for (int a = tid; a < d; a += 64 * kSmWaves) zs[a] = p.uz[a];
  const int kl = lane >> 4, cl = lane & 15;
  dbl4 acc[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
  double ax[NXR];
#pragma unroll
  for (int r = 0; r < NXR; ++r) ax[r] = 0.0;
  const int tot = p.list_tot[j];
  const int n0 = (int)((long long)tot * c / nch), n1 = (int)((long long)tot * (c + 1) / nch);
  const int *lst = p.list + (size_t)j * p.list_cap;
  // one pair's operands: A values per k-slice, B values per (tile, k-slice), its Z and
  // its sum_nu_1 / sum_xi entries; a ring of PD of them (PD - 1 pairs' loads in flight
  // while a pair's MFMAs run)
  struct Ops {
    double ta[KSM], ub[NTW][KSM], xv[NXR], z;
  };
  bool ta_ok[KSM];  // this lane's A entry (state cl, base state 4 kk + kl) exists
#pragma unroll
  for (int kk = 0; kk < KSM; ++kk) ta_ok[kk] = cl < S && 4 * kk + kl < SB;
  Ops buf[PD];
  auto load = [&](int i, Ops &o) {
    // wave-uniform bases (SGPRs), 32-bit lane offsets: saddr loads, no 64-bit address
    // arithmetic per lane
    const size_t lp = (size_t)(i - p.i_buf0) * K + j;
    // Z by a vector load (an address in VGPRs), in order with the pair's other loads: a
    // scalar load would be waited for (lgkmcnt(0)) at the start of the next pair
    unsigned zo = (unsigned)lp;  // (a 32-bit offset: the laundered pointer would be flat)
    asm("" : "+v"(zo));
    o.z = p.Z[zo];
    const double *us = p.Us + (size_t)i * SBP * NUP;
    const double *tp = p.tnu + lp * OT, *n1p = p.nu1 + lp * S, *xp = p.xi + lp * S * S;
    // lane-varying bounds by clamped (always valid) loads, not branches; the select that
    // zeroes the clamped lanes waits for compute (a select here would wait for the load,
    // and with it for every load issued before it: no prefetch at all)
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk) {
      const int b = 4 * kk + kl;
      o.ta[kk] = tp[ta_ok[kk] ? (unsigned)(cl * SB + b) : 0u];
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int ft = min(tg + TG * t, ntile - 1);  // past ntile: a repeat, never used
        o.ub[t][kk] = us[(unsigned)((ft * SBP + b) * 16 + cl)];  // b < SBP: in the block
      }
    }
    // one load from a lane-selected address (lanes past NX read xi[0]: their sums are
    // never stored)
#pragma unroll
    for (int r = 0; r < NXR; ++r) {
      const int x = lane + 64 * (tg + TG * r);
      o.xv[r] = *(x < S ? n1p + x : xp + (x < NX ? x - S : 0));
    }
  };
  auto compute = [&](const Ops &o) {
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk) {
      const double av = o.z * (ta_ok[kk] ? o.ta[kk] : 0.0);
#pragma unroll
      for (int t = 0; t < NTW; ++t)
        if (tg + TG * t < ntile) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, o.ub[t][kk], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < NXR; ++r) ax[r] = fma(o.z, o.xv[r], ax[r]);
  };
  // this wave's pairs: n0 + pg + G k, k < cnt.  The loop body is branch-free around the
  // loads (every slot loaded, the cursor clamped to the last pair; the list entries by
  // scalar loads one pair ahead), so the compiler's wait before a pair's MFMAs counts
  // exactly the PD - 1 later pairs' loads instead of draining them at a join.
  const int nf = n0 + pg;
  const int cnt = nf < n1 ? (n1 - nf + G - 1) / G : 0;
  if (cnt > 0) {  // wave-uniform
    const int kmax = cnt - 1;
    const int *lw = lst + nf;
#pragma unroll
    for (int u = 0; u < PD - 1; ++u) load(lw[G * min(u, kmax)], buf[u]);
    int inext = lw[G * min(PD - 1, kmax)];
    for (int k0 = 0; k0 < cnt; k0 += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        const int k = k0 + u;
        const int il = inext;
        inext = lw[G * min(k + PD, kmax)];
        load(il, buf[(u + PD - 1) % PD]);  // pair min(k + PD - 1, cnt - 1)
        if (k < cnt) compute(buf[u]);      // wave-uniform
      }
    }
  }
  // the pair groups' sums into the block's LDS record in group order, then su_output
  for (int g = 0; g < G; ++g) {
    if (pg == g) {
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int f = 16 * (tg + TG * t) + cl;
        if (tg + TG * t < ntile && f < NU)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int s2 = kl + 4 * v;
            if (s2 < S) {
              double *r = red + (size_t)s2 * NU + f;
              *r = g == 0 ? acc[t][v] : *r + acc[t][v];
            }
          }
      }
#pragma unroll
      for (int r = 0; r < NXR; ++r) {
        const int x = lane + 64 * (tg + TG * r);
        if (x < NX) {
          double *o = red + (size_t)S * NU + x;
          *o = g == 0 ? ax[r] : *o + ax[r];
        }
      }
    }
    __syncthreads();
  }
  su_output(p, red, zs, c, nch, j, tid);
}

// stats_list_g_kernel<LG, SM>: stats_list_u_kernel for small moment vectors
// (NU <= LG <= 32, e.g. d = 2 diag: NU = 5): a wavefront is 64 / LG lane groups, each
// taking its own pair (group g of wave w: pairs w G + g, + 4 G, ...), so a pair
// no longer leaves 59 of 64 lanes idle.  Per group a private LDS slab; the groups
// and waves reduce in fixed order (bit-reproducible), output as stats_list_u_kernel.
template <int LG, int SM>
__global__ __launch_bounds__(64 * kSuWaves) void stats_list_g_kernel(const StatsArgs p) {
  extern __shared__ double lds[];
  constexpr int NG = 64 / LG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = lane / LG, gl = lane - grp * LG;
  const int K = p.K, S = p.S, SB = p.SB, d = p.d, NU = p.NU, kq = p.ukdp / 4;
  const bool full = p.covmode == kCovFull;
  const int NPF = full ? d * (d + 1) / 2 : d;
  const int j = blockIdx.y, c = blockIdx.x, nch = gridDim.x;
  const int OT = S * SB, TS = (OT + 1) / 2 * 2, KP = p.ukdp + 1;
  const int WS = TS + (SB * KP + 1) / 2 * 2;
  double *tw = lds + (size_t)(wave * NG + grp) * WS;   // [SB][S] Z tnu of the group's pair
  double *uw = tw + TS;                                 // [SB][KP] its U columns
  double *red = lds + (size_t)kSuWaves * NG * WS;      // [S][NU] | [S] | [S][S]
  double *zs = red + (size_t)S * NU + S + S * S;       // [d]
  for (int a = tid; a < d; a += 64 * kSuWaves) zs[a] = p.uz[a];
  const bool fv = gl < NU;
  const int ue = gl == 0 ? -1 : gl <= d ? NPF + gl - 1 : gl - 1 - d;
  double acc[SM], accx[4], accn = 0.0;
#pragma unroll
  for (int s2 = 0; s2 < SM; ++s2) acc[s2] = 0.0;
#pragma unroll
  for (int e = 0; e < 4; ++e) accx[e] = 0.0;
  const int tot = p.list_tot[j];
  const int n0 = (int)((long long)tot * c / nch), n1 = (int)((long long)tot * (c + 1) / nch);
  const int *lst = p.list + (size_t)j * p.list_cap;
  const double *Ub0 = p.U + kUHead;
  const int nu4 = 4 * kq * SB;
  // wave-uniform trip count; a group past the part's end stages a zero-weight copy
  for (int nb = n0 + wave * NG; nb < n1; nb += kSuWaves * NG) {
    const int n = nb + grp;
    const bool pv = n < n1;
    const int i = lst[pv ? n : n0];
    const size_t lp = (size_t)(i - p.i_buf0) * K + j;
    const double z = pv ? p.Z[lp] : 0.0;
    double tv[4], xv[4], uv[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = gl + LG * e;
      tv[e] = x < OT ? p.tnu[lp * OT + x] : 0.0;
      xv[e] = x < S * S ? p.xi[lp * S * S + x] : 0.0;
    }
    const double nv = gl < S ? p.nu1[lp * S + gl] : 0.0;
    const long long c0 = (long long)i * SB - p.u_col0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int x = gl + LG * e;
      const int t4 = x / SB, b = x - t4 * SB;
      const long long col = c0 + b;
      uv[e] = x < nu4 ? Ub0[(size_t)(col >> 4) * kq * 64 + (t4 >> 2) * 64 + (t4 & 3) * 16 + (col & 15)]
                      : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int x = gl + LG * e;
      if (x < OT) {
        const int s2 = x / SB, b = x - s2 * SB;
        tw[b * S + s2] = z * tv[e];
      }
      accx[e] = fma(z, xv[e], accx[e]);
    }
    accn = fma(z, nv, accn);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int x = gl + LG * e;
      const int t4 = x / SB, b = x - t4 * SB;
      if (x < nu4) uw[b * KP + t4] = uv[e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (fv) {
#pragma unroll 1
      for (int b = 0; b < SB; ++b) {
        const double u = ue < 0 ? 1.0 : uw[b * KP + ue];
#pragma unroll
        for (int s2 = 0; s2 < SM; ++s2)
          if (s2 < S) acc[s2] = fma(tw[b * S + s2], u, acc[s2]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // fixed-order reduction: waves in order, and within a wave its groups in order
  // (exec-masked stores of one wavefront retire in program order)
  for (int w = 0; w < kSuWaves; ++w) {
    if (wave == w) {
      for (int g = 0; g < NG; ++g) {
        if (grp == g) {
          const bool first = w == 0 && g == 0;
#pragma unroll
          for (int s2 = 0; s2 < SM; ++s2)
            if (fv && s2 < S) {
              double *r = red + (size_t)s2 * NU + gl;
              *r = first ? acc[s2] : *r + acc[s2];
            }
          if (gl < S) {
            double *r = red + (size_t)S * NU + gl;
            *r = first ? accn : *r + accn;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int x = gl + LG * e;
            if (x < S * S) {
              double *r = red + (size_t)S * NU + S + x;
              *r = first ? accx[e] : *r + accx[e];
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    __syncthreads();
  }
  su_output(p, red, zs, c, nch, j, tid);
}

size_t gate_list_lds(int K) {
  const size_t ints = (size_t)2 * K + kListThreads / 64 + 2 * kListThreads;
  return (ints + 1) / 2 * 2 * sizeof(int) +
         (size_t)(kListThreads / 64) * K * sizeof(unsigned long long);
}

hipError_t launch_gate_list(const StatsArgs &a, int nchunk, hipStream_t st) {
  // the per-wave ballot masks grow with K: above 64 KB the launch needs the attribute
  // (the caller keeps the gated schedule only while this fits a CU, gate_list_lds)
  const size_t lds = gate_list_lds(a.K);
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&gate_list_kernel), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gate_list_kernel, dim3(nchunk), dim3(kListThreads), lds, st, a);
  return hipGetLastError();
}

namespace {
constexpr size_t kSlLdsBudget = 48 * 1024;
int sl_record(const StatsArgs &a) {
  const int OU = a.S * a.SB + a.S + a.S * a.S;
  return (OU + a.SB * a.NU + 1) / 2 * 2;
}
}  // namespace

bool plan_stats_list(StatsArgs &a, size_t &lds) {
  const size_t rs = (size_t)sl_record(a) * sizeof(double);
  const size_t tab = (size_t)(a.NU + 1) / 2 * 2 * sizeof(int);
  if (rs + tab + 12 > kSlLdsBudget) return false;
  // small batches: many resident blocks hide the gather latency (6 measured best at C4)
  a.PB = (int)std::min<size_t>(6, (kSlLdsBudget - tab) / (rs + 12));
  lds = (size_t)a.PB * (rs + 12) + tab;  // records + tab + Z / base index per pair
  return a.PB >= 1;
}

template <int FPL, int SM>
static hipError_t launch_su(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  const int OT = a.S * a.SB, KP = a.ukdp + 1;
  const size_t ws = (size_t)(OT + 1) / 2 * 2 + ((size_t)a.SB * KP + 1) / 2 * 2;
  const size_t lds = ((size_t)kSuWaves * ws + (size_t)a.S * a.NU + a.S + (size_t)a.S * a.S + a.d) *
                     sizeof(double);
  auto *fn = &stats_list_u_kernel<FPL, SM>;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, grid, dim3(64 * kSuWaves), lds, st, a);
  return hipGetLastError();
}

template <int NTW, int G, int KSM, int NXR, int PD>
static hipError_t launch_sm_pd(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  const size_t lds = ((size_t)a.S * a.NU + a.S + (size_t)a.S * a.S + a.d) * sizeof(double);
  auto *fn = &stats_list_m_kernel<NTW, G, KSM, NXR, PD>;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  // one generation of resident blocks (the kernel is latency-bound: a second round of
  // blocks repeats every block's start-up chain; C4: 1024 blocks 0.177 ms per step of
  // statistics, 2048 0.211, 4096 0.188 at the ring depth 2), at least one per cluster,
  // at most the slab count per cluster (grid.x is the cap from launch_stats_list)
  long long nb = (long long)resident_per_cu(reinterpret_cast<const void *>(fn), 64 * kSmWaves, lds) *
                 device_cus();
  if (const char *ev = std::getenv("VBHEM_SU_BLOCKS")) nb = std::atoll(ev);  // A/B
  nb = std::min<long long>(std::max<long long>(nb, a.K + 1), grid.x);
  hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(64 * kSmWaves), lds, st, a);
  return hipGetLastError();
}

// ring depth 3 since the load phase is branch-free (profiles/r05ad_ab_stats_ring_depth.txt:
// statistics per step C4 0.160 -> 0.155 ms, C5 4.7-4.9 -> 4.5-4.7 ms, shard and C3 equal;
// depth 4 in between).  Before that fix depth 3 lost: the ring never filled and its
// registers cost residency (C5 7.7 vs 5.8 ms)
#ifndef VBHEM_SM_PDD
#define VBHEM_SM_PDD 3   // the ring depth (build switch for A/B)
#endif
template <int NTW, int G, int KSM, int NXR>
static hipError_t launch_sm(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  return launch_sm_pd<NTW, G, KSM, NXR, VBHEM_SM_PDD>(a, grid, st);
}

// the sum_nu_1 | sum_xi chunks per wave: ceil(ceil((S + S^2) / 64) / tile groups)
template <int NTW, int G, int KSM>
static hipError_t launch_sm_x(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  constexpr int TG = kSmWaves / G;
  const int nxr = ((a.S + a.S * a.S + 63) / 64 + TG - 1) / TG;
  if (nxr <= 1) return launch_sm<NTW, G, KSM, 1>(a, grid, st);
  if (nxr <= 2) return launch_sm<NTW, G, KSM, 2>(a, grid, st);
  if (nxr <= 3) return launch_sm<NTW, G, KSM, 3>(a, grid, st);
  return launch_sm<NTW, G, KSM, 5>(a, grid, st);
}

// stats_list_m_kernel's variant: 4 pair groups (every wave all feature tiles) up to 4
// tiles (NU <= 64), 2 groups up to 8 tiles, else one group of 4 tile groups
// (C4: 1 or 2 pair groups measured 0.41 / 0.25 ms of statistics per step against 0.21)
template <int KSM>
static hipError_t launch_sm_k(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  const int nt = us_nup(a.NU) / 16;
  switch (nt) {
    case 1: return launch_sm_x<1, 4, KSM>(a, grid, st);
    case 2: return launch_sm_x<2, 4, KSM>(a, grid, st);
    case 3: return launch_sm_x<3, 4, KSM>(a, grid, st);
    case 4: return launch_sm_x<4, 4, KSM>(a, grid, st);
    case 5: case 6: return launch_sm_x<3, 2, KSM>(a, grid, st);
    case 7: case 8: return launch_sm_x<4, 2, KSM>(a, grid, st);
    default: return launch_sm_x<3, 1, KSM>(a, grid, st);
  }
}

template <int LG, int SM>
static hipError_t launch_sg(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  const int OT = a.S * a.SB, KP = a.ukdp + 1;
  const size_t ws = (size_t)(OT + 1) / 2 * 2 + ((size_t)a.SB * KP + 1) / 2 * 2;
  const size_t lds = ((size_t)kSuWaves * (64 / LG) * ws + (size_t)a.S * a.NU + a.S +
                      (size_t)a.S * a.S + a.d) * sizeof(double);
  auto *fn = &stats_list_g_kernel<LG, SM>;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(fn, grid, dim3(64 * kSuWaves), lds, st, a);
  return hipGetLastError();
}

// lanes per pair group for the grouped kernel (0: shape too large for it)
static int sg_lanes(const StatsArgs &a) {
  if (std::getenv("VBHEM_NO_STATS_G")) return 0;
  const int OT = a.S * a.SB, nu4 = a.ukdp * a.SB;
  for (int LG : {8, 16, 32})
    if (a.NU <= LG && OT <= 4 * LG && a.S * a.S <= 4 * LG && nu4 <= 8 * LG) return LG;
  return 0;
}

template <int LG>
static hipError_t launch_sg_s(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  if (a.S <= 4) return launch_sg<LG, 4>(a, grid, st);
  if (a.S <= 8) return launch_sg<LG, 8>(a, grid, st);
  if (a.S <= 12) return launch_sg<LG, 12>(a, grid, st);
  return launch_sg<LG, 16>(a, grid, st);
}

template <int FPL>
static hipError_t launch_su_s(const StatsArgs &a, const dim3 &grid, hipStream_t st) {
  if (a.S <= 4) return launch_su<FPL, 4>(a, grid, st);
  if (a.S <= 8) return launch_su<FPL, 8>(a, grid, st);
  if (a.S <= 12) return launch_su<FPL, 12>(a, grid, st);
  return launch_su<FPL, 16>(a, grid, st);
}

hipError_t launch_stats_list(const StatsArgs &a, int nchunk, size_t lds, hipStream_t st,
                             int *stats_slabs) {
  if (stats_slabs) *stats_slabs = nchunk;
  const int NO = a.S + a.S * a.S + a.S * a.NU;
  const dim3 grid(nchunk, a.K);
  const bool no_u = std::getenv("VBHEM_NO_STATS_U") != nullptr;
  // blocks of the list kernels on the prepared operand: the per-block cost (wave
  // reduction, slab writes) grows with the output count NO: at most ~4M block outputs
  // per launch (C4: 512 x 16 blocks of 432, C5: 64 x 32 of 1992 -- measured: 16384
  // blocks of 1992 ran 1.3x slower than 2048), and at most 4096 blocks in all (C4: 256
  // parts per cluster instead of 512, statistics 0.245 -> 0.231 ms; 3072 blocks 0.243,
  // 6144 0.235)
  const long long NOb = (long long)a.S + (long long)a.S * a.S + (long long)a.S * a.NU;
  long long cap = (4ll << 20) / (NOb * std::max(1, a.K));
  cap = std::min<long long>(cap, 4096 / std::max(1, a.K));
  if (const char *ev = std::getenv("VBHEM_SU_BLOCKS"))  // A/B
    cap = std::atoi(ev) / std::max(1, a.K);
  const int nb = (int)std::max(1ll, std::min((long long)nchunk, cap));
  const dim3 g2(nb, a.K);
  StatsArgs b = a;
  b.nzero = nchunk;
  const int lg = a.U ? sg_lanes(a) : 0;
  // the gate-list pass's flagged pairs (resp_kernel folded the backward pass's): an
  // fb_exact_kernel launch from flag_count[3] before any statistics kernel reads them.
  // (Folded into stats_list_m_kernel as well it measured no faster when nothing is
  // flagged -- its inlined fallback cost the kernel ~9 us at C4 -- and 3x slower when
  // every base is flagged: one worker wave per block there)
  if (a.fold == 1) {  // (2: the list kernel recomputed its flagged pairs itself)
    hipError_t e = launch_fb_exact(a.fx, a.xscratch, (size_t)a.xstride, kExactSlots, st, true);
    if (e != hipSuccess) return e;
  }
  // the MFMA kernel on the statistics copy Us (prepared base sets; S <= 16 rows of one
  // MFMA tile, SB <= 16, at most 12 feature tiles over 4 waves); also for the small
  // moment vectors of the grouped kernel (C3: statistics 0.039 -> 0.032 ms per step)
  // (it reads Z at the 32-bit offset (i - i_buf0) K + j: the base group times K must stay
  // below 2^32 -- always so for a workspace group, checked anyway)
  const bool z32 = (unsigned long long)(a.i_end - a.i_buf0) * (unsigned long long)a.K < (1ull << 32);
  if (a.Us && !no_u && z32 && a.S <= 16 && a.SB <= 16 && us_nup(a.NU) <= 12 * 16 &&
      !std::getenv("VBHEM_NO_STATS_M")) {
    // one 1-D grid over all clusters' gated pairs (balanced parts; the block maps
    // itself to (cluster, part)); at most nzero_m parts per cluster, so the slabs past
    // them hold none of its N1 / M / U entries (stats_final_kernel reads only those)
    if (a.nzero_m > 0) b.nzero = std::min(a.nzero_m, nchunk);
    if (stats_slabs) *stats_slabs = b.nzero;
    const dim3 g1((unsigned)std::min<long long>((long long)nchunk * a.K, 1ll << 30));
    switch (us_sbp(a.SB) / 4) {  // the k-slices of four base states, exact
      case 1: return launch_sm_k<1>(b, g1, st);
      case 2: return launch_sm_k<2>(b, g1, st);
      case 3: return launch_sm_k<3>(b, g1, st);
      default: return launch_sm_k<4>(b, g1, st);
    }
  }
  // on the prepared operand's tile layout when the call has one (S <= 16: the split
  // kernel's range) (NU > 64, e.g. d = 16 full at C5: the covariance gather of
  // stats_list_kernel measured 2 % faster, 1.74 vs 1.78 ms per 100 k-base step;
  // VBHEM_STATS_U=1 forces it)
  const bool su = a.NU <= 64 || std::getenv("VBHEM_STATS_U");
  if (a.U && su && a.S <= 16 && a.SB <= a.S && a.NU <= 3 * 64 && !no_u) {
    // the grouped kernel runs 64 / LG pairs per wave at once: half the blocks (C3,
    // 80 per cluster: statistics 0.047 -> 0.043 ms; with 156 it was 0.057)
    const dim3 gg(std::getenv("VBHEM_SU_BLOCKS") ? nb : std::max(1, nb / 2), a.K);
    switch (lg) {
      case 8: return launch_sg_s<8>(b, gg, st);
      case 16: return launch_sg_s<16>(b, gg, st);
      case 32: return launch_sg_s<32>(b, gg, st);
      default: break;
    }
    if (a.NU <= 64) return launch_su_s<1>(b, g2, st);
    if (a.NU <= 128) return launch_su_s<2>(b, g2, st);
    return launch_su_s<3>(b, g2, st);
  }
  if (NO <= 4 * kSlThreads) {
    hipLaunchKernelGGL((stats_list_kernel<4>), grid, dim3(kSlThreads), lds, st, a);
  } else {
    hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(&stats_list_kernel<8>), lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((stats_list_kernel<8>), grid, dim3(kSlThreads), lds, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_stats_final(const double *slabs, int nslab, int nslab_stats, int slab_len, int KT,
                              int S, int SL, double *out, hipStream_t st, int *fpre,
                              unsigned long long *done, unsigned long long done_val) {
  if (nslab_stats < 1 || nslab_stats > nslab || SL < 1 || slab_len % SL != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stats_final_kernel, dim3((slab_len + kFinalCols - 1) / kFinalCols), dim3(256),
                     0, st, slabs, nslab, nslab_stats, slab_len, KT, S, SL, out, fpre,
                     fpre ? flag_tag() : 0ull, fpre ? done : nullptr, done_val);
  return hipGetLastError();
}

}  // namespace vbhem

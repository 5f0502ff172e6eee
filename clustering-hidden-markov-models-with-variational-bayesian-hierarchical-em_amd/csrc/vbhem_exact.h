// vbhem_exact.h -- the reference-order recursion of one flagged pair (mex.c:715-1298
// step by step: K1, the backward LSE with stored Theta, termination, the forward sweep),
// shared by fb_exact_kernel and the kernels that fold the fallback into their prologue
// (resp_kernel, through fold_exact): one wavefront per pair
// (exact_pair_wave).  Internal.
#pragma once
#include <hip/hip_runtime.h>

#include "vbhem_internal.h"

namespace vbhem {

constexpr double kExactLog2Pi = 1.8378770664093454835606594728112353;  // log(2*pi)

// doubles per wavefront of exact_pair_wave: E, L, ls, Ln (= foo), nu, tn [S][SB],
// xi [S][S], l1 [SB], and the pair's inputs staged once: log A' [S][S], log pi [S],
// the base's A [SB][SB] and prior [SB]
static __host__ __device__ inline int exact_wave_lds(int S, int SB) {
  return 6 * S * SB + 2 * S * S + S + SB * SB + 2 * SB;
}

// the pair's small arrays live in LDS when they take at most 16 KB per wavefront (S = SB
// = 14 and below: 128 KB for fb_exact_kernel's 8 waves, 64 KB for resp_kernel's 4
// workers), else in the tail of the wave's global scratch slot
static __host__ __device__ inline bool exact_wave_in_lds(int S, int SB) {
  return exact_wave_lds(S, SB) <= 2048;
}

// wave-level ordering of the exchanges below (one wavefront works on one pair):
// LDS -- program order within the wave; global -- stores complete and the L1 lines
// dropped before other lanes read them
template <bool G>
static __device__ __forceinline__ void wave_sync() {
  if (G)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
  else
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// the reference-order recursion of one flagged pair with one WAVEFRONT: every element
// loop of mex.c:715-1298 spread over the lanes (lane = element, a pair's S x SB
// elements in ceil(S SB / 64) rounds), every sum in the reference's order.  Theta
// stays in the wave's global scratch slot w ([T][S][S][SB], then exact_wave_lds(S, SB)
// more doubles); the small arrays in the wavefront's LDS region lw (G = false: lw
// points into the kernel's __shared__ array, so every access compiles to an LDS
// instruction) or, G = true, in the slot's tail.
typedef __attribute__((address_space(3))) double lds_f64;  // an LDS double

template <bool G, class LP>
static __device__ __forceinline__ void exact_pair_body(const FbArgs &p, int pair, double *w, LP lw) {
  const int S = p.S, SB = p.SB, d = p.d, T = p.T, n = S * SB;
  auto wave_sync = []() { vbhem::wave_sync<G>(); };
  // the lane index, opaque to the optimizer at every use: otherwise each element loop's
  // per-lane addresses are hoisted out of the step loops, ~40 registers more than the
  // kernels that inline this function can spare (resp_kernel keeps 4 waves per SIMD)
  auto lane_id = []() {
    int l = (int)(threadIdx.x & 63);
    __asm__ volatile("" : "+v"(l));
    return l;
  };
  const LP E = lw, L = E + n, ls = L + n, Ln = ls + n, nu = Ln + n, tn = nu + n, xi = tn + n,
           l1 = xi + S * S, la = l1 + SB, lpj = la + S * S, Ab = lpj + S, pb = Ab + SB * SB;
  const int i = pair / p.K, j = pair - (pair / p.K) * p.K;
  const size_t lp = (size_t)(i - p.i_buf0) * p.K + j;
  {
    const int lane = lane_id();
    const double *Ag = p.A + (size_t)i * SB * SB, *pg = p.prior + (size_t)i * SB;
    const double *lag = p.logA + (size_t)j * S * S, *lpg = p.logPi + (size_t)j * S;
    for (int e = lane; e < S * S; e += 64) la[e] = lag[e];
    for (int e = lane; e < SB * SB; e += 64) Ab[e] = Ag[e];
    for (int e = lane; e < S; e += 64) lpj[e] = lpg[e];
    for (int e = lane; e < SB; e += 64) pb[e] = pg[e];
  }
  // K1 (mex.c:715-880): lane (s, be)
  for (int e = lane_id(); e < n; e += 64) {
    const int s = e / SB, be = e - s * SB;
    const double *mm = p.m + ((size_t)j * S + s) * d;
    const double *mu = p.centres + ((size_t)i * SB + be) * d;
    double ell = d * kExactLog2Pi + p.c[(size_t)j * S + s];
    if (p.covmode == kCovFull) {
      const double *P = p.P + ((size_t)j * S + s) * d * d;
      const double *C = p.covars + ((size_t)i * SB + be) * d * d;
      for (int k = 0; k < d * d; ++k) ell += P[k] * C[k];
      for (int c2 = 0; c2 < d; ++c2) {
        double col = 0.0;
        for (int r = 0; r < d; ++r) col += (mu[r] - mm[r]) * P[r * d + c2];
        ell += col * (mu[c2] - mm[c2]);
      }
    } else {
      const double *P = p.P + ((size_t)j * S + s) * d;
      const double *C = p.covars + ((size_t)i * SB + be) * d;
      for (int r = 0; r < d; ++r) {
        const double x = mu[r] - mm[r];
        ell += P[r] * C[r];
        ell += P[r] * (x * x);
      }
    }
    E[e] = p.smooth != 1.0 ? (-0.5 * ell) / p.smooth : -0.5 * ell;
    L[e] = 0.0;
  }
  wave_sync();
  // K2 (mex.c:915-1080), steps T-1 .. 1
  for (int t = T - 1; t >= 1; --t) {
    double *Tt = w + (size_t)t * S * S * SB;  // Theta_t [S][S][SB]
    // lane (rho, be): the column log-sum-exp of rho's lt over sigma and rho's Theta_t
    for (int e = lane_id(); e < n; e += 64) {
      const int rho = e / SB, be = e - rho * SB;
      const LP lar = la + rho * S, Eb = E + be, Lb = L + be;
      double mv = lar[0] + Eb[0] + Lb[0];
      for (int s2 = 1; s2 < S; ++s2) mv = fmax(mv, lar[s2] + Eb[s2 * SB] + Lb[s2 * SB]);
      double acc = 0.0;
#pragma unroll 1
      for (int s2 = 0; s2 < S; ++s2) acc += exp(lar[s2] + Eb[s2 * SB] + Lb[s2 * SB] - mv);
      const double lsv = mv + log(acc);
      ls[e] = lsv;
      double *Tr = Tt + rho * S * SB + be;
#pragma unroll 1
      for (int s2 = 0; s2 < S; ++s2) Tr[s2 * SB] = exp(lar[s2] + Eb[s2 * SB] + Lb[s2 * SB] - lsv);
    }
    wave_sync();
    // lane (rho, g): Ln[rho][g] = sum_be Ab[g][be] ls[rho][be]
    for (int e = lane_id(); e < n; e += 64) {
      const int rho = e / SB, g = e - rho * SB;
      double acc = 0.0;
      for (int be = 0; be < SB; ++be) acc += Ab[g * SB + be] * ls[rho * SB + be];
      Ln[e] = acc;
    }
    wave_sync();
    for (int e = lane_id(); e < n; e += 64) L[e] = Ln[e];
    wave_sync();
  }
  // K3 (mex.c:1080-1130): lane be
  for (int be = lane_id(); be < SB; be += 64) {
    double mv = lpj[0] + E[be] + L[be];
    for (int s2 = 1; s2 < S; ++s2) mv = fmax(mv, lpj[s2] + E[s2 * SB + be] + L[s2 * SB + be]);
    double acc = 0.0;
#pragma unroll 1
    for (int s2 = 0; s2 < S; ++s2) acc += exp(lpj[s2] + E[s2 * SB + be] + L[s2 * SB + be] - mv);
    const double lv = mv + log(acc);
    l1[be] = lv;
#pragma unroll 1
    for (int s2 = 0; s2 < S; ++s2)
      nu[s2 * SB + be] = pb[be] * exp(lpj[s2] + E[s2 * SB + be] + L[s2 * SB + be] - lv);
  }
  wave_sync();
  {
    const int lane = lane_id();
    if (lane == 0) {
      double LLv = 0.0;
      for (int be = 0; be < SB; ++be) LLv += pb[be] * l1[be];
      p.LL[pair] = LLv;
    }
    for (int s2 = lane; s2 < S; s2 += 64) {
      double acc = 0.0;
      for (int be = 0; be < SB; ++be) acc += nu[s2 * SB + be];
      p.nu1[lp * S + s2] = acc;
    }
    for (int e = lane; e < n; e += 64) tn[e] = nu[e];
    for (int e = lane; e < S * S; e += 64) xi[e] = 0.0;
  }
  // Theta_t written by other lanes is read below: device-scope fence (stores done,
  // no stale L1 lines from the slot's previous pair)
  __threadfence();
  wave_sync();
  // K4 (mex.c:1130-1298), steps 1 .. T-1
  for (int t = 1; t < T; ++t) {
    const double *Tt = w + (size_t)t * S * S * SB;
    const LP foo = Ln;
    for (int e = lane_id(); e < n; e += 64) {  // lane (rho, g)
      const int rho = e / SB, g = e - rho * SB;
      double acc = 0.0;
      for (int be = 0; be < SB; ++be) acc += nu[rho * SB + be] * Ab[be * SB + g];
      foo[e] = acc;
    }
    wave_sync();
    for (int e = lane_id(); e < S * S; e += 64) {  // lane (rho, s): xi[rho][s]
      const int rho = e / S, s2 = e - rho * S;
      const double *Tr = Tt + (rho * S + s2) * SB;
      const LP fr = foo + rho * SB;
      double acc = 0.0;
      for (int g = 0; g < SB; ++g) acc += fr[g] * Tr[g];
      xi[e] += acc;
    }
    for (int e = lane_id(); e < n; e += 64) {  // lane (s, g): nu[s][g]
      const int s2 = e / SB, g = e - s2 * SB;
      const double *Tc = Tt + s2 * SB + g;
      double acc = 0.0;
      for (int rho = 0; rho < S; ++rho) acc += foo[rho * SB + g] * Tc[rho * S * SB];
      nu[e] = acc;
    }
    wave_sync();
    for (int e = lane_id(); e < n; e += 64) tn[e] += nu[e];
    wave_sync();
  }
  {
    const int lane = lane_id();
    for (int e = lane; e < n; e += 64) p.tnu[lp * S * SB + e] = tn[e];
    for (int e = lane; e < S * S; e += 64) p.xi[lp * S * S + e] = xi[e];
  }
  wave_sync();
}

template <bool G>
static __device__ __forceinline__ void exact_pair_wave(const FbArgs &p, int pair, double *w,
                                                       double *lw) {
  if (G)
    exact_pair_body<true>(p, pair, w, w + (size_t)p.T * p.S * p.S * p.SB);
  else
    exact_pair_body<false>(p, pair, w, (lds_f64 *)lw);
}

// dynamic LDS a folding kernel adds for nw worker waves: the queue (threads + 1 ints,
// rounded to doubles) and, when they fit, the waves' regions
static __host__ __device__ inline size_t fold_lds_bytes(int threads, int nw, int S, int SB) {
  const size_t qb = ((size_t)(threads + 1) * sizeof(int) + 7) / 8 * 8;
  return qb + (exact_wave_in_lds(S, SB) ? (size_t)nw * exact_wave_lds(S, SB) * sizeof(double) : 0);
}

// The exact fallback folded into a consumer kernel's prologue (resp_kernel):
// the flagged pairs flag_list[x0, x1) that `mine` accepts are
// found by the whole block, blockDim entries per round (coalesced), queued in LDS
// (q [blockDim], *qn), and recomputed by the block's first `nw` WAVEFRONTS
// (exact_pair_wave), wave k on scratch slot slot0 + k and LDS region lw + k *
// exact_wave_lds(S, SB) (G: the slots' tails) -- the block's own slots,
// so no two waves of the grid share one.  Block-uniform: every thread calls it; it
// ends with a barrier.
template <bool G, class Mine>
static __device__ __forceinline__ void fold_exact(const FbArgs &fx, int x0, int x1, Mine mine,
                                                  double *scratch, long long stride, int slot0,
                                                  int nw, int *q, int *qn, double *lw) {
  const int tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6;
  const int lws = exact_wave_lds(fx.S, fx.SB);
  #pragma unroll 1
  for (int b = x0; b < x1; b += nt) {
    if (tid == 0) *qn = 0;
    __syncthreads();
    const int x = b + tid;
    if (x < x1) {
      const int pair = fx.flag_list[x];
      if (mine(pair)) q[atomicAdd(qn, 1)] = pair;
    }
    __syncthreads();
    const int n = *qn;
    if (wave < nw)
      #pragma unroll 1
      for (int y = wave; y < n; y += nw)
        exact_pair_wave<G>(fx, q[y], scratch + (size_t)(slot0 + wave) * stride,
                           G ? nullptr : lw + (size_t)wave * lws);
    __syncthreads();
  }
}

}  // namespace vbhem

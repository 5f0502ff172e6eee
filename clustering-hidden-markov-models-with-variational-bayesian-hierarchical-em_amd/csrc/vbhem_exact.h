// vbhem_exact.h -- the reference-order recursion of one flagged pair (mex.c:715-1298
// step by step: K1, the backward LSE with stored Theta, termination, the forward sweep),
// shared by fb_exact_kernel and the kernels that fold the fallback into their prologue
// (resp_kernel, stats_list_m_kernel, through fold_exact).  w: the thread's scratch slot (exact_stride doubles:
// E, L, Ln, lt, nu, tn [S][SB] each, ls [SB], Theta [T][S][S][SB]).  Internal.
#pragma once
#include <hip/hip_runtime.h>

#include "vbhem_internal.h"

namespace vbhem {

constexpr double kExactLog2Pi = 1.8378770664093454835606594728112353;  // log(2*pi)

static __device__ __forceinline__ void exact_pair(const FbArgs &p, int pair, double *w) {
  const int S = p.S, SB = p.SB, d = p.d, T = p.T;
  double *E = w, *L = E + S * SB, *Ln = L + S * SB, *lt = Ln + S * SB, *nu = lt + S * SB,
         *tn = nu + S * SB, *ls = tn + S * SB, *Th = ls + SB;  // Th [T][S][S][SB]
  const int i = pair / p.K, j = pair - (pair / p.K) * p.K;
  const size_t lp = (size_t)(i - p.i_buf0) * p.K + j;
  const double *Ab = p.A + (size_t)i * SB * SB;
  const double *pb = p.prior + (size_t)i * SB;
  const double *la = p.logA + (size_t)j * S * S;
  const double *lpj = p.logPi + (size_t)j * S;
  for (int s = 0; s < S; ++s)
    for (int be = 0; be < SB; ++be) {
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
      E[s * SB + be] = p.smooth != 1.0 ? (-0.5 * ell) / p.smooth : -0.5 * ell;
      L[s * SB + be] = 0.0;
    }
  for (int t = T - 1; t >= 1; --t) {
    for (int rho = 0; rho < S; ++rho) {
      for (int s = 0; s < S; ++s)
        for (int be = 0; be < SB; ++be) lt[s * SB + be] = la[rho * S + s] + E[s * SB + be] + L[s * SB + be];
      for (int be = 0; be < SB; ++be) {
        double mv = lt[be];
        for (int s = 1; s < S; ++s) mv = fmax(mv, lt[s * SB + be]);
        double acc = 0.0;
        for (int s = 0; s < S; ++s) acc += exp(lt[s * SB + be] - mv);
        ls[be] = mv + log(acc);
        for (int s = 0; s < S; ++s)
          Th[(((size_t)t * S + rho) * S + s) * SB + be] = exp(lt[s * SB + be] - ls[be]);
      }
      for (int g = 0; g < SB; ++g) {
        double acc = 0.0;
        for (int be = 0; be < SB; ++be) acc += Ab[g * SB + be] * ls[be];
        Ln[rho * SB + g] = acc;
      }
    }
    for (int k = 0; k < S * SB; ++k) L[k] = Ln[k];
  }
  double LLv = 0.0;
  for (int s = 0; s < S; ++s)
    for (int be = 0; be < SB; ++be) lt[s * SB + be] = lpj[s] + E[s * SB + be] + L[s * SB + be];
  for (int be = 0; be < SB; ++be) {
    double mv = lt[be];
    for (int s = 1; s < S; ++s) mv = fmax(mv, lt[s * SB + be]);
    double acc = 0.0;
    for (int s = 0; s < S; ++s) acc += exp(lt[s * SB + be] - mv);
    const double l1 = mv + log(acc);
    LLv += pb[be] * l1;
    for (int s = 0; s < S; ++s) nu[s * SB + be] = pb[be] * exp(lt[s * SB + be] - l1);
  }
  p.LL[pair] = LLv;
  for (int s = 0; s < S; ++s) {
    double acc = 0.0;
    for (int be = 0; be < SB; ++be) acc += nu[s * SB + be];
    p.nu1[lp * S + s] = acc;
  }
  for (int k = 0; k < S * SB; ++k) tn[k] = nu[k];
  // sum_xi accumulates in the thread's own scratch (Theta's slice t = 0, never used
  // by the recursion) and is stored once at the end: a pair listed twice in one
  // fallback launch (flagged by both passes) is then two threads storing the same
  // values, never two threads adding into the same output
  double *xi = Th;
  for (int k = 0; k < S * S; ++k) xi[k] = 0.0;
  for (int t = 1; t < T; ++t) {
    double *foo = Ln;
    for (int rho = 0; rho < S; ++rho)
      for (int g = 0; g < SB; ++g) {
        double acc = 0.0;
        for (int be = 0; be < SB; ++be) acc += nu[rho * SB + be] * Ab[be * SB + g];
        foo[rho * SB + g] = acc;
      }
    for (int s = 0; s < S; ++s) {
      for (int rho = 0; rho < S; ++rho) {
        double acc = 0.0;
        for (int g = 0; g < SB; ++g)
          acc += foo[rho * SB + g] * Th[(((size_t)t * S + rho) * S + s) * SB + g];
        xi[rho * S + s] += acc;
      }
      for (int g = 0; g < SB; ++g) {
        double acc = 0.0;
        for (int rho = 0; rho < S; ++rho)
          acc += foo[rho * SB + g] * Th[(((size_t)t * S + rho) * S + s) * SB + g];
        nu[s * SB + g] = acc;
      }
    }
    for (int k = 0; k < S * SB; ++k) tn[k] += nu[k];
  }
  for (int k = 0; k < S * SB; ++k) p.tnu[lp * S * SB + k] = tn[k];
  for (int k = 0; k < S * S; ++k) p.xi[lp * S * S + k] = xi[k];
}

// The exact fallback folded into a consumer kernel's prologue (resp_kernel,
// stats_list_m_kernel): the flagged pairs flag_list[x0, x1) that `mine` accepts are
// found by the whole block, blockDim entries per round (coalesced), queued in LDS
// (q [blockDim], *qn), and recomputed by the block's first `nw` threads, thread t on
// scratch slot slot0 + t -- the block's own slots, so no two threads of the grid
// share one.  A block whose bases were all flagged (a diverged trial) runs its
// pairs nw at a time instead of one after another.  Block-uniform: every thread
// calls it; it ends with a barrier.
template <class Mine>
static __device__ __forceinline__ void fold_exact(const FbArgs &fx, int x0, int x1, Mine mine,
                                                  double *scratch, long long stride, int slot0,
                                                  int nw, int *q, int *qn) {
  const int tid = threadIdx.x, nt = blockDim.x;
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
    if (tid < nw)
      for (int y = tid; y < n; y += nw) exact_pair(fx, q[y], scratch + (size_t)(slot0 + tid) * stride);
    __syncthreads();
  }
}

}  // namespace vbhem

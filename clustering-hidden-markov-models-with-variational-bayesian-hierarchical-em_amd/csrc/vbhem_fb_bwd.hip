// vbhem_fb_bwd.hip -- the gated schedule's backward-only pass for S <= 16: K2 (the
// backward recursion, mex.c:915-1015) and K3 (termination, mex.c:1020-1080) for
// EVERY pair, writing L_elbo; the forward quantities of the gated pairs come from
// fb_split_kernel's list mode afterwards (vbhem_fb_split.hip).
//
// Why a kernel of its own (measured): the backward sweep is
// fp64-VALU bound with no MFMA to offload to (on gfx950 v_mfma_f64_* and the fp64
// VALU do not run concurrently: scripts/ubench_valu.hip), and in fb_split_kernel's
// one-column-per-lane layout a third of the kernel time went to waiting on the
// scalar loads of the cluster matrix A' (64 doubles do not fit the 102 SGPRs, so
// every step reloaded them).  Here A' is spread over the 16 lanes of each DPP row
// and applied by v_fmac_f64 with a row_newbcast operand, and for S <= 8 every lane
// owns TWO base-state columns of its pair, so each broadcast and each slab read
// feeds two FMAs and the lane has twice the independent exp/log chains.
//
// Layout.  CPL = 2 (S <= 8) or 1 columns per lane, LPP = ceil(S/CPL) lanes per
// pair, PPW = floor(64/LPP) pairs per wavefront (pairs never straddle a wavefront:
// every exchange is wave-local), one cluster j per block, tiles of one wavefront's
// PPW consecutive bases dealt wave-major.  Lane w of a pair owns columns b = w (and
// b = w + LPP) (padded columns past SB duplicate column SB-1 with zero base
// transitions and prior: exact no-ops, as in fb_split_kernel).  In registers per
// column: Ef[S], V[S] = Ef + Lf, arow[S] (Ab row b).  Per step:
//   M = max_s V, G = exp(V - M)                       (table exp, LDS table)
//   Z = A' G                                          (A' rows by DPP broadcast)
//   sv = M + log Z                                    (table log, LDS table)
//   V = Ef + sum_b' Ab[b][b'] sv[.][b']               (per-pair LDS slab)
// with the cluster row maxima folded out of the loop: A' = exp(logA - amax),
// sv_ref = sv + amax, so L_ref = Lf + amax * rowsum(Ab) and E + L_ref = Ef + Lf
// with Ef = E + amax * rowsum(Ab) (once per pair).  exp / log are the
// short-series exp_tabe_n / log_tabe_n (vbhem_math.h): 8 fp64 operations each.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "vbhem_internal.h"
#include "vbhem_log_table.h"
#include "vbhem_math.h"

// waves per SIMD the kernel is compiled for (register budget 512 / W)
#ifndef VBHEM_BWD2_WAVES
#define VBHEM_BWD2_WAVES(S) ((S) <= 12 ? 3 : 2)
#endif
// slab column padding past the even row length (doubles; build switch for A/B)
#ifndef VBHEM_BWD2_XPAD
#define VBHEM_BWD2_XPAD(S) 2
#endif

namespace vbhem {

namespace {

// underflow guard of the column sums Z (the fallback to fb_exact_kernel):
// Z < 2^-665 (~7.6e-201), tested on the high word as a signed integer (negative Z,
// zero and denormals below it too); NaN shows in the pair's termination value
constexpr int kZMinHi = 0x16600000;
alignas(16) __device__ const double kLogTabB[2 * kLogTabEEntries] = VBHEM_LOG1024_TABLE_INIT;
alignas(16) __device__ const double kExpTabB[kExpTabEEntries] = VBHEM_EXP2048_TABLE_INIT;

// LDS tables of exp_tabe_n / log_tabe_n (vbhem_math.h), 16 KB each: staged once
// per block, one block per CU
constexpr int kTabExpD = kExpTabEEntries;       // 2048 doubles
constexpr int kTabLogD = 2 * kLogTabEEntries;   // 2048 doubles
constexpr int kTabD = kTabExpD + kTabLogD;

// acc += bcast(a from lane N of this lane's 16-lane row) * b: v_fmac_f64 with DPP
// row_newbcast, the one DPP control the fp64 ALU takes
template <int N>
__device__ __forceinline__ void dpp_fmac_bcast(double &acc, double a, double b) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(a), "v"(b), "i"(N));
}

// max of v[0..N) as a balanced tree (dependency depth log2 N instead of N - 1)
template <int N, int O = 0>
__device__ __forceinline__ double tree_max_at(const double *v) {
  if constexpr (N == 1) return v[O];
  else return fmax(tree_max_at<N / 2, O>(v), tree_max_at<N - N / 2, O + N / 2>(v));
}
template <int N>
__device__ __forceinline__ double tree_max(const double (&v)[N]) {
  return tree_max_at<N>(v);
}

// f(integral_constant<int, I>) for I = B .. E-1, in order
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int S>
struct Bwd2Layout {
  static constexpr int CPL = S <= 8 ? 2 : 1;         // base-state columns per lane
  static constexpr int LPP = (S + CPL - 1) / CPL;    // lanes per pair
  static constexpr int PPW = 64 / LPP;               // pairs per wavefront
  static constexpr int NA = (S * S + 15) / 16 > 4 ? (S * S + 15) / 16 : 4;  // A' doubles per lane
  static constexpr int SP = CPL * LPP;               // slab columns (padded)
  static constexpr int XCS = (S + 1) / 2 * 2 + VBHEM_BWD2_XPAD(S);  // slab column stride (even: 16-B rows)
  static constexpr int XP = SP * XCS + 2;            // per-pair slab (doubles)
  static constexpr int OFF_CL = 0;                   // amax [S], lpi [S] (dynamic LDS)
  // the in-kernel K1's cluster operands (SplitArgs::eU): W' [kdp <= 8][S], bias' [S]
  static constexpr int OFF_K1 = 2 * S;
  static constexpr int OFF_X = (2 * S + (kK1InKernelMaxKdp + 1) * S + 1) / 2 * 2;
};

}  // namespace

template <int S>
__global__ __launch_bounds__(256 * VBHEM_BWD2_WAVES(S)) __attribute__((amdgpu_waves_per_eu(VBHEM_BWD2_WAVES(S))))
void fb_bwd2_kernel(const SplitArgs p) {
  // the tables in static LDS (offset 0: table addresses fold into the ds_read
  // offsets), the per-pair state in the dynamic part after them
  __shared__ __attribute__((aligned(16))) double tabs[kTabD];
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using LY = Bwd2Layout<S>;
  constexpr int LPP = LY::LPP, PPW = LY::PPW, CPL = LY::CPL, NA = LY::NA;
  const int tid = threadIdx.x, NT = blockDim.x, NW = NT >> 6;
  const int PPB = NW * PPW;
  const int SB = p.SB, K = p.K, T = p.T;
  double *etab = tabs;                   // [2048]
  double *ltab = tabs + kTabExpD;        // [1024][2] of {1/(2c), -log(1/c)}
  double *amax = lds + LY::OFF_CL;       // [S]
  double *lpi = amax + S;                // [S]
  double *Xall = lds + LY::OFF_X;        // [PPB][XP]
  int *F = reinterpret_cast<int *>(Xall + (size_t)PPB * LY::XP);  // [PPB]

  for (int x = tid; x < kTabExpD; x += NT) etab[x] = kExpTabB[x];
  for (int x = tid; x < kTabLogD; x += NT) ltab[x] = kLogTabB[x];
  // persistent: NB blocks per cluster; XCD-aware when NB % 8 == 0 (the K blocks
  // walking the same bases share one XCD's L2, as fb_split_kernel's backward mode)
  const int bk = blockIdx.x, NB = (int)gridDim.x / K;
  int j, t0;
  if (NB % 8 == 0) {
    const int r = bk / 8;
    j = r % K;
    t0 = (r / K) * 8 + bk % 8;
  } else {
    j = bk % K;
    t0 = bk / K;
  }
  j = __builtin_amdgcn_readfirstlane(j);
  if (tid < S) {
    const double *la = p.logA + ((size_t)j * S + tid) * S;
    double mx = la[0];
    for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[s2]);
    amax[tid] = mx;
    lpi[tid] = p.logPi[(size_t)j * S + tid];
  }
  // in-kernel K1 (p.eU): cluster j's W' columns and bias' staged once per block, read
  // as LDS broadcasts by every tile's prologue
  double *k1w = lds + LY::OFF_K1;  // [kdp][S], then bias' [S]
  // cluster j's A' = exp(logA - rowmax) (prep: computed here, else staged from Atg) in
  // the lattice space until the tiles start
  double *Ast = Xall;
  if (p.eU && p.prep) {
    // emission_prep_kernel's work for cluster j (same arithmetic, vbhem_internal.h em_*):
    // wave 1 the W' columns and bias' of rows j S + s, waves 2.. A', wave 7 the flag head
    const int s = tid - 64, d = p.d, kdp = p.ekdp;
    if (s >= 0 && s < S) {
      const int r = j * S + s;
      const double *mr = p.pm + (size_t)r * d, *zs = p.pz;
      double q = 0.0;
      int e = 0;
      if (p.covmode == kCovFull) {
        const double *P = p.pP + (size_t)r * d * d;
        for (int a = 0; a < d; ++a)  // packed upper (a <= b), row-major
          for (int b = a; b < d; ++b) k1w[(e++) * S + s] = em_w_full(P, a, b, d);
        for (int a = 0; a < d; ++a) {
          const double v = em_pm_full(P, mr, zs, a, d);
          k1w[(e++) * S + s] = v;
          q = fma(mr[a] - zs[a], v, q);
        }
      } else {
        const double *P = p.pP + (size_t)r * d;
        for (int a = 0; a < d; ++a) k1w[(e++) * S + s] = -0.5 * P[a];
        for (int a = 0; a < d; ++a) {
          const double ma = mr[a] - zs[a];
          k1w[(e++) * S + s] = P[a] * ma;
          q = fma(P[a] * ma, ma, q);
        }
      }
      for (; e < kdp; ++e) k1w[e * S + s] = 0.0;
      k1w[kdp * S + s] = em_bias(d, p.pc[r], q);
    }
    const int x = tid - 128;
    if (x >= 0 && x < S * S) {
      const int r = x / S, k = x - r * S;
      const double *la = p.logA + ((size_t)j * S + r) * S;
      double mx = la[0];
      for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[s2]);
      Ast[x] = exp_nonpos(la[k] - mx);
    }
    if (tid == 448) {
      // the counters are clean when the last call closed them (stats_final_kernel wrote
      // the tag); else block 0 zeroes them and publishes the tag while the other blocks
      // wait for it (block 0 is dispatched first and never waits)
      if (__hip_atomic_load(p.ftag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != p.ftag_val) {
        if (bk == 0) {
          for (int c = 0; c < kFlagHead; ++c)
            __hip_atomic_store(p.flag_count + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.ftag, p.ftag_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          // bounded (a lost tag must not hang the device): ~2^22 polls
          bool seen = false;
          for (int g = 0; g < (1 << 22) && !seen; ++g) {
            seen = __hip_atomic_load(p.ftag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == p.ftag_val;
            if (!seen) __builtin_amdgcn_s_sleep(4);
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          // timed out: pairs this block flags may be zeroed away by block 0, so the
          // call's results cannot be trusted -- the sticky word [3] of the flag head
          // makes stats_final_kernel write NaN statistics (loud, never silent)
          if (!seen)
            __hip_atomic_store(reinterpret_cast<int *>(p.ftag) + kFlagLost, kFlagLostMark, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  } else {
    if (p.eU) {
      for (int x = tid; x < p.ekdp * S; x += NT) {
        const int e = x / S, k = x - e * S;
        k1w[x] = p.eW[(size_t)e * p.eksp + (size_t)j * S + k];
      }
      for (int k = tid; k < S; k += NT) k1w[p.ekdp * S + k] = p.ebias[(size_t)j * S + k];
    }
    for (int x = tid; x < S * S; x += NT) Ast[x] = p.Atg[(size_t)j * S * S + x];
  }
  __syncthreads();
  const bool prep = p.eU && p.prep;
  if (prep && t0 == 0) {
    // the first block of cluster j: its W' / bias' / A' for the gate-list pass (and the
    // padding k-rows of W'), block 0 the shift
    double *gW = const_cast<double *>(p.eW), *gb = const_cast<double *>(p.ebias);
    double *gA = const_cast<double *>(p.Atg);
    for (int x = tid; x < p.ekdp * S; x += NT) {
      const int e = x / S, k = x - e * S;
      gW[(size_t)e * p.eksp + (size_t)j * S + k] = k1w[x];
    }
    for (int k = tid; k < S; k += NT) gb[(size_t)j * S + k] = k1w[p.ekdp * S + k];
    for (int x = tid; x < S * S; x += NT) gA[(size_t)j * S * S + x] = Ast[x];
    if (bk == 0)
      for (int a = tid; a < p.d; a += NT) p.pshift[a] = p.pz[a];
  }

  const int lane = tid & 63, wave = tid >> 6;
  const int qw = lane / LPP, w = lane - qw * LPP;
  const bool valid = qw < PPW;
  const int q = wave * PPW + (valid ? qw : 0);
  double *X = Xall + (size_t)q * LY::XP;
  // wave-granular tiles of PPW pairs, dealt wave-major over the cluster's NB blocks
  // (wave w of block t0 takes tiles w NB + t0, + NB NW, ...): the tiles left over
  // past a whole number of rounds land one per CU instead of all on the first
  // blocks' CUs (small shards: 12 500 bases = 4.07 rounds ran as 5)
  const int ntile = (p.i_end - p.i_begin + PPW - 1) / PPW;
  // A' spread over the 16 lanes of every DPP row: entry e = r S + k in register e % NA
  // of row lane e / NA (16 NA >= S^2)
  double aq[NA];
#pragma unroll
  for (int x = 0; x < NA; ++x) {
    const int e = NA * (lane & 15) + x;
    aq[x] = e < S * S ? Ast[e] : 0.0;
  }
  // A'[r][0], block-uniform: kept in SGPRs
  double a0[S];
#pragma unroll
  for (int r = 0; r < S; ++r) {
    const long long v = __double_as_longlong(Ast[r * S]);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    a0[r] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  }
  __syncthreads();  // A' read before the tiles overwrite the lattice space

  for (int tile = wave * NB + t0; tile < ntile; tile += NB * NW) {
    const int i = p.i_begin + tile * PPW + (valid ? qw : 0);
    const bool active = valid && i < p.i_end;
    const int ic = active ? i : p.i_begin;
    if (valid && w == 0) F[q] = 0;
    // ---- per-pair inputs: CPL columns ----
    // V = Ef + L carried whole: the L sum of every step starts from Ef
    double Ef[CPL][S], V[CPL][S], arow[CPL][S], pb[CPL];
    bool bv[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int b = w + c * LPP;
      bv[c] = b < SB;
      const int bc = bv[c] ? b : SB - 1;
      const double *Ep = p.E + (size_t)j * S * p.e_ld + (size_t)(ic - p.i_buf0) * SB + bc;
      const double *Ai = p.A + ((size_t)ic * SB + bc) * SB;
      double rs = 0.0;
#pragma unroll
      for (int be = 0; be < S; ++be) {
        const double a = Ai[be < SB ? be : SB - 1];
        arow[c][be] = (bv[c] && be < SB) ? a : 0.0;
        rs += arow[c][be];
      }
      if (p.eU) {  // K1 here (short inner dimension): no E buffer
        double u[kK1InKernelMaxKdp];
        k1_column(p, (long long)ic * SB + bc, u);
        const int kdp = p.ekdp;
#pragma unroll
        for (int k = 0; k < S; ++k) {
          double e = k1w[kdp * S + k];  // bias', then W' u in e order
#pragma unroll
          for (int x = 0; x < kK1InKernelMaxKdp; ++x)
            if (x < kdp) e = fma(k1w[x * S + k], u[x], e);
          V[c][k] = e;
        }
        // the VHEM division behind a uniform branch (as a select it ran on every entry)
        if (__builtin_amdgcn_readfirstlane((int)(p.esmooth != 1.0))) {
#pragma unroll
          for (int k = 0; k < S; ++k) V[c][k] = V[c][k] / p.esmooth;
        }
#pragma unroll
        for (int k = 0; k < S; ++k) Ef[c][k] = V[c][k] + amax[k] * rs;
      } else {
#pragma unroll
        for (int k = 0; k < S; ++k) {
          const double e = Ep[(size_t)k * p.e_ld];
          Ef[c][k] = e + amax[k] * rs;
          V[c][k] = e;
        }
      }
      const double pr = p.prior[(size_t)ic * SB + bc];
      pb[c] = bv[c] ? pr : 0.0;
    }
    // column maxima of V, taken where V is produced (an fma result: no canonicalizing
    // max(x, x) per element as on a loop-carried value)
    double Mx[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) Mx[c] = tree_max<S>(V[c]);
    int zmin[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) zmin[c] = 0x7fffffff;

    // ---- K2: backward recursion, t = T-1 .. 1 ----
    for (int t = T - 1; t >= 1; --t) {
      double G[CPL][S], M[CPL];
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        double v[S];
        const double m = Mx[c];
        M[c] = m;
#pragma unroll
        for (int k = 0; k < S; ++k) v[k] = V[c][k] - m;
        exp_tabe_n<S>(G[c], v, etab);
      }
      double Z[CPL][S];
      // Z = A' G with A'[r][k] broadcast from lane (r S + k) / NA of the lane's DPP row:
      // no LDS (sums in k order, as fma chains); each chain starts with a plain
      // multiply by A'[r][0] held in SGPRs (no zeroing move per accumulator)
#pragma unroll
      for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int r = 0; r < S; ++r) Z[c][r] = a0[r] * G[c][0];
      // k outer, r inner: consecutive DPP fmacs write different accumulators (a DPP
      // instruction reading a VGPR the previous VALU instruction wrote needs two wait
      // states: r-inner chains cost an s_nop per fmac at S = 12); per-r order unchanged
      static_for<0, S * S>([&](auto ec) {
        constexpr int f = decltype(ec)::value, k = f / S, r = f % S, e = r * S + k;
        if constexpr (k > 0) {
#pragma unroll
          for (int c = 0; c < CPL; ++c) dpp_fmac_bcast<e / NA>(Z[c][r], aq[e % NA], G[c][k]);
        }
      });
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        double lz[S];
#pragma unroll
        for (int k = 0; k < S; ++k) zmin[c] = min(zmin[c], __double2hiint(Z[c][k]));
        log_tabe_n<S>(lz, Z[c], ltab);
        double sv[S];
#pragma unroll
        for (int k = 0; k < S; ++k) sv[k] = M[c] + lz[k];
        if (valid) {
          double *xc = X + (w + c * LPP) * LY::XCS;
          if constexpr (S % 2 == 0) {
#pragma unroll
            for (int k = 0; k < S; k += 2)
              *reinterpret_cast<double2 *>(xc + k) = make_double2(sv[k], sv[k + 1]);
          } else {
#pragma unroll
            for (int k = 0; k < S; ++k) xc[k] = sv[k];
          }
        }
      }
      wave_sync();
#pragma unroll
      for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int k = 0; k < S; ++k) V[c][k] = Ef[c][k];
#pragma unroll
      for (int be = 0; be < S; ++be) {
        const double *xc = X + be * LY::XCS;
        double xs[S];
        if constexpr (S % 2 == 0) {
#pragma unroll
          for (int k = 0; k < S; k += 2) {
            const double2 v = *reinterpret_cast<const double2 *>(__builtin_assume_aligned(xc + k, 16));
            xs[k] = v.x;
            xs[k + 1] = v.y;
          }
        } else {
#pragma unroll
          for (int k = 0; k < S; ++k) xs[k] = xc[k];
        }
#pragma unroll
        for (int k = 0; k < S; ++k)
#pragma unroll
          for (int c = 0; c < CPL; ++c) V[c][k] = fma(arow[c][be], xs[k], V[c][k]);
      }
#pragma unroll
      for (int c = 0; c < CPL; ++c) Mx[c] = tree_max<S>(V[c]);
      wave_sync();
    }

    // ---- K3: termination, L_elbo(i, j) = sum_b prior_b * log sum_s exp(lpi + E + L) ----
    double Y[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      double v1[S], ev[S], m1 = -INFINITY;
#pragma unroll
      for (int k = 0; k < S; ++k) {
        v1[k] = lpi[k] + V[c][k];
        m1 = fmax(m1, v1[k]);
      }
#pragma unroll
      for (int k = 0; k < S; ++k) v1[k] -= m1;
      exp_tabe_n<S>(ev, v1, etab);
      double zs = 0.0;
#pragma unroll
      for (int k = 0; k < S; ++k) zs += ev[k];
      double lzs[1];
      const double zsa[1] = {zs};
      log_tabe_n<1>(lzs, zsa, ltab);
      Y[c] = pb[c] * (m1 + lzs[0]);
    }
    bool bad = false;
#pragma unroll
    for (int c = 0; c < CPL; ++c) bad |= bv[c] && (zmin[c] < kZMinHi || !isfinite(Y[c]));
    if (valid) {
#pragma unroll
      for (int c = 0; c < CPL; ++c) X[(w + c * LPP) * LY::XCS] = Y[c];
    }
    // fallback flags, as fb_split_kernel: underflow with finite inputs -> exact
    // kernel; non-finite cluster constants or emissions -> L_elbo NaN
    if (bad && active) {
      bool nf = false;
#pragma unroll
      for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int k = 0; k < S; ++k) nf |= !isfinite(Ef[c][k]);
      for (int x = 0; x < S; ++x) nf |= isnan(amax[x]) || isnan(lpi[x]);
      atomicOr(&F[q], kFlagBad | (nf ? kFlagNonFinite : 0));
    }
    wave_sync();
    if (active && w == 0) {
      const size_t pair = (size_t)ic * K + j;
      double ll = 0.0;
      for (int be = 0; be < SB; ++be) ll += X[be * LY::XCS];
      const int f = F[q];
      if (f == kFlagBad) {
        const int slot = atomicAdd(p.flag_count, 1);
        atomicAdd(p.flag_count + 1, 1);
        p.flag_list[slot] = (int)pair;
        p.LL[pair] = ll;
      } else {
        p.LL[pair] = (f & kFlagNonFinite) ? __builtin_nan("") : ll;
      }
    }
    wave_sync();
  }
}

// ---------------------------------------------------------------------------
// one block of 4 x (waves per SIMD) waves per CU: the 32 KB of tables once per CU
int bwd2_waves(int S) { return 4 * VBHEM_BWD2_WAVES(S); }

size_t bwd2_lds(int S, int nwb) {
  if (S < 1 || S > kBwd2MaxS) return 0;
  const int CPL = S <= 8 ? 2 : 1, LPP = (S + CPL - 1) / CPL, PPW = 64 / LPP;
  const int XCS = (S + 1) / 2 * 2 + VBHEM_BWD2_XPAD(S), XP = CPL * LPP * XCS + 2;
  // dynamic part only (the tables are static): amax, lpi, the in-kernel K1's W' and bias'
  const int off_x = (2 * S + (kK1InKernelMaxKdp + 1) * S + 1) / 2 * 2;
  const int ppb = nwb * PPW;
  return ((size_t)off_x + (size_t)ppb * XP + (ppb + 1) / 2 + 1) * sizeof(double);
}

int bwd2_ppb(int S, int nwb) {
  const int CPL = S <= 8 ? 2 : 1;
  return nwb * (64 / ((S + CPL - 1) / CPL));
}

template <int S>
static const void *bwd2_fn() {
  return reinterpret_cast<const void *>(&fb_bwd2_kernel<S>);
}

static const void *bwd2_fn_s(int S) {
  switch (S) {
    case 1: return bwd2_fn<1>();
    case 2: return bwd2_fn<2>();
    case 3: return bwd2_fn<3>();
    case 4: return bwd2_fn<4>();
    case 5: return bwd2_fn<5>();
    case 6: return bwd2_fn<6>();
    case 7: return bwd2_fn<7>();
    case 8: return bwd2_fn<8>();
    case 9: return bwd2_fn<9>();
    case 10: return bwd2_fn<10>();
    case 11: return bwd2_fn<11>();
    case 12: return bwd2_fn<12>();
    case 13: return bwd2_fn<13>();
    case 14: return bwd2_fn<14>();
    case 15: return bwd2_fn<15>();
    case 16: return bwd2_fn<16>();
    default: return nullptr;
  }
}

int bwd2_resident_blocks(int S, int nwb, size_t lds) {
  const void *fn = bwd2_fn_s(S);
  return fn ? resident_per_cu(fn, nwb * 64, lds) : 1;
}

hipError_t launch_bwd2(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st, hipEvent_t t0,
                       hipEvent_t t1) {
  const void *fn = bwd2_fn_s(a.S);
  if (!fn || a.SB > a.S || !a.Atg) return hipErrorInvalidValue;
  // prep: threads 64 + S (W' rows), 128 + S^2 (A') and 448 (flag head) must exist
  if (a.prep && (!a.eU || !a.ftag || !a.pm || !a.pP || !a.pc || !a.pz || !a.pshift ||
                 a.nwb * 64 < 512 || a.ekdp > kK1InKernelMaxKdp))
    return hipErrorInvalidValue;
  hipError_t e = set_dyn_lds(fn, lds);
  if (e != hipSuccess) return e;
  switch (a.S) {
#define VBHEM_B2(s)                                                                         \
  case s:                                                                                   \
    if (t0)                                                                                 \
      hipExtLaunchKernelGGL(fb_bwd2_kernel<s>, dim3(grid), dim3(a.nwb * 64), lds, st, t0, t1, 0, a); \
    else                                                                                    \
      hipLaunchKernelGGL(fb_bwd2_kernel<s>, dim3(grid), dim3(a.nwb * 64), lds, st, a);     \
    break;
    VBHEM_B2(1) VBHEM_B2(2) VBHEM_B2(3) VBHEM_B2(4) VBHEM_B2(5) VBHEM_B2(6) VBHEM_B2(7) VBHEM_B2(8)
    VBHEM_B2(9) VBHEM_B2(10) VBHEM_B2(11) VBHEM_B2(12) VBHEM_B2(13) VBHEM_B2(14) VBHEM_B2(15)
    VBHEM_B2(16)
#undef VBHEM_B2
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace vbhem

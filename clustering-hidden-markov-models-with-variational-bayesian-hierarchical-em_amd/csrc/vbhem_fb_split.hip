// vbhem_fb_split.hip -- the E-step recursion, one base-state column per LPC lanes.
//
// Mapping (gfx950, wave64).  A workgroup of NWB wavefronts owns PPB pairs
// (consecutive bases) x ONE cluster j.  Within a pair, base state b (padded to S
// columns) is owned by a group of LPC adjacent lanes; lane h of the group holds
// rows sigma in [h*SH, h*SH+SH) (SH = ceil(S/LPC)) of every S x Sb pair matrix
// column in registers:   E, L, G, nu, tnu   (SH each)  and  H (SH x S).
// * cluster-side contractions (Z = A' G, nu' = G .* (A'^T g)): each lane forms
//   partial sums over its rows for all S outputs, then a DPP reduce-scatter
//   across the LPC lanes (quad_perm swaps, no LDS);
// * max / sum over sigma: DPP all-reduce;
// * base-side contractions (L = Ab s, f = nu Ab): columns exchanged through a
//   per-pair LDS slab (ds_read_b128);
// * backward lattice G_t (t = 1..T-2): lane-private LDS; G_{T-1} = exp(E-max E)
//   recomputed in the forward sweep;
// * sum_xi: per-lane outer products H += g G^T (G all-gathered by DPP),
//   reduced over the pair's columns once at the end.
// LPC = 1 (S <= 4), 2 (S <= 8), 4 (S <= 16) keeps per-lane registers ~<= 256
// and per-wave LDS ~<= 20 KB so two or more waves share each SIMD.
//
// Padded base states (b >= SB) and padded rows (sigma >= S when LPC does not
// divide S) are exact no-ops: zero prior / Ab rows & columns; E = -inf rows
// give G = 0 (mex.c:964-971, 1054-1058, 1196-1206).
//
// Reference: src/vbhem/vbhem_hmm_bwd_fwd_mex.c  K1 :715-865, K2 :915-1015,
// K3 :1020-1080, K4 :1093-1298.  Factorised log-sum-exp: vbhem_kernels.hip, DESIGN.md.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vbhem_internal.h"
#include "vbhem_exact.h"
#include "vbhem_log_table.h"
#include "vbhem_math.h"

// waves per SIMD the backward-only mode is compiled for (register budget 512 / W):
// 4 where the 128-VGPR budget costs at most a few spills outside the step loop
// (S = 8: 138 -> 128 VGPRs, 10 spilled, -3 % kernel time at C4), else 3
#ifndef VBHEM_BWD_WAVES
#define VBHEM_BWD_WAVES(S) (((S) <= 4 || ((S) >= 7 && (S) <= 10)) ? 4 : 3)
#endif

namespace vbhem {

namespace {

constexpr double kZMinS = 1e-200;

// log_tab_n's table (backward mode stages it in LDS once per persistent block)
alignas(16) __device__ const double kLogTab[kLogTabDoubles] = VBHEM_LOG_TABLE_INIT;
alignas(16) __device__ const double kExpTab[kExpTabDoubles] = VBHEM_EXP_TABLE_INIT;

// ---- DPP lane exchange inside aligned lane quads -------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  // bound_ctrl: no 'old' operand to initialise (quad_perm never reads out of bounds)
  const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, true);
  const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi2, lo2);
}
constexpr int kXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kXor2 = 0x4E;  // quad_perm [2,3,0,1]

template <int M>
__device__ __forceinline__ double xchg(double v) {
  if constexpr (M == 1) return dpp_d<kXor1>(v);
  else return dpp_d<kXor2>(v);
}

template <int LPC>
__device__ __forceinline__ double allmax(double v) {
  if constexpr (LPC >= 2) v = fmax(v, xchg<1>(v));
  if constexpr (LPC >= 4) v = fmax(v, xchg<2>(v));
  return v;
}
template <int LPC>
__device__ __forceinline__ double allsum(double v) {
  if constexpr (LPC >= 2) v += xchg<1>(v);
  if constexpr (LPC >= 4) v += xchg<2>(v);
  return v;
}

// Owner-relative ordering: a lane keeps per-owner blocks of SH values indexed by
// o' = o ^ h (o the owning lane's h), so its own block is always first and the
// butterfly exchanges below need no selects.  Absolute row of relative index x:
//   rel_row<SH>(x, h) = ((x / SH) ^ h) * SH + x % SH.
template <int SH>
__device__ __forceinline__ int rel_row(int x, int h) {
  return ((x / SH) ^ h) * SH + x % SH;
}

// Reduce-scatter: in[LPC*SH] = this lane's partial sums for every owner block
// (owner-relative order); out[SH] = the group's sums for this lane's rows.
template <int LPC, int SH>
__device__ __forceinline__ void reduce_scatter(const double (&in)[LPC * SH], double (&out)[SH]) {
  if constexpr (LPC == 1) {
#pragma unroll
    for (int k = 0; k < SH; ++k) out[k] = in[k];
  } else if constexpr (LPC == 2) {
#pragma unroll
    for (int k = 0; k < SH; ++k) out[k] = in[k] + xchg<1>(in[SH + k]);
  } else {
    double t[2 * SH];  // relative owners 0, 1 (o = h, h ^ 1) summed over lanes h, h ^ 2
#pragma unroll
    for (int q = 0; q < 2 * SH; ++q) t[q] = in[q] + xchg<2>(in[2 * SH + q]);
#pragma unroll
    for (int k = 0; k < SH; ++k) out[k] = t[k] + xchg<1>(t[SH + k]);
  }
}

// All-gather: in[SH] (this lane's rows) -> out[LPC*SH] (all rows, owner-relative).
template <int LPC, int SH>
__device__ __forceinline__ void all_gather(const double (&in)[SH], double (&out)[LPC * SH]) {
#pragma unroll
  for (int k = 0; k < SH; ++k) out[k] = in[k];
  if constexpr (LPC >= 2) {
#pragma unroll
    for (int k = 0; k < SH; ++k) out[SH + k] = xchg<1>(in[k]);
  }
  if constexpr (LPC == 4) {
#pragma unroll
    for (int q = 0; q < 2 * SH; ++q) out[2 * SH + q] = xchg<2>(out[q]);
  }
}

// Barrier for the per-pair LDS exchange.  When a pair's lanes never straddle a
// wavefront (lanes per pair a power of two) the exchange is wave-local: LDS
// requests of one wave are processed in issue order, so a code-motion barrier
// with wavefront-scope fences suffices and the waves of a block run decoupled.
template <bool WAVE>
__device__ __forceinline__ void pair_sync() {
  if constexpr (WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

template <int n>
__device__ __forceinline__ void lds_ld(double (&dst)[n], const double *src) {
  if constexpr (n % 2 == 0) {
    const double2 *s2 = reinterpret_cast<const double2 *>(__builtin_assume_aligned(src, 16));
#pragma unroll
    for (int k = 0; k < n / 2; ++k) {
      const double2 v = s2[k];
      dst[2 * k] = v.x;
      dst[2 * k + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int k = 0; k < n; ++k) dst[k] = src[k];
  }
}

template <int n>
__device__ __forceinline__ void lds_st(double *dst, const double (&src)[n]) {
  if constexpr (n % 2 == 0) {
    double2 *d2 = reinterpret_cast<double2 *>(__builtin_assume_aligned(dst, 16));
#pragma unroll
    for (int k = 0; k < n / 2; ++k) d2[k] = make_double2(src[2 * k], src[2 * k + 1]);
  } else {
#pragma unroll
    for (int k = 0; k < n; ++k) dst[k] = src[k];
  }
}

// row[r0 .. r0+SH) of an S-wide LDS row (clamped to S-1 beyond the end)
template <int S, int SH, int LPC>
__device__ __forceinline__ void load_row(double (&dst)[SH], const double *row, int r0) {
  if constexpr (S % LPC == 0 && SH % 2 == 0 && S % 2 == 0) {
    lds_ld<SH>(dst, row + r0);
  } else {
#pragma unroll
    for (int k = 0; k < SH; ++k) {
      const int s = r0 + k < S ? r0 + k : S - 1;
      dst[k] = row[s];
    }
  }
}

}  // namespace

// One workgroup = NWB wavefronts = PPB pairs of ONE cluster.  Dense / backward
// modes: block (tile, j) = bases [i_begin + tile*PPB, +PPB) x cluster blockIdx % K.
// List mode: the gated pairs of every cluster cut into PPB-pair work items,
// contiguous item ranges per block (cluster constants restaged when j changes).
template <int S, int LPC, int MODE>
__global__ __launch_bounds__(MODE == kFbList ? 512 : 256) __attribute__((amdgpu_waves_per_eu(MODE == kFbBackward ? VBHEM_BWD_WAVES(S) : 2)))
void fb_split_kernel(const SplitArgs p) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  using LY = SplitLayout<S, LPC>;
  constexpr int SH = LY::SH;
  constexpr int LPP = S * LPC;  // lanes per pair
  constexpr bool kWaveLocal = (LPP & (LPP - 1)) == 0;  // pairs never straddle a wave
  constexpr bool kFwd = MODE != kFbBackward;
  constexpr bool kTab = MODE != kFbDense;  // tables in LDS (list mode: the compact pair)
  constexpr bool kTabC = MODE == kFbList;   // exp_tabc_n / log_tabc_n on 4 KB of tables
  const int tid = threadIdx.x;
  const int NT = p.nwb * 64;
  const int PPB = NT / LPP;
  const int SB = p.SB, T = p.T, K = p.K;

  double *At = lds;              // [S][S]
  double *AtT = At + S * S;      // [S][S]
  double *amax = AtT + S * S;    // [S]
  double *lpi = amax + S;        // [S]
  double *R = lds + p.off_R;     // lattice [(T-2)][SH][NT]
  int *F = reinterpret_cast<int *>(lds + p.off_F);  // [PPB] fallback flags
  // backward mode: the padded tables staged in LDS; list mode: the compact ones
  // (exp 2^(j/256) [256] | log {1/c, log c} [128][2]: 4 KB next to the lattice, one
  // 8-wave block per CU); dense mode (LDS taken by the lattice) reads them from
  // global memory (8 KB, L1/L2-resident)
  const double *ltab = kTabC ? lds + p.off_T + kExpTabEntries : kTab ? lds + p.off_T : kLogTab;
  const double *etab = kTabC ? lds + p.off_T : kTab ? lds + p.off_T + kLogTabDoubles : kExpTab;

  // ---------------- cluster constants: A' = exp(logA - rowmax), rowmax, logPi --------------
  auto stage_cluster = [&](int j) {
    const double *la = p.logA + (size_t)j * S * S;
    if (tid < S) {
      double mx = la[tid * S];
      for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[tid * S + s2]);
      amax[tid] = mx;
      lpi[tid] = p.logPi[(size_t)j * S + tid];
    }
    __syncthreads();
    for (int x = tid; x < S * S; x += NT) {
      const int r = x / S, s2 = x - r * S;
      const double a = exp_nonpos(la[x] - amax[r]);
      At[x] = a;
      AtT[s2 * S + r] = a;
    }
    __syncthreads();
  };

  // ---------------- one pair per LPP lanes: (ic, j) --------------------------------------------
  // pair n0 + q of the item: base i = lst ? lst[n0 + q] : n0 + q, active while n0 + q < lim
  // (ipre >= 0: the base index, already loaded by the caller)
  auto run_pair = [&](int j, int n0, int lim, const int *lst, int ipre) {
    // lane geometry recomputed from an opaque copy of the thread id: in the list
    // mode's item loop this keeps LICM from hoisting every lane-invariant address
    // out of the loop (which costs ~90 VGPRs of live ranges)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    // the arguments re-read through a laundered kernarg-segment pointer, for the same
    // reason (SGPR live ranges); p is the kernel's only argument, at offset 0
    const SplitArgs *pap = (const SplitArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(pap));
    const SplitArgs &pa = *pap;
    const int q = tid / LPP;
    const int w = tid - q * LPP;
    const int b = w / LPC;
    const int h = w - b * LPC;
    const bool valid = q < PPB;
    const bool bvalid = b < SB;
    const int bc = bvalid ? b : SB - 1;
    __builtin_assume(h >= 0 && h < LPC);
    const int r0 = h * SH;  // first row owned by this lane
    double *X = lds + LY::OFF_X + (valid ? q : 0) * LY::XP;   // slab [col][XCS]
    double *Y = lds + pa.off_Y + (valid ? q : 0) * S;
    const bool active = valid && n0 + q < lim;
    const int i = active ? (ipre >= 0 ? ipre : lst ? lst[n0 + q] : n0 + q) : pa.i_begin;
    const int ic = i;
    const size_t lp = (size_t)(ic - pa.i_buf0) * K + j;
    if (valid && w == 0) F[q] = 0;  // read back only after this pair's later syncs
    // per-pair inputs: E (K1, precomputed), Ab row/column, prior
    double E[SH];
    if (pa.eU) {  // K1 here (short inner dimension): no E buffer
      double u[kK1InKernelMaxKdp];
      k1_column(pa, (long long)ic * SB + bc, u);
#pragma unroll
      for (int k = 0; k < SH; ++k) {
        const bool rv = r0 + k < S;
        const double v = k1_entry(pa, j * S + (rv ? r0 + k : S - 1), u);
        E[k] = rv ? v : -INFINITY;
      }
      if (__builtin_amdgcn_readfirstlane((int)(pa.esmooth != 1.0))) {  // VHEM (uniform)
#pragma unroll
        for (int k = 0; k < SH; ++k) E[k] = E[k] / pa.esmooth;
      }
    } else {
      const double *Ep = pa.E + (size_t)j * S * pa.e_ld + (size_t)(ic - pa.i_buf0) * SB + bc;
#pragma unroll
      for (int k = 0; k < SH; ++k) {
        const bool rv = r0 + k < S;
        const double v = Ep[(size_t)(rv ? r0 + k : S - 1) * pa.e_ld];
        E[k] = rv ? v : -INFINITY;
      }
    }
    double arow[S], acol[kFwd ? S : 1];
    {
      const double *Ai = pa.A + (size_t)ic * SB * SB;
#pragma unroll
      for (int be = 0; be < S; ++be) {
        const int bb = be < SB ? be : SB - 1;
        const bool ok = bvalid && be < SB;
        const double r1 = Ai[bc * SB + bb];
        arow[be] = ok ? r1 : 0.0;
        if constexpr (kFwd) {
          const double c1 = Ai[bb * SB + bc];
          acol[be] = ok ? c1 : 0.0;
        }
      }
    }
    const double pb0 = pa.prior[(size_t)ic * SB + bc];
    const double pb = bvalid ? pb0 : 0.0;

    // ---------------- K2: backward recursion -----------------------------------------------
    // A'(rows of every owner block, my columns r0..r0+SH): register-resident for both sweeps
    // (occupancy is bounded by LDS, not registers)
#ifndef VBHEM_SPLIT_LIST_ATREG_MAXS
#define VBHEM_SPLIT_LIST_ATREG_MAXS 16
#endif
    constexpr bool kAtReg = LPC * SH * SH <= 48 &&  // <= 96 VGPRs
                            (MODE != kFbList || S <= VBHEM_SPLIT_LIST_ATREG_MAXS);
    // LPC = 1 (one lane per column, rows uniform across the wave): A' is read as
    // scalar operands from global memory (s_load, scalar cache) instead of LDS
    constexpr bool kAtScalar = MODE == kFbBackward && LPC == 1 && !kAtReg;
    double atr[kAtReg ? LPC * SH : 1][SH];
    if constexpr (kAtReg) {
#pragma unroll
      for (int r = 0; r < LPC * SH; ++r) {
        const int ra = rel_row<SH>(r, h);
        load_row<S, SH, LPC>(atr[r], At + (ra < S ? ra : S - 1) * S, r0);
      }
    }
    double am[SH];  // amax of my rows (LDS -> registers once)
#pragma unroll
    for (int k = 0; k < SH; ++k) am[k] = amax[r0 + k < S ? r0 + k : S - 1];
    double L[SH];
#pragma unroll
    for (int k = 0; k < SH; ++k) L[k] = 0.0;
    bool bad = false;
    for (int t = T - 1; t >= 1; --t) {
      double G[SH], M = -INFINITY;
#pragma unroll
      for (int k = 0; k < SH; ++k) M = fmax(M, E[k] + L[k]);
      M = allmax<LPC>(M);
      {
        double ex[SH];
#pragma unroll
        for (int k = 0; k < SH; ++k) ex[k] = (E[k] + L[k]) - M;
        if constexpr (kTabC) exp_tabc_n<SH>(G, ex, etab);
        else exp_tabf_n<SH>(G, ex, etab);
      }
      // partial Z for every owner's rows, then reduce-scatter
      double Pz[LPC * SH];
      typedef const double __attribute__((address_space(4))) cdouble;
      // (the kernel argument itself, not the laundered pointer: an asm output counts
      // as divergent, which would turn these into vector loads)
      const double *Agp = p.Atg + __builtin_amdgcn_readfirstlane(j * S * S);
#pragma unroll
      for (int r = 0; r < LPC * SH; ++r) {
        double ar[SH];
        if constexpr (kAtReg) {
#pragma unroll
          for (int k = 0; k < SH; ++k) ar[k] = atr[r][k];
        } else if constexpr (kAtScalar) {
          const cdouble *Ac = (const cdouble *)Agp;
#pragma unroll
          for (int k = 0; k < SH; ++k) ar[k] = Ac[r * S + k];
        } else {
          const int ra = rel_row<SH>(r, h);
          load_row<S, SH, LPC>(ar, At + (ra < S ? ra : S - 1) * S, r0);
        }
        double z = 0.0;
#pragma unroll
        for (int k = 0; k < SH; ++k) z = fma(ar[k], G[k], z);
        Pz[r] = z;
      }
      double Z[SH];
      reduce_scatter<LPC, SH>(Pz, Z);
      double sv[SH], zz[SH], lz[SH];
#pragma unroll
      for (int k = 0; k < SH; ++k) {
        const bool rv = r0 + k < S;
        bad |= bvalid && rv && !(Z[k] >= kZMinS);
        zz[k] = rv ? Z[k] : 1.0;
      }
      if constexpr (kTabC) log_tabc_n<SH>(lz, zz, ltab);
      else log_tabf_n<SH>(lz, zz, ltab);
#pragma unroll
      for (int k = 0; k < SH; ++k) sv[k] = M + am[k] + lz[k];
      if (kFwd && t <= T - 2) {
        double *slot = R + (size_t)(t - 1) * SH * NT + tid;
#pragma unroll
        for (int k = 0; k < SH; ++k) slot[k * NT] = G[k];
      }
      if (valid) lds_st<SH>(X + b * LY::XCS + r0, sv);
      pair_sync<kWaveLocal>();
#pragma unroll
      for (int k = 0; k < SH; ++k) L[k] = 0.0;
#pragma unroll
      for (int be = 0; be < S; ++be) {
        double xs[SH];
        lds_ld<SH>(xs, X + be * LY::XCS + r0);
#pragma unroll
        for (int k = 0; k < SH; ++k) L[k] = fma(arow[be], xs[k], L[k]);
      }
      pair_sync<kWaveLocal>();
    }

    // ---------------- K3: termination --------------------------------------------------------
    double nu[SH];
    {
      double v1[SH], M1 = -INFINITY;
#pragma unroll
      for (int k = 0; k < SH; ++k) {
        const int r = r0 + k < S ? r0 + k : S - 1;
        v1[k] = lpi[r] + E[k] + L[k];
        M1 = fmax(M1, v1[k]);
      }
      M1 = allmax<LPC>(M1);
      double ex[SH], ev[SH];
#pragma unroll
      for (int k = 0; k < SH; ++k) ex[k] = v1[k] - M1;
      exp_nonpos_n<SH>(ev, ex);
      double zs = 0.0;
#pragma unroll
      for (int k = 0; k < SH; ++k) zs += ev[k];
      zs = allsum<LPC>(zs);
      const double s1 = M1 + log_pos(zs);
      if constexpr (kFwd) {
#pragma unroll
        for (int k = 0; k < SH; ++k) ex[k] = v1[k] - s1;
        exp_nonpos_n<SH>(ev, ex);
#pragma unroll
        for (int k = 0; k < SH; ++k) nu[k] = pb * ev[k];
      }
      if (valid) {
        if (MODE != kFbList && h == 0) Y[b] = pb * s1;
        if constexpr (kFwd) lds_st<SH>(X + b * LY::XCS + r0, nu);
      }
    }
    pair_sync<kWaveLocal>();
    const size_t pair = (size_t)ic * K + j;
    if (active) {
      if (MODE != kFbList && w == 0) {
        double ll = 0.0;
        for (int be = 0; be < SB; ++be) ll += Y[be];
        pa.LL[pair] = ll;
      }
      if (kFwd && w < S) {
        double n1 = 0.0;
#pragma unroll
        for (int be = 0; be < S; ++be) n1 += X[be * LY::XCS + w];
        pa.nu1[lp * S + w] = n1;
      }
    }

    if constexpr (kFwd) {
      // ---------------- K4: forward recursion ------------------------------------------------
      double tn[SH], H[SH][LPC * SH];
#pragma unroll
      for (int k = 0; k < SH; ++k) {
        tn[k] = nu[k];
#pragma unroll
        for (int s = 0; s < LPC * SH; ++s) H[k][s] = 0.0;
      }
      for (int t = 1; t < T; ++t) {
        double G[SH];
        if (t == T - 1) {
          double M = -INFINITY;
#pragma unroll
          for (int k = 0; k < SH; ++k) M = fmax(M, E[k]);
          M = allmax<LPC>(M);
          double ex[SH];
#pragma unroll
          for (int k = 0; k < SH; ++k) ex[k] = E[k] - M;
          // the backward sweep's G_{T-1}, bit for bit
          if constexpr (kTabC) exp_tabc_n<SH>(G, ex, etab);
          else exp_tabf_n<SH>(G, ex, etab);
        } else {
          const double *slot = R + (size_t)(t - 1) * SH * NT + tid;
#pragma unroll
          for (int k = 0; k < SH; ++k) G[k] = slot[k * NT];
        }
        pair_sync<kWaveLocal>();  // X holds nu
        double f[SH];
#pragma unroll
        for (int k = 0; k < SH; ++k) f[k] = 0.0;
#pragma unroll
        for (int be = 0; be < S; ++be) {
          double xs[SH];
          lds_ld<SH>(xs, X + be * LY::XCS + r0);
#pragma unroll
          for (int k = 0; k < SH; ++k) f[k] = fma(xs[k], acol[be], f[k]);
        }
        // Z recomputed exactly as in the backward pass
        double Pz[LPC * SH];
#pragma unroll
        for (int r = 0; r < LPC * SH; ++r) {
          double ar[SH];
          if constexpr (kAtReg) {
#pragma unroll
            for (int k = 0; k < SH; ++k) ar[k] = atr[r][k];
          } else {
            const int ra = rel_row<SH>(r, h);
            load_row<S, SH, LPC>(ar, At + (ra < S ? ra : S - 1) * S, r0);
          }
          double z = 0.0;
#pragma unroll
          for (int k = 0; k < SH; ++k) z = fma(ar[k], G[k], z);
          Pz[r] = z;
        }
        double Z[SH], g[SH];
        reduce_scatter<LPC, SH>(Pz, Z);
        {
          double zr[SH], rz[SH];
#pragma unroll
          for (int k = 0; k < SH; ++k) zr[k] = (r0 + k < S) ? Z[k] : 1.0;
          rcp_pos_n<SH>(rz, zr);
#pragma unroll
          for (int k = 0; k < SH; ++k) g[k] = (r0 + k < S) ? f[k] * rz[k] : 0.0;
        }
        // nu'(s) = G(s) * sum_r A'(r, s) g(r): partial over my rows r for every s
        double Pn[LPC * SH];
#pragma unroll
        for (int s = 0; s < LPC * SH; ++s) {
          const int sa = rel_row<SH>(s, h);
          const int ss = sa < S ? sa : S - 1;
          double ac[SH];
          load_row<S, SH, LPC>(ac, AtT + ss * S, r0);
          double a = 0.0;
#pragma unroll
          for (int k = 0; k < SH; ++k) a = fma(ac[k], g[k], a);
          Pn[s] = a;
        }
        double Q[SH];
        reduce_scatter<LPC, SH>(Pn, Q);
#pragma unroll
        for (int k = 0; k < SH; ++k) {
          nu[k] = G[k] * Q[k];
          tn[k] += nu[k];
        }
        double Ga[LPC * SH];
        all_gather<LPC, SH>(G, Ga);
#pragma unroll
        for (int k = 0; k < SH; ++k)
#pragma unroll
          for (int s = 0; s < LPC * SH; ++s) H[k][s] = fma(g[k], Ga[s], H[k][s]);
        pair_sync<kWaveLocal>();  // all reads of X done
        if (valid) lds_st<SH>(X + b * LY::XCS + r0, nu);
      }

      // ---------------- outputs ---------------------------------------------------------------
      if (active && bvalid) {
#pragma unroll
        for (int k = 0; k < SH; ++k)
          if (r0 + k < S) pa.tnu[(lp * S + r0 + k) * SB + b] = tn[k];
      }
      // sum_xi(r, s) = A'(r, s) * sum_b H_b(r, s).
      //  S > 8 : every lane parks its H block in the (now dead) lattice region, one
      //          barrier, then each lane of the pair reduces S*S/LPP outputs;
      //  S <= 8: one wave-local round per row r through the pair's slab.
      if constexpr (S > 8) {
        constexpr int HW = LPC * SH;                      // values per H row (owner-relative)
        __syncthreads();                                  // all lattice reads of the block done
        double *Hq = R + (size_t)(valid ? q : 0) * S * S * HW;   // [b][r][HW]
        if (valid && b < S) {
#pragma unroll
          for (int k = 0; k < SH; ++k)
            if (r0 + k < S) lds_st<HW>(Hq + ((size_t)b * S + r0 + k) * HW, H[k]);
        }
        __syncthreads();
        if (active) {
          for (int o = w; o < S * S; o += LPP) {
            const int r = o / S, s2 = o - r * S;
            const int sr = rel_row<SH>(s2, r / SH);       // s2 in row r's owner-relative order
            double acc = 0.0;
#pragma unroll
            for (int be = 0; be < S; ++be) acc += Hq[((size_t)be * S + r) * HW + sr];
            pa.xi[lp * S * S + o] = At[o] * acc;
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < S; ++r) {
          pair_sync<kWaveLocal>();
          if (valid && h == r / SH) lds_st<LPC * SH>(X + b * LY::XCS, H[r % SH]);  // owner-relative
          pair_sync<kWaveLocal>();
          if (active && w < S) {
            const int wr = rel_row<SH>(w, r / SH);  // w's position in row r's owner-relative order
            double acc = 0.0;
#pragma unroll
            for (int be = 0; be < S; ++be) acc += X[be * LY::XCS + wr];
            pa.xi[(lp * S + r) * S + w] = At[r * S + w] * acc;
          }
        }
      }
    }
    // fallback flags (one per pair).  !(Z >= kZMinS) also catches NaN; a pair whose
    // inputs are not finite (a diverged cluster) is not sent to the exact fallback,
    // its L_elbo is NaN (the table-driven log need not propagate NaN by itself)
    if (bad && active) {
      bool nf = false;
#pragma unroll
      for (int k = 0; k < SH; ++k) nf |= (r0 + k < S) && !isfinite(E[k]);
      for (int x = 0; x < S; ++x) nf |= isnan(amax[x]) || isnan(lpi[x]);
      atomicOr(&F[q], kFlagBad | (nf ? kFlagNonFinite : 0));
    }
    pair_sync<kWaveLocal>();
    // inline only for 4 <= S <= 6 (kSplitInline*): past 6 the exact recursion's
    // registers would push the list kernel into scratch, below 4 they would cost it
    // occupancy (S = 3: 139 -> 197 VGPRs); at 4..6 the kernel stays at 2 waves per SIMD
    constexpr bool kXin = MODE == kFbList && S >= kSplitInlineMinS && S <= kSplitInlineMaxS;
    const bool xin = kXin && pa.xinline;
    if (active && w == 0) {
      const int f = F[q];
      if (f == kFlagBad) {
        atomicAdd(pa.flag_count + 1, 1);
        if (!xin) {
          const int slot = atomicAdd(pa.flag_count, 1);
          pa.flag_list[slot] = (int)pair;
        }
      } else if ((f & kFlagNonFinite) && MODE != kFbList) {
        pa.LL[pair] = __builtin_nan("");
      }
    }
    if constexpr (kXin) {
      if (xin) {  // wave-uniform: this wave's flagged pairs, recomputed by the whole wave
        unsigned long long fm = __ballot(active && w == 0 && F[q] == kFlagBad);
        while (fm) {
          const int l = __builtin_ctzll(fm);
          fm &= fm - 1;
          const int pl = __builtin_amdgcn_readlane((int)pair, l);
          exact_pair_wave<true>(pa.xf, pl,
                                pa.xscr + ((size_t)blockIdx.x * (NT >> 6) + (tid >> 6)) * pa.xstride,
                                nullptr);
        }
      }
    }
  };

  if constexpr (MODE == kFbDense) {
    const int j = blockIdx.x % K;
    stage_cluster(j);
    run_pair(j, p.i_begin + (int)(blockIdx.x / K) * PPB, p.i_end, nullptr, -1);
  } else if constexpr (MODE == kFbBackward) {
    // persistent: NB blocks per cluster, each keeps its cluster and strides over the
    // tiles.  XCD-aware when NB % 8 == 0: workgroups are dealt round-robin to the 8
    // XCDs (b % 8), so the K blocks that walk the same tiles (same base transitions,
    // read by all K clusters) are put on one XCD and share its L2.
    for (int x = tid; x < kLogTabDoubles; x += NT) lds[p.off_T + x] = kLogTab[x];
    for (int x = tid; x < kExpTabDoubles; x += NT) lds[p.off_T + kLogTabDoubles + x] = kExpTab[x];
    const int b = blockIdx.x, NB = (int)gridDim.x / K;
    int j, t0;
    if (NB % 8 == 0) {
      const int r = b / 8;
      j = r % K;
      t0 = (r / K) * 8 + b % 8;
    } else {
      j = b % K;
      t0 = b / K;
    }
    stage_cluster(j);  // (its barriers also publish the table)
    const int ntile = (p.i_end - p.i_begin + PPB - 1) / PPB;
    for (int tile = t0; tile < ntile; tile += NB)
      run_pair(j, p.i_begin + tile * PPB, p.i_end, nullptr, -1);
  } else {
    // work items: cluster j owns ceil(list_tot[j] / PPB) consecutive items
    for (int x = tid; x < kExpTabEntries; x += NT) lds[p.off_T + x] = kExpTab[2 * x];
    for (int x = tid; x < kLogTabEntries; x += NT) {
      lds[p.off_T + kExpTabEntries + 2 * x] = kLogTab[4 * x];
      lds[p.off_T + kExpTabEntries + 2 * x + 1] = kLogTab[4 * x + 1];
    }
    int *pre = reinterpret_cast<int *>(lds + p.off_L);  // [K + 1]
    if (tid == 0) {
      int s = 0;
      for (int jj = 0; jj < K; ++jj) {
        pre[jj] = s;
        s += (p.list_tot[jj] + PPB - 1) / PPB;
      }
      pre[K] = s;
    }
    __syncthreads();
    const int nitem = __builtin_amdgcn_readfirstlane(pre[K]);  // block-uniform: keep in SGPRs
    const int per = (nitem + (int)gridDim.x - 1) / (int)gridDim.x;
    const int w0 = (int)blockIdx.x * per, w1 = min(nitem, w0 + per);
    // the item's cluster (block-uniform) and this lane's base, -1 past the list's end
    const int q = tid / LPP;
    auto item = [&](int wi, int jfrom, int &jj) -> int {
      jj = jfrom;
      while (pre[jj + 1] <= wi) ++jj;
      jj = __builtin_amdgcn_readfirstlane(jj);
      const int n = (wi - pre[jj]) * PPB + q;
      return (q < PPB && n < p.list_tot[jj]) ? p.list[(size_t)jj * p.list_cap + n] : -1;
    };
    int jn = 0;
    int inext = w0 < w1 ? item(w0, 0, jn) : -1;
    int jcur = -1;
    for (int wi = w0; wi < w1; ++wi) {
      const int jj = jn;
      const int icur = inext;
      if (wi + 1 < w1) inext = item(wi + 1, jj, jn);  // next item's base: in flight now
      // a block barrier only where LDS is shared across waves: the cluster constants
      // (restaged when the cluster changes) and, for S > 8, the parked H blocks; slabs,
      // flags and lattice are wave-private (pairs never straddle a wave), so the waves
      // otherwise drift apart and one wave's load stall at an item start hides behind
      // the other's compute
      if (!(kWaveLocal && S <= 8) || jj != jcur) __syncthreads();
      if (jj != jcur) {
        stage_cluster(jj);
        jcur = jj;
      }
      const int tot = __builtin_amdgcn_readfirstlane(p.list_tot[jj]);
      run_pair(jj, (wi - pre[jj]) * PPB, tot, nullptr, icur);
    }
  }
}

// ---------------------------------------------------------------------------
template <int S, int LPC, int MODE>
static hipError_t launch_split_slm(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st) {
  auto *fn = &fb_split_kernel<S, LPC, MODE>;
  hipError_t e = set_dyn_lds(reinterpret_cast<const void *>(fn), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((fb_split_kernel<S, LPC, MODE>), dim3(grid), dim3(a.nwb * 64), lds, st, a);
  return hipGetLastError();
}

template <int S, int LPC>
static hipError_t launch_split_sl(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st) {
  switch (a.mode) {
    case kFbDense: return launch_split_slm<S, LPC, kFbDense>(a, grid, lds, st);
    case kFbList: return launch_split_slm<S, LPC, kFbList>(a, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

template <int S, int LPC, int MODE>
static int resident_slm(const SplitArgs &a, size_t lds) {
  return resident_per_cu(reinterpret_cast<const void *>(&fb_split_kernel<S, LPC, MODE>),
                         a.nwb * 64, lds);
}

template <int S>
static int resident_s(const SplitArgs &a, size_t lds) {
  constexpr int LPC = SplitLPC<S>::value, LB = BwdLPC<S>::value;
  switch (a.mode) {
    case kFbDense: return resident_slm<S, LPC, kFbDense>(a, lds);
    case kFbBackward: return resident_slm<S, LB, kFbBackward>(a, lds);
    default: return resident_slm<S, LPC, kFbList>(a, lds);
  }
}

int split_resident_blocks(const SplitArgs &a, size_t lds) {
  switch (a.S) {
#define VBHEM_RS(s) case s: return resident_s<s>(a, lds);
    VBHEM_RS(1) VBHEM_RS(2) VBHEM_RS(3) VBHEM_RS(4) VBHEM_RS(5) VBHEM_RS(6) VBHEM_RS(7)
    VBHEM_RS(8) VBHEM_RS(9) VBHEM_RS(10) VBHEM_RS(11) VBHEM_RS(12) VBHEM_RS(13) VBHEM_RS(14)
    VBHEM_RS(15) VBHEM_RS(16)
#undef VBHEM_RS
    default: return 1;
  }
}

template <int S>
static hipError_t launch_split_s(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st) {
  constexpr int LB = BwdLPC<S>::value;
  if (a.mode == kFbBackward) {
    if (a.lpc != LB) return hipErrorInvalidValue;
    return launch_split_slm<S, LB, kFbBackward>(a, grid, lds, st);
  }
  if (a.lpc != SplitLPC<S>::value) return hipErrorInvalidValue;
  return launch_split_sl<S, SplitLPC<S>::value>(a, grid, lds, st);
}

hipError_t launch_split(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st) {
  switch (a.S) {
    case 1: return launch_split_s<1>(a, grid, lds, st);
    case 2: return launch_split_s<2>(a, grid, lds, st);
    case 3: return launch_split_s<3>(a, grid, lds, st);
    case 4: return launch_split_s<4>(a, grid, lds, st);
    case 5: return launch_split_s<5>(a, grid, lds, st);
    case 6: return launch_split_s<6>(a, grid, lds, st);
    case 7: return launch_split_s<7>(a, grid, lds, st);
    case 8: return launch_split_s<8>(a, grid, lds, st);
    case 9: return launch_split_s<9>(a, grid, lds, st);
    case 10: return launch_split_s<10>(a, grid, lds, st);
    case 11: return launch_split_s<11>(a, grid, lds, st);
    case 12: return launch_split_s<12>(a, grid, lds, st);
    case 13: return launch_split_s<13>(a, grid, lds, st);
    case 14: return launch_split_s<14>(a, grid, lds, st);
    case 15: return launch_split_s<15>(a, grid, lds, st);
    case 16: return launch_split_s<16>(a, grid, lds, st);
    default: return hipErrorInvalidValue;
  }
}

bool split_supported(int S, int SB, int d) {
  return S >= 1 && S <= kSplitMaxS && SB >= 1 && SB <= S && d >= 1 && d <= 64;
}

int split_lpc(int S) {
#ifdef VBHEM_SPLIT_LPC5
  if (S == 5) return VBHEM_SPLIT_LPC5;
#endif
  return S <= 4 ? 1 : S <= 8 ? 2 : 4;
}
int split_lpc_bwd(int S) { return S <= 8 ? 1 : 2; }

}  // namespace vbhem

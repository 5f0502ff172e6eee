// vbhem_fb_bwd4.hip -- the gated schedule's backward-only pass (K2 backward
// recursion, mex.c:915-1015, and K3 termination, mex.c:1020-1080, writing L_elbo)
// for S = 8 cluster states and SB <= 8 base states, with both per-step contractions
// on the fp64 matrix cores (v_mfma_f64_4x4x4f64, 4 blocks of 4x4x4 per instruction).
//
// Per pair and step (the factorised recursion of fb_bwd2_kernel):
//   G  = exp(V - M)            M[b] = column maximum over the cluster states
//   Z  = A' G                  A' = exp(logA - amax), the cluster's transitions
//   sv = M + log Z
//   V  = Ef + sv Ab^T          Ab = the base's transitions, Ef = E + amax rowsum(Ab)
// A wavefront holds one quad of 4 pairs (4 consecutive bases of one cluster); the
// 4 pairs of a quad are the 4 blocks of every MFMA, so no operand is padded.  With
//   P layout:  X[i][j] of block (I, J) in lane 16 (i - 4I) + 4 pair + (j - 4J)
//   Q layout:  X[i][j] of block (I, J) in lane 16 (j - 4J) + 4 pair + (i - 4I)
// an MFMA takes A in Q, B in P and returns D in P (scripts/ubench_valu.hip probes
// the lane maps), and the recursion closes without any data movement:
//   Z^T = G^T A'^T : A = G (V's P layout read as G^T in Q), B = A'^T (constant),
//                    D = Z^T in P = Z in Q
//   V   = sv Ab^T + Ef : A = sv (Z's Q layout), B = Ab^T (per pair, loaded once),
//                    C = Ef, D = V in P.
// Per element and step the VALU keeps the exp and the log (6 + 5 fp64 operations,
// table-driven with LDS tables) and a share of the column maxima; the 16 fmas of
// the two contractions go to the matrix cores (4 MFMAs per 64 elements).  A wave's
// next tile inputs (A, E, the prior) are loaded while it runs the current tile's
// recursion (C4: 1.51 -> 1.41 ms per launch on one box, profiles/r05u_ab_c4_*).
//
// Column maxima without fp64 work.  The exp's range reduction s = V * 2048/ln2 +
// (1.5 2^52 + 2^31) leaves n + 2^31 (n = round(V 2048/ln2)) in the low word of s as
// an unsigned integer whose order is V's; the column maximum is an integer max of
// those words (two v_permlane swaps reduce the four lane rows of both column blocks
// at once), rounded down to k = floor(n_max / 2048) (M = k ln 2), the shift by M is an
// integer subtraction inside the exp's exponent arithmetic, and M comes back in the
// log's integer exponent: log Z + M = (e + k) ln 2 + log(mantissa).  The maxima reach
// the Q layout of the log by one ds_bpermute per column block.  This needs |V| <
// 2^31 ln2/2048 (7.3e5); pairs whose inputs could exceed 7e5 over T steps (|V| <=
// T (max |E| + log S) for row sums <= 1) go to the exact fallback.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "vbhem_internal.h"
#include "vbhem_mfma4.h"

#ifndef VBHEM_BWD4_WAVES
#define VBHEM_BWD4_WAVES 4   // waves per SIMD
#endif

// The step as measured best over rounds 3-6 (the variants that lost are
// in git history and DESIGN.md 8):
//   * the log from an 8192-interval table ({1/c, -log(1/c)}, 128 KB of LDS: one 16-wave
//     block per CU) with log1p to second order (|r| <= 2^-14: the dropped r^3/3 <= 7.6e-14)
//   * column maxima rounded down to a multiple of ln 2 (M = k ln2): the exp table index
//     n mod 2048 does not depend on the maximum, so its LDS read issues right after the
//     range reduction, beside the cross-lane maximum chain
//   * no per-step underflow test of Z for a cluster whose A' entries are all >= 2^-600
//     (Z >= min A' G_max >= 2^-601 > 2^-665 always): the tile loop is versioned on it
//   * Ef = E + amax rowsum(Ab) by one fma per element from the row sums the range check
//     computes on the matrix cores
//   * the range check (|E|, |Ef| < vlim, Ab row sums <= 1) as ordered compares into a wave
//     mask (an fmax chain compiles with NaN canonicalisation)
//   * round 6: the log's exponent applied to the table's 1/c by one v_mad_i32_i24
//     instead of inserting 1.0's exponent into Z (v_bfi_b32 + v_mov_b32; vbhem_mfma4.h
//     log_x_n): 104 -> 100 VALU instructions per quad-step, same bits, 1.249 -> 1.238 ms
//     per C4 launch (profiles/r06d_ab_c4_bwd4_logx_emask.txt, profiles/r06_isa_step.txt)

namespace vbhem {

namespace {

constexpr int kWaves = VBHEM_BWD4_WAVES;
constexpr int kNWB = 16;   // waves per block: one block per CU, the 144 KB of tables once per CU
using namespace m4;

}  // namespace

template <bool O32>
__global__ __launch_bounds__(64 * kNWB) __attribute__((amdgpu_waves_per_eu(kWaves)))
void fb_bwd4_kernel(const SplitArgs p) {
  constexpr int S = 8;
  // one array, the exp table first: both tables' LDS offsets then fit the 16-bit
  // offset field of ds_read (no address add per lookup)
  __shared__ __attribute__((aligned(16))) double tabs[2048 + 2 * 8192];
  double *const etab = tabs;                 // 2^(i/2048 - 1010)
  double *const ltab8 = tabs + 2048;         // {2^1023/c, -log(1/c)} (stage_log8k_x)
  __shared__ double amax[S], lpi[S];
  const int tid = threadIdx.x;
  for (int x = tid; x < 2048; x += 64 * kNWB) etab[x] = kExpTab4[x] * 0x1p-1010;
  stage_log8k_x(ltab8, tid, 64 * kNWB);
  const int SB = p.SB, K = p.K, T = p.T;
  // persistent: NB blocks per cluster; XCD-aware when NB % 8 == 0 (as fb_bwd2_kernel)
  const int bk = blockIdx.x, NB = (int)gridDim.x / K;
  int j, t0;
  if (NB % 8 == 0) {
    const int rr = bk / 8;
    j = rr % K;
    t0 = (rr / K) * 8 + bk % 8;
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
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane >> 4, b = (lane >> 2) & 3, c = lane & 3;
  // B operand of Z^T = G^T A'^T, block (K, I'): A'[4I' + c][4K + r]
  double AT[2][2];
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) AT[k2][i2] = p.Atg[(size_t)j * S * S + (4 * i2 + c) * S + 4 * k2 + r];
  // amax (P layout: sigma = 4I + r) and lpi are read from LDS where they are used (once
  // per tile), not held in registers across the loop
  bool cl_nf = false;
#pragma unroll
  for (int x = 0; x < S; ++x) cl_nf |= isnan(amax[x]) || isnan(lpi[x]);
  // the lanes hold the 64 entries of A' between them: a wave minimum (once per block)
  bool zsafe;
  {
    double am = fmin(fmin(AT[0][0], AT[0][1]), fmin(AT[1][0], AT[1][1]));
    for (int o = 32; o >= 1; o >>= 1) am = fmin(am, __shfl_xor(am, o, 64));
    zsafe = am >= 0x1p-600;  // NaN: not safe
  }
  zsafe = __builtin_amdgcn_readfirstlane((int)zsafe) != 0;
  // ds_bpermute sources of the log's column maxima (Q layout: column 4J + r)
  const int qsrc0 = (0 * 16 + 4 * b + r) << 2, qsrc1 = (1 * 16 + 4 * b + r) << 2;
  const unsigned long long pmask = 0x000F000F000F000Full << (4 * b);
  // the integer maxima's range: |V| <= T (max |Ef| + log S) for row sums <= 1
  const double vlim = kVMax / (double)T - 3.0;

  // the tile loop, versioned on the underflow test (ZS: the cluster's A' makes it
  // unnecessary) and on SB == 8 (F8: every base state present, so no clamp or zero
  // select is left in the tile's addresses and operands)
  auto tiles = [&](auto zs_tag, auto f8_tag) {
  constexpr bool ZS = decltype(zs_tag)::value;
  constexpr bool F8 = decltype(f8_tag)::value;
  const int SBk = F8 ? 8 : SB;
  const int ntile = (p.i_end - p.i_begin + 3) / 4;
  const int tstride = NB * kNWB;
  // a tile's global inputs (A, E, the prior), loaded one tile ahead: the next tile's
  // loads are in flight during this tile's recursion instead of each tile starting
  // with a full memory latency (clamped addresses, no selects on the loaded values
  // until the tile is processed)
  struct TileIn {
    double a[2][2], e[2][2], pr;
  };
  // O32: 32-bit element offsets from the uniform base pointers (launch_bwd4 checks that
  // A, the prior and E stay below 4 GB), so every load is one offset computation and a
  // saddr load instead of 64-bit address arithmetic
  using off_t_ = typename std::conditional<O32, unsigned, size_t>::type;
  auto ld = [](const double *base, off_t_ x) {
    if constexpr (O32)
      return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + x * 8u);
    else
      return base[x];
  };
  auto load_tile = [&](int tile, TileIn &in) {
    const int i = p.i_begin + tile * 4 + b;
    const int ic = i < p.i_end ? i : p.i_end - 1;
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int be = 4 * jj + c, bp = 4 * j2 + r;
        const off_t_ x = ((off_t_)ic * SBk + (be < SBk ? be : SBk - 1)) * SBk + (bp < SBk ? bp : SBk - 1);
        in.a[j2][jj] = ld(p.A, x);
      }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int be = 4 * jj + c;
        const off_t_ x = (off_t_)(j * S + 4 * i2 + r) * (off_t_)p.e_ld +
                         (off_t_)(ic - p.i_buf0) * SBk + (be < SBk ? be : SBk - 1);
        in.e[i2][jj] = ld(p.E, x);
      }
    const int be = 4 * (r & 1) + c;
    in.pr = ld(p.prior, (off_t_)ic * SBk + (be < SBk ? be : SBk - 1));
  };
  TileIn cur;
  if (wave * NB + t0 < ntile) load_tile(wave * NB + t0, cur);
  for (int tile = wave * NB + t0; tile < ntile; tile += tstride) {
    const int i = p.i_begin + tile * 4 + b;
    TileIn nxt;
    load_tile(min(tile + tstride, ntile - 1), nxt);  // (past the last tile: a repeat)
    double Ef[2][2], V[2][2], AbT[2][2];
    // B operand of V = sv Ab^T + Ef, block (J', J): Ab[4J + c][4J' + r] (zero past SB)
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int be = 4 * jj + c, bp = 4 * j2 + r;
        AbT[j2][jj] = (be < SBk && bp < SBk) ? cur.a[j2][jj] : 0.0;
      }
    bool nf = false;
    uint64_t bigm = 0;  // the lanes failing the range check
    // row sums of Ab (P layout: every lane row holds column 4J + c's sum), then
    // Ef = E + amax[sigma] rowsum(Ab)[beta] as one fma per element (the P layout's row
    // sigma = 4I + r)
    double rsj[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) rsj[jj] = mfma4(1.0, AbT[1][jj], mfma4(1.0, AbT[0][jj], 0.0));
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const double amr = amax[4 * i2 + r];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const double e = cur.e[i2][jj];
        V[i2][jj] = e;
        Ef[i2][jj] = fma(amr, rsj[jj], e);
        bigm |= ge_mask(fabs(e), vlim);
        bigm |= ge_mask(fabs(Ef[i2][jj]), vlim);
        nf |= !isfinite(Ef[i2][jj]);
      }
    }
    bigm |= gt_mask(rsj[0], 1.0 + 1e-6);
    bigm |= gt_mask(rsj[1], 1.0 + 1e-6);
    int zmin = 0x7fffffff;

    // ---- K2: backward recursion, t = T-1 .. 1 ----
    // (column maxima -> exp -> 2 MFMA -> log -> 2 MFMA per step)
    for (int t = T - 1; t >= 1; --t) {
      double sf[4], tv[4], vv[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        vv[x] = V[x / 2][x % 2];
        sf[x] = red_s(vv[x]);
      }
      // table values first (they do not need the maxima), then the maxima chain
#pragma unroll
      for (int x = 0; x < 4; ++x) tv[x] = etab_at(etab, sf[x]);
      const unsigned w = colmax_rows(max(lo_u(sf[0]), lo_u(sf[2])), max(lo_u(sf[1]), lo_u(sf[3]))) >> 11;
      const int wq = (int)w - (1 << 20) - 1023;
      int mq[2];
      mq[0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq);
      mq[1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq);
      unsigned wph[2];
      split_rows(w - 1010u, wph[0], wph[1]);
      double G[2][2];
      {
        double gg[4];
        const unsigned wpf[4] = {wph[0], wph[1], wph[0], wph[1]};
        exp_d_n<4>(gg, vv, sf, tv, wpf);
#pragma unroll
        for (int x = 0; x < 4; ++x) G[x / 2][x % 2] = gg[x];
      }
      // Z^T block (J, I') = sum_K G^T(J, K) A'^T(K, I'); G^T(J, K) is V's block (K, J)
      double Z[2][2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) Z[jj][i2] = mfma4(G[0][jj], AT[0][i2], 0.0);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) Z[jj][i2] = mfma4(G[1][jj], AT[1][i2], Z[jj][i2]);
      double sv[2][2];
      {
        double zf[4], yf[4];
        const int wqf[4] = {mq[0], mq[0], mq[1], mq[1]};
#pragma unroll
        for (int x = 0; x < 4; ++x) zf[x] = Z[x / 2][x % 2];
        if constexpr (!ZS)
          zmin = min(zmin, min(min(__double2hiint(zf[0]), __double2hiint(zf[1])),
                               min(__double2hiint(zf[2]), __double2hiint(zf[3]))));
        log_x_n<4, true>(yf, zf, wqf, ltab8);
#pragma unroll
        for (int x = 0; x < 4; ++x) sv[x / 2][x % 2] = yf[x];
      }
      // V block (I, J) = Ef + sum_J' sv(I, J') Ab^T(J', J); sv(I, J') is Z^T's block (J', I)
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) V[i2][jj] = mfma4(sv[0][i2], AbT[0][jj], Ef[i2][jj]);
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) V[i2][jj] = mfma4(sv[1][i2], AbT[1][jj], V[i2][jj]);
    }

    // ---- K3: termination, L_elbo = sum_beta prior_beta log sum_sigma exp(lpi + E + L) ----
    // (the x1 reduction: m = the full column maximum of lo(s), M = m ln2/2048)
    {
      double W[2][2], s[2][2];
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          // (a state of zero initial probability: lpi = -inf, kept in the integer range)
          W[i2][jj] = fmax(lpi[4 * i2 + r] + V[i2][jj], -7.2e5);
          s[i2][jj] = red_s(W[i2][jj]);
        }
      const unsigned w = colmax_rows(max(lo_u(s[0][0]), lo_u(s[1][0])), max(lo_u(s[0][1]), lo_u(s[1][1])));
      unsigned wp[2];
      split_rows(w - kBias, wp[0], wp[1]);
      double ev[2][2];
      {
        const double wf[4] = {W[0][0], W[0][1], W[1][0], W[1][1]};
        const double sf[4] = {s[0][0], s[0][1], s[1][0], s[1][1]};
        const unsigned wpf[4] = {wp[0], wp[1], wp[0], wp[1]};
        double ef[4];
        exp_m_n<4>(ef, wf, sf, wpf, etab);
        ev[0][0] = ef[0]; ev[0][1] = ef[1]; ev[1][0] = ef[2]; ev[1][1] = ef[3];
      }
      // row r: column 4 (r & 1) + c, the layout of w
      const double zs = colsum_rows(ev[0][0] + ev[1][0], ev[0][1] + ev[1][1]);
      double lse1[1];
      {
        const double zsf[1] = {zs};
        const int wqf[1] = {(int)(w + kWq0)};
        log_x_n<1, false>(lse1, zsf, wqf, ltab8);
      }
      const double lse = lse1[0];
      const int be = 4 * (r & 1) + c;
      const double pr = be < SBk ? cur.pr : 0.0;
      double y = r < 2 ? pr * lse : 0.0;
      const bool bad = zmin < kZMinHi || !isfinite(y);
      y += shfl_xor_d(y, 1);
      y += shfl_xor_d(y, 2);
      y += shfl_xor_d(y, 16);
      const bool pbad = ((__ballot(bad) | bigm) & pmask) != 0;
      const bool pnf = cl_nf || (__ballot(nf) & pmask) != 0;
      if (lane == 4 * b && r == 0 && i < p.i_end) {
        const size_t pair = (size_t)i * K + j;
        if (pbad && !pnf) {
          // underflow or range with finite inputs: the exact kernel recomputes the pair
          const int slot = atomicAdd(p.flag_count, 1);
          atomicAdd(p.flag_count + 1, 1);
          p.flag_list[slot] = (int)pair;
          p.LL[pair] = y;
        } else {
          p.LL[pair] = (pbad && pnf) ? __builtin_nan("") : y;
        }
      }
    }
    cur = nxt;
  }
  };
  if (SB == 8) {
    if (zsafe) tiles(std::true_type{}, std::true_type{});
    else tiles(std::false_type{}, std::true_type{});
  } else {
    if (zsafe) tiles(std::true_type{}, std::false_type{});
    else tiles(std::false_type{}, std::false_type{});
  }
}

// ---------------------------------------------------------------------------
bool bwd4_supported(int S, int SB) { return S == 8 && SB >= 1 && SB <= 8; }
int bwd4_waves() { return kNWB; }
int bwd4_ppb() { return kNWB * 4; }
int bwd4_resident_blocks() {
  return resident_per_cu(reinterpret_cast<const void *>(&fb_bwd4_kernel<true>), 64 * kNWB, 0);
}
// the O32 version when every byte offset of A, the prior and E fits 32 bits
bool bwd4_o32(const SplitArgs &a) {
  const unsigned long long lim = 0xffffffffull / 8;
  return (unsigned long long)a.i_end * a.SB * a.SB < lim &&
         (unsigned long long)a.K * a.S * (unsigned long long)a.e_ld < lim;
}

hipError_t launch_bwd4(const SplitArgs &a, unsigned grid, hipStream_t st, hipEvent_t t0,
                       hipEvent_t t1) {
  if (!bwd4_supported(a.S, a.SB) || !a.Atg) return hipErrorInvalidValue;
  auto *fn = bwd4_o32(a) ? &fb_bwd4_kernel<true> : &fb_bwd4_kernel<false>;
  if (t0)  // timing events recorded by the dispatch itself (the bench's roofline)
    hipExtLaunchKernelGGL(fn, dim3(grid), dim3(64 * kNWB), 0, st, t0, t1, 0, a);
  else
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * kNWB), 0, st, a);
  return hipGetLastError();
}

}  // namespace vbhem

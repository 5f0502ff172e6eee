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
// A wavefront holds QPW quads of 4 pairs (4 consecutive bases of one cluster); the
// 4 pairs of a quad are the 4 blocks of every MFMA, so no operand is padded.  With
//   P layout:  X[i][j] of block (I, J) in lane 16 (i - 4I) + 4 pair + (j - 4J)
//   Q layout:  X[i][j] of block (I, J) in lane 16 (j - 4J) + 4 pair + (i - 4I)
// an MFMA takes A in Q, B in P and returns D in P (scripts/ubench_valu.hip probes
// the lane maps), and the recursion closes without any data movement:
//   Z^T = G^T A'^T : A = G (V's P layout read as G^T in Q), B = A'^T (constant),
//                    D = Z^T in P = Z in Q
//   V   = sv Ab^T + Ef : A = sv (Z's Q layout), B = Ab^T (per pair, loaded once),
//                    C = Ef, D = V in P.
// Per element and step the VALU keeps the exp and the log (7 + 8 fp64 operations,
// table-driven with LDS tables) and a share of the column maxima; the 16 fmas of
// the two contractions go to the matrix cores (4 MFMAs per 64 elements).  A wave's
// next tile inputs (A, E, the prior) are loaded while it runs the current tile's
// recursion (C4: 1.51 -> 1.41 ms per launch on one box, profiles/r05u_ab_c4_*).
//
// Column maxima without fp64 work.  The exp's range reduction s = V * 2048/ln2 +
// (1.5 2^52 + 2^31) leaves n + 2^31 (n = round(V 2048/ln2)) in the low word of s as
// an unsigned integer whose order is V's; the column maximum m is an integer max of
// those words (two v_permlane swaps reduce the four lane rows of both column blocks
// at once), the shift by M = m ln2/2048 is an integer subtraction inside the exp's
// exponent arithmetic, and M comes back in the log's integer exponent: log Z + M =
// (k 2048 + m) ln2/2048 + log(mantissa).  The maxima reach the Q layout of the log
// by one ds_bpermute per column block.  This needs |V| < 2^31 ln2/2048 (7.3e5);
// pairs whose inputs could exceed 7e5 over T steps (|V| <= T (max |E| + log S) for
// row sums <= 1) go to the exact fallback.
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
#ifndef VBHEM_BWD4_QPW
#define VBHEM_BWD4_QPW 1     // quads (of 4 pairs) per wavefront
#endif

// Step-loop variants (A/B switches; the defaults are the measured best -- all three on:
// 1.553 -> 1.496 ms per C4 launch on one box, gpurun_out r04a A/B):
//   VBHEM_BWD4_BIGLOG   the log from an 8192-interval table ({1/c, -log(1/c)}, 128 KB
//                       of LDS: one 16-wave block per CU) with log1p to second order
//                       (|r| <= 2^-14: the dropped r^3/3 <= 7.6e-14), two fp64
//                       operations less per element and step than the 1024-interval
//                       table's third-order series
//   VBHEM_BWD4_DECOUPLE column maxima rounded down to a multiple of ln 2 (M = k ln2):
//                       the exp table index n mod 2048 no longer depends on the maximum,
//                       so its LDS read issues right after the range reduction, beside
//                       the cross-lane maximum chain instead of after it
//   VBHEM_BWD4_ZSAFE    no per-step underflow test of Z for a cluster whose A' entries
//                       are all >= 2^-600 (Z >= min A' G_max >= 2^-601 > 2^-665 always)
#ifndef VBHEM_BWD4_BIGLOG
#define VBHEM_BWD4_BIGLOG 1
#endif
#ifndef VBHEM_BWD4_DECOUPLE
#define VBHEM_BWD4_DECOUPLE 1
#endif
#ifndef VBHEM_BWD4_ZSAFE
#define VBHEM_BWD4_ZSAFE 1
#endif
//   VBHEM_BWD4_SKEW     two quads per wavefront on skewed halves of the step: while
//                       one quad takes its log and second contraction, the other takes
//                       its exp and first contraction (independent work side by side
//                       in every half-step; needs VBHEM_BWD4_QPW=2, BIGLOG, DECOUPLE)
#ifndef VBHEM_BWD4_SKEW
#define VBHEM_BWD4_SKEW 0
#endif
//   VBHEM_BWD4_SB       a scheduling barrier right after the exp table reads (A/B)
#ifndef VBHEM_BWD4_SB
#define VBHEM_BWD4_SB 0
#endif
//   VBHEM_BWD4_PRIO     static priority 1 for the second half of the block's waves
//                       (MI355X_MICROARCH.md, two waves per SIMD, item 4) (A/B)
#ifndef VBHEM_BWD4_PRIO
#define VBHEM_BWD4_PRIO 0
#endif
//   VBHEM_BWD4_ETAB2    the exp table as {t, t/2} pairs (vbhem_mfma4.h exp_d2_n: one fp64
//                       operation less per element and step); its 32 KB and the log
//                       table's 128 KB fill the CU's 160 KB, so the cluster's row maxima of
//                       logA (stored past A') and log pi are read from global memory.
//                       Measured no faster (C4 1.43-1.49 vs 1.42-1.44 ms per launch, shard
//                       0.189 vs 0.184-0.187 ms; profiles/r05am_ab_bwd4_etab2.txt): the
//                       16-byte table reads cost what the fp64 operation saved.  A/B switch
//   VBHEM_EF_VALU       Ef = E + amax rowsum(Ab) as one fma per element from the row sums
//                       the range check computes anyway, instead of 2 MFMAs per element
//                       (8 of a tile's 12 setup MFMAs); the same in fb_bwd12_kernel
#ifndef VBHEM_EF_VALU
#define VBHEM_EF_VALU 1
#endif
#ifndef VBHEM_BWD4_ETAB2
#define VBHEM_BWD4_ETAB2 0
#endif
#if VBHEM_BWD4_ETAB2 && (VBHEM_BWD4_SKEW || !VBHEM_BWD4_BIGLOG || !VBHEM_BWD4_DECOUPLE)
#error "VBHEM_BWD4_ETAB2 needs BIGLOG and DECOUPLE, without SKEW"
#endif
#if VBHEM_BWD4_SKEW && !(VBHEM_BWD4_QPW == 2 && VBHEM_BWD4_BIGLOG && VBHEM_BWD4_DECOUPLE)
#error "VBHEM_BWD4_SKEW needs VBHEM_BWD4_QPW=2 with BIGLOG and DECOUPLE"
#endif

namespace vbhem {

namespace {

constexpr int kQPW = VBHEM_BWD4_QPW;
constexpr int kWaves = VBHEM_BWD4_WAVES;
#ifndef VBHEM_BWD4_NWB
#if VBHEM_BWD4_BIGLOG
#define VBHEM_BWD4_NWB 16   // one block per CU: the 144 KB of tables once per CU
#else
#define VBHEM_BWD4_NWB 4
#endif
#endif
// waves per block (the 32 KB of tables once per block; LDS then allows 4 blocks per CU):
// 5 waves per SIMD (VBHEM_BWD4_WAVES=5, NWB=10, with the lane geometry recomputed per
// tile to fit) measured 1.87 vs 1.69 ms, 8-wave blocks 1.69-1.72: more waves per SIMD
// only add contention between the MFMA and VALU work
constexpr int kNWB = VBHEM_BWD4_NWB;
constexpr int kPPW = 4 * kQPW;      // pairs per wavefront (one tile)
using namespace m4;

}  // namespace

template <bool O32>
__global__ __launch_bounds__(64 * kNWB) __attribute__((amdgpu_waves_per_eu(kWaves)))
void fb_bwd4_kernel(const SplitArgs p) {
  constexpr int S = 8;
#if VBHEM_BWD4_ETAB2
  // 163,840 B: all of the CU's LDS (one block per CU)
  __shared__ __attribute__((aligned(16))) double tabs[2 * 2048 + 2 * 8192];
  double *const etab = tabs;                 // {2^(i/2048 - 1010), half of it}
  double *const ltab8 = tabs + 2 * 2048;     // {1/c, -log(1/c)}
#elif VBHEM_BWD4_BIGLOG
  // one array, the exp table first: both tables' LDS offsets then fit the 16-bit
  // offset field of ds_read (no address add per lookup)
  __shared__ __attribute__((aligned(16))) double tabs[2048 + 2 * 8192];
  double *const etab = tabs;                 // 2^(i/2048 - 1010)
  double *const ltab8 = tabs + 2048;         // {1/c, -log(1/c)}
#else
  __shared__ __attribute__((aligned(16))) double etab[2048];      // 2^(i/2048 - 1010)
  __shared__ __attribute__((aligned(16))) double ltab[2 * 1024];  // {1/(2c), -log(1/c)}
#endif
#if !VBHEM_BWD4_ETAB2
  __shared__ double amax[S], lpi[S];
#endif
  const int tid = threadIdx.x;
#if VBHEM_BWD4_ETAB2
  stage_etab2(etab, tid, 64 * kNWB);
  stage_log8k<false>(ltab8, tid, 64 * kNWB);
#elif VBHEM_BWD4_BIGLOG
  for (int x = tid; x < 2048; x += 64 * kNWB) etab[x] = kExpTab4[x] * 0x1p-1010;
  stage_log8k<false>(ltab8, tid, 64 * kNWB);
#else
  stage_tables(etab, ltab, tid, 64 * kNWB);
#endif
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
#if VBHEM_BWD4_ETAB2
  // the row maxima of logA in global memory past A' ([K][S] after the [K][S][S] block,
  // every block of the cluster writing the same values), read once per tile with log pi
  // where they are used (L1 hits; kept in registers they would spill)
  double *const amax = const_cast<double *>(p.Atg) + (size_t)K * S * S + (size_t)j * S;
  const double *const lpi = p.logPi + (size_t)j * S;
  if (tid < S) {
    const double *la = p.logA + ((size_t)j * S + tid) * S;
    double mx = la[0];
    for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[s2]);
    amax[tid] = mx;
  }
  __syncthreads();
#else
  if (tid < S) {
    const double *la = p.logA + ((size_t)j * S + tid) * S;
    double mx = la[0];
    for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[s2]);
    amax[tid] = mx;
    lpi[tid] = p.logPi[(size_t)j * S + tid];
  }
  __syncthreads();
#endif

  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane >> 4, b = (lane >> 2) & 3, c = lane & 3;
  // B operand of Z^T = G^T A'^T, block (K, I'): A'[4I' + c][4K + r]
  double AT[2][2];
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) AT[k2][i2] = p.Atg[(size_t)j * S * S + (4 * i2 + c) * S + 4 * k2 + r];
  // A operand of the amax fold (rows amax[sigma], Q layout: sigma = 4I + c)
  // amax (Q layout: sigma = 4I + c) and lpi (P layout: sigma = 4I + r) are read from
  // LDS where they are used (once per tile), not held in registers across the loop
  bool cl_nf = false;
#pragma unroll
  for (int x = 0; x < S; ++x) cl_nf |= isnan(amax[x]) || isnan(lpi[x]);
#if VBHEM_BWD4_ZSAFE
  // the lanes hold the 64 entries of A' between them: a wave minimum (once per block)
  bool zsafe;
  {
    double am = fmin(fmin(AT[0][0], AT[0][1]), fmin(AT[1][0], AT[1][1]));
    for (int o = 32; o >= 1; o >>= 1) am = fmin(am, __shfl_xor(am, o, 64));
    zsafe = am >= 0x1p-600;  // NaN: not safe
  }
  zsafe = __builtin_amdgcn_readfirstlane((int)zsafe) != 0;
#else
  constexpr bool zsafe = false;
#endif
  // ds_bpermute sources of the log's column maxima (Q layout: column 4J + r)
  const int qsrc0 = (0 * 16 + 4 * b + r) << 2, qsrc1 = (1 * 16 + 4 * b + r) << 2;
  const unsigned long long pmask = 0x000F000F000F000Full << (4 * b);
  const double vlim = kVMax / (double)T - 3.0;

#if VBHEM_BWD4_PRIO
  if (wave >= kNWB / 2) __builtin_amdgcn_s_setprio(1);
#endif
  // the tile loop, versioned on the underflow test (ZS: the cluster's A' makes it
  // unnecessary, VBHEM_BWD4_ZSAFE)
  // and on SB == 8 (F8: every base state present, so no clamp or zero select is
  // left in the tile's addresses and operands)
  auto tiles = [&](auto zs_tag, auto f8_tag) {
  constexpr bool ZS = decltype(zs_tag)::value;
  constexpr bool F8 = decltype(f8_tag)::value;
  const int SBk = F8 ? 8 : SB;
  const int ntile = (p.i_end - p.i_begin + kPPW - 1) / kPPW;
  const int tstride = NB * kNWB;
  // a tile's global inputs (A, E, the prior), loaded one tile ahead: the next tile's
  // loads are in flight during this tile's recursion instead of each tile starting
  // with a full memory latency (clamped addresses, no selects on the loaded values
  // until the tile is processed)
  struct TileIn {
    double a[kQPW][2][2], e[kQPW][2][2], pr[kQPW];
  };
  // O32: 32-bit element offsets from the uniform base pointers (launch_bwd4 checks that
  // A, the prior and E stay below 4 GB), so every load is one offset computation and a
  // saddr load instead of 64-bit address arithmetic (with the SB == 8 versions this
  // also took the kernel's last 12 bytes of scratch away)
  using off_t_ = typename std::conditional<O32, unsigned, size_t>::type;
  auto ld = [](const double *base, off_t_ x) {
    if constexpr (O32)
      return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + x * 8u);
    else
      return base[x];
  };
  auto load_tile = [&](int tile, TileIn &in) {
    const int i0 = p.i_begin + tile * kPPW;
#pragma unroll
    for (int q = 0; q < kQPW; ++q) {
      const int i = i0 + 4 * q + b;
      const int ic = i < p.i_end ? i : p.i_end - 1;
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int be = 4 * jj + c, bp = 4 * j2 + r;
          const off_t_ x = ((off_t_)ic * SBk + (be < SBk ? be : SBk - 1)) * SBk + (bp < SBk ? bp : SBk - 1);
          in.a[q][j2][jj] = ld(p.A, x);
        }
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int be = 4 * jj + c;
          const off_t_ x = (off_t_)(j * S + 4 * i2 + r) * (off_t_)p.e_ld +
                           (off_t_)(ic - p.i_buf0) * SBk + (be < SBk ? be : SBk - 1);
          in.e[q][i2][jj] = ld(p.E, x);
        }
      const int be = 4 * (r & 1) + c;
      in.pr[q] = ld(p.prior, (off_t_)ic * SBk + (be < SBk ? be : SBk - 1));
    }
  };
  TileIn cur;
  if (wave * NB + t0 < ntile) load_tile(wave * NB + t0, cur);
  for (int tile = wave * NB + t0; tile < ntile; tile += tstride) {
    const int i0 = p.i_begin + tile * kPPW;
    TileIn nxt;
    load_tile(min(tile + tstride, ntile - 1), nxt);  // (past the last tile: a repeat)
    double Ef[kQPW][2][2], V[kQPW][2][2], AbT[kQPW][2][2];
    bool rbad[kQPW], nfb[kQPW];
    uint64_t rbadm[kQPW];
    int zmin[kQPW];
#pragma unroll
    for (int q = 0; q < kQPW; ++q) {
      // B operand of V = sv Ab^T + Ef, block (J', J): Ab[4J + c][4J' + r] (zero past SB)
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int be = 4 * jj + c, bp = 4 * j2 + r;
          AbT[q][j2][jj] = (be < SBk && bp < SBk) ? cur.a[q][j2][jj] : 0.0;
        }
      double mabs = 0.0, rs = 0.0;
      bool nf = false;
      uint64_t bigm = 0;  // VBHEM_RANGE_CMP: the lanes failing the range check
#if VBHEM_EF_VALU
      // row sums of Ab (P layout: every lane row holds column 4J + c's sum), then
      // Ef = E + amax[sigma] rowsum(Ab)[beta] as one fma per element (the P layout's row
      // sigma = 4I + r) instead of two MFMAs
      double rsj[2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) rsj[jj] = mfma4(1.0, AbT[q][1][jj], mfma4(1.0, AbT[q][0][jj], 0.0));
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        const double amr = amax[4 * i2 + r];
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const double e = cur.e[q][i2][jj];
          V[q][i2][jj] = e;
          Ef[q][i2][jj] = fma(amr, rsj[jj], e);
#if VBHEM_RANGE_CMP
          bigm |= ge_mask(fabs(e), vlim);
          bigm |= ge_mask(fabs(Ef[q][i2][jj]), vlim);
#else
          mabs = fmax(mabs, fmax(fabs(e), fabs(Ef[q][i2][jj])));
#endif
          nf |= !isfinite(Ef[q][i2][jj]);
        }
      }
#if VBHEM_RANGE_CMP
      bigm |= gt_mask(rsj[0], 1.0 + 1e-6);
      bigm |= gt_mask(rsj[1], 1.0 + 1e-6);
#else
      rs = fmax(rsj[0], rsj[1]);
#endif
#else
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const double e = cur.e[q][i2][jj];
          V[q][i2][jj] = e;
          // Ef = E + amax[sigma] sum_b' Ab[beta][b'] on the matrix cores
          const double am = amax[4 * i2 + c];
          Ef[q][i2][jj] = mfma4(am, AbT[q][1][jj], mfma4(am, AbT[q][0][jj], e));
          mabs = fmax(mabs, fmax(fabs(e), fabs(Ef[q][i2][jj])));
          nf |= !isfinite(Ef[q][i2][jj]);
        }
      // row sums of Ab (P layout, column 4J + c): the |V| bound assumes <= 1
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) rs = fmax(rs, mfma4(1.0, AbT[q][1][jj], mfma4(1.0, AbT[q][0][jj], 0.0)));
#endif
      // bigm (VBHEM_RANGE_CMP): the same test as a wave mask, joined at the ballot
      rbad[q] = !(mabs < vlim) || rs > 1.0 + 1e-6;
      rbadm[q] = bigm;
      nfb[q] = nf;
      zmin[q] = 0x7fffffff;
    }

    // ---- K2: backward recursion, t = T-1 .. 1 ----
#if VBHEM_BWD4_SKEW
    // the first half of a step for quad q: maxima, exp, Z^T = G^T A'^T (-> Zs, mqs)
    double Zs[kQPW][2][2];
    int mqs[kQPW][2];
    auto half_e = [&](int q) {
      double sf[4], tv[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) sf[x] = red_s(V[q][x / 2][x % 2]);
#pragma unroll
      for (int x = 0; x < 4; ++x) tv[x] = etab_at(etab, sf[x]);
      const unsigned w = colmax_rows(max(lo_u(sf[0]), lo_u(sf[2])), max(lo_u(sf[1]), lo_u(sf[3]))) >> 11;
      const int wq = (int)w - (1 << 20) - 1023;
      mqs[q][0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq);
      mqs[q][1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq);
      unsigned wp0, wp1;
      split_rows(w - 1010u, wp0, wp1);
      double vv[4], gg[4];
      const unsigned wpf[4] = {wp0, wp1, wp0, wp1};
#pragma unroll
      for (int x = 0; x < 4; ++x) vv[x] = V[q][x / 2][x % 2];
      exp_d_n<4>(gg, vv, sf, tv, wpf);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
          Zs[q][jj][i2] = mfma4(gg[2 + jj], AT[1][i2], mfma4(gg[jj], AT[0][i2], 0.0));
    };
    // the second half: sv = M + log Z, V = Ef + sv Ab^T
    auto half_l = [&](int q, auto zs_tag) {
      constexpr bool ZS_ = decltype(zs_tag)::value;
      double zf[4], yf[4];
      const int wqf[4] = {mqs[q][0], mqs[q][0], mqs[q][1], mqs[q][1]};
#pragma unroll
      for (int x = 0; x < 4; ++x) zf[x] = Zs[q][x / 2][x % 2];
      if constexpr (!ZS_)
        zmin[q] = min(zmin[q], min(min(__double2hiint(zf[0]), __double2hiint(zf[1])),
                                   min(__double2hiint(zf[2]), __double2hiint(zf[3]))));
      log_q_n<4, true, false>(yf, zf, wqf, ltab8);
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          V[q][i2][jj] = mfma4(yf[2 + i2], AbT[q][1][jj], mfma4(yf[i2], AbT[q][0][jj], Ef[q][i2][jj]));
    };
    half_e(0);
    for (int t = T - 1; t >= 1; --t) {
      half_l(0, zs_tag);
      half_e(1);
      if (t > 1) half_e(0);
      half_l(1, zs_tag);
    }
#else
    // each phase over all quads of the wavefront before the next one, so the
    // independent quads sit next to each other in the dependency chain of a step
    // (column maxima -> exp -> MFMA -> log -> MFMA)
    for (int t = T - 1; t >= 1; --t) {
      double s[kQPW][2][2];
      int mq[kQPW][2];
      constexpr int NE = 4 * kQPW;  // elements per lane: (q, I, J) flattened
      double G[kQPW][2][2];
#if VBHEM_BWD4_DECOUPLE
      // table values first (they do not need the maxima), then the maxima chain
#if VBHEM_BWD4_ETAB2
      double2 tv[NE];
#else
      double tv[NE];
#endif
      unsigned wph[kQPW][2];
#pragma unroll
      for (int q = 0; q < kQPW; ++q)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) s[q][i2][jj] = red_s(V[q][i2][jj]);
#pragma unroll
#if VBHEM_BWD4_ETAB2
      for (int x = 0; x < NE; ++x) tv[x] = etab2_at(etab, s[x / 4][(x / 2) % 2][x % 2]);
#else
      for (int x = 0; x < NE; ++x) tv[x] = etab_at(etab, s[x / 4][(x / 2) % 2][x % 2]);
#endif
#ifdef VBHEM_ABL_NOETAB  // ablation (timing only, wrong results): no exp table read
#pragma unroll
      for (int x = 0; x < NE; ++x) tv[x] = {};
#endif
#if VBHEM_BWD4_SB
      // A/B: every exp table read issued before anything after it (no interleaving that
      // waits on the first read before the others are out)
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int q = 0; q < kQPW; ++q) {
        const unsigned w = colmax_rows(max(lo_u(s[q][0][0]), lo_u(s[q][1][0])),
                                       max(lo_u(s[q][0][1]), lo_u(s[q][1][1]))) >> 11;
        const int wq = (int)w - (1 << 20) - 1023;
        mq[q][0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq);
        mq[q][1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq);
        split_rows(w - 1010u, wph[q][0], wph[q][1]);
      }
      {
        double vv[NE], sf[NE], gg[NE];
        unsigned wpf[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) {
          vv[x] = V[x / 4][(x / 2) % 2][x % 2];
          sf[x] = s[x / 4][(x / 2) % 2][x % 2];
          wpf[x] = wph[x / 4][x % 2];
        }
#if VBHEM_BWD4_ETAB2
        exp_d2_n<NE>(gg, vv, sf, tv, wpf);
#else
        exp_d_n<NE>(gg, vv, sf, tv, wpf);
#endif
#pragma unroll
        for (int x = 0; x < NE; ++x) G[x / 4][(x / 2) % 2][x % 2] = gg[x];
      }
#else
      unsigned wp[kQPW][2];
#pragma unroll
      for (int q = 0; q < kQPW; ++q) {
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) s[q][i2][jj] = red_s(V[q][i2][jj]);
        const unsigned w = colmax_rows(max(lo_u(s[q][0][0]), lo_u(s[q][1][0])),
                                       max(lo_u(s[q][0][1]), lo_u(s[q][1][1])));
        const int wq = (int)(w + kWq0);
        mq[q][0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq);
        mq[q][1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq);
        split_rows(w - kBias, wp[q][0], wp[q][1]);
      }
      {
        double vv[NE], sf[NE], gg[NE];
        unsigned wpf[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) {
          vv[x] = V[x / 4][(x / 2) % 2][x % 2];
          sf[x] = s[x / 4][(x / 2) % 2][x % 2];
          wpf[x] = wp[x / 4][x % 2];
        }
        exp_m_n<NE>(gg, vv, sf, wpf, etab);
#pragma unroll
        for (int x = 0; x < NE; ++x) G[x / 4][(x / 2) % 2][x % 2] = gg[x];
      }
#endif
      // Z^T block (J, I') = sum_K G^T(J, K) A'^T(K, I'); G^T(J, K) is V's block (K, J)
      double Z[kQPW][2][2];
#pragma unroll
      for (int q = 0; q < kQPW; ++q)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int i2 = 0; i2 < 2; ++i2) Z[q][jj][i2] = mfma4(G[q][0][jj], AT[0][i2], 0.0);
#pragma unroll
      for (int q = 0; q < kQPW; ++q)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int i2 = 0; i2 < 2; ++i2) Z[q][jj][i2] = mfma4(G[q][1][jj], AT[1][i2], Z[q][jj][i2]);
      double sv[kQPW][2][2];
      {
        double zf[NE], yf[NE];
        int wqf[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) {
          zf[x] = Z[x / 4][(x / 2) % 2][x % 2];
          wqf[x] = mq[x / 4][(x / 2) % 2];
        }
        if constexpr (!ZS) {
#pragma unroll
          for (int q = 0; q < kQPW; ++q)
            zmin[q] = min(zmin[q], min(min(__double2hiint(zf[4 * q]), __double2hiint(zf[4 * q + 1])),
                                       min(__double2hiint(zf[4 * q + 2]), __double2hiint(zf[4 * q + 3]))));
        }
#if VBHEM_BWD4_BIGLOG
        log_q_n<NE, VBHEM_BWD4_DECOUPLE != 0, false>(yf, zf, wqf, ltab8);
#elif VBHEM_BWD4_DECOUPLE
        log_d_n<NE>(yf, zf, wqf, ltab);
#else
        log_m_n<NE>(yf, zf, wqf, ltab);
#endif
#pragma unroll
        for (int x = 0; x < NE; ++x) sv[x / 4][(x / 2) % 2][x % 2] = yf[x];
      }
      // V block (I, J) = Ef + sum_J' sv(I, J') Ab^T(J', J); sv(I, J') is Z^T's block (J', I)
#pragma unroll
      for (int q = 0; q < kQPW; ++q)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) V[q][i2][jj] = mfma4(sv[q][0][i2], AbT[q][0][jj], Ef[q][i2][jj]);
#pragma unroll
      for (int q = 0; q < kQPW; ++q)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) V[q][i2][jj] = mfma4(sv[q][1][i2], AbT[q][1][jj], V[q][i2][jj]);
    }
#endif

    // ---- K3: termination, L_elbo = sum_beta prior_beta log sum_sigma exp(lpi + E + L) ----
#pragma unroll
    for (int q = 0; q < kQPW; ++q) {
      const int i = i0 + 4 * q + b;
      const int ic = i < p.i_end ? i : p.i_end - 1;
      double W[2][2], s[2][2];
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          // (a state of zero initial probability: lpi = -inf, kept in the integer range)
          W[i2][jj] = fmax(lpi[4 * i2 + r] + V[q][i2][jj], -7.2e5);
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
#if VBHEM_BWD4_ETAB2
        exp_m2_n<4>(ef, wf, sf, wpf, etab);
#else
        exp_m_n<4>(ef, wf, sf, wpf, etab);
#endif
        ev[0][0] = ef[0]; ev[0][1] = ef[1]; ev[1][0] = ef[2]; ev[1][1] = ef[3];
      }
      // row r: column 4 (r & 1) + c, the layout of w
      const double zs = colsum_rows(ev[0][0] + ev[1][0], ev[0][1] + ev[1][1]);
      double lse1[1];
      {
        const double zsf[1] = {zs};
        const int wqf[1] = {(int)(w + kWq0)};
#if VBHEM_BWD4_BIGLOG
        log_q_n<1, false, false>(lse1, zsf, wqf, ltab8);
#else
        log_m_n<1>(lse1, zsf, wqf, ltab);
#endif
      }
      const double lse = lse1[0];
      const int be = 4 * (r & 1) + c;
      const double pr = be < SBk ? cur.pr[q] : 0.0;
      double y = r < 2 ? pr * lse : 0.0;
      const bool bad = zmin[q] < kZMinHi || !isfinite(y) || rbad[q];
      y += shfl_xor_d(y, 1);
      y += shfl_xor_d(y, 2);
      y += shfl_xor_d(y, 16);
      const bool pbad = ((__ballot(bad) | rbadm[q]) & pmask) != 0;
      const bool pnf = cl_nf || (__ballot(nfb[q]) & pmask) != 0;
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
int bwd4_ppb() { return kNWB * kPPW; }
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

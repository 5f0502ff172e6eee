// vbhem_fb_bwd12.hip -- the gated schedule's backward-only pass (K2 backward
// recursion, mex.c:915-1015, and K3 termination, mex.c:1020-1080, writing L_elbo)
// for S = 12 cluster states and SB <= 12 base states (C5's shape) with both per-step
// contractions on v_mfma_f64_4x4x4f64: fb_bwd4_kernel's scheme (vbhem_fb_bwd4.hip,
// DESIGN.md 4.4c) on 3 x 3 blocks of 4 x 4 instead of 2 x 2.
//
// A wavefront holds one quad of 4 pairs (4 consecutive bases of one cluster), the 4
// blocks of every MFMA; each pair's 12 x 12 matrices are 3 x 3 blocks of 4 x 4, one
// register per block (P layout: X[i][j] of block (I, J) in lane 16 (i - 4I) + 4 pair +
// (j - 4J)).  Per step
//   G  = exp(V - M)                   M[b] = column maximum over the 12 cluster states
//   Z^T = G^T A'^T                    27 MFMAs: D block (J, I') = sum_K G(K, J)^T A'^T(K, I')
//   sv = M + log Z                    elementwise on Z^T (the log's maxima by ds_bpermute)
//   V  = Ef + sv Ab^T                 27 MFMAs: V(I, J) = Ef + sum_J' sv(I, J') Ab^T(J', J)
// 54 MFMAs per quad-step carry the 2 x 12 x 12 x 12 FMAs of the 4 pairs' contractions;
// the VALU keeps the exp and the log of every element (9 per lane) and the maxima.
// Column maxima: blocks J = 0, 1 as fb_bwd4_kernel (one permlane16 / permlane32 pair
// reduces both, row r then holds block r & 1), block J = 2 by its own full row
// reduction.  The exp / log are fb_bwd4_kernel's: maxima rounded to a
// multiple of ln 2 (the exp table index independent of the maximum), the 8192-interval
// log table with a second-order log1p and the exponent applied to the table's 1/c
// (round 6, vbhem_mfma4.h); the tables take 144 KB of LDS,
// one block per CU, two waves per SIMD, each with its next tile's inputs in flight
// (as fb_bwd4_kernel).  Underflow / range / non-finite handling as fb_bwd4_kernel: a pair
// whose inputs could leave the integer range of the maxima, or whose Z underflowed,
// is flagged to the exact fallback; the per-step underflow test runs only for a
// cluster with an A' entry below 2^-600.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "vbhem_internal.h"
#include "vbhem_mfma4.h"

#ifndef VBHEM_BWD12_WAVES
// waves per SIMD (the register budget): 2, with the next tile's inputs in flight in
// 239 VGPRs.  C5, backward pass per 71 k-base group (profiles/r05u_ab_c5_bwd12_prefetch.txt):
// 3 waves without the prefetch 5.10-5.13 ms (84 bytes of scratch), 3 with it 5.72
// (284 bytes), 2 without it 5.37-5.40, 2 with it 4.93-4.96
#define VBHEM_BWD12_WAVES 2
#endif

namespace vbhem {

namespace {
constexpr int kWaves12 = VBHEM_BWD12_WAVES;
constexpr int kNWB12 = 4 * kWaves12;   // one block per CU (the LDS tables)
using namespace m4;

// this lane row's values of the three column blocks -> the column maxima: w01 (row r:
// block r & 1, as colmax_rows) and w2 (block 2, every row)
__device__ __forceinline__ void colmax3(unsigned x0, unsigned x1, unsigned x2, unsigned &w01,
                                        unsigned &w2) {
  w01 = colmax_rows(x0, x1);
  const auto a = __builtin_amdgcn_permlane16_swap(x2, x2, false, false);
  const unsigned u = max((unsigned)a[0], (unsigned)a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  w2 = max((unsigned)b[0], (unsigned)b[1]);
}

// the full row sum of a double (all 4 lane rows), every row
__device__ __forceinline__ double rowsum_all(double x) {
  const auto al = __builtin_amdgcn_permlane16_swap(lo_u(x), lo_u(x), false, false);
  const auto ah = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x),
                                                   (unsigned)__double2hiint(x), false, false);
  const double u = __hiloint2double((int)ah[0], (int)al[0]) + __hiloint2double((int)ah[1], (int)al[1]);
  const auto bl = __builtin_amdgcn_permlane32_swap(lo_u(u), lo_u(u), false, false);
  const auto bh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(u),
                                                   (unsigned)__double2hiint(u), false, false);
  return __hiloint2double((int)bh[0], (int)bl[0]) + __hiloint2double((int)bh[1], (int)bl[1]);
}
}  // namespace

template <bool O32>
__global__ __launch_bounds__(64 * kNWB12) __attribute__((amdgpu_waves_per_eu(kWaves12)))
void fb_bwd12_kernel(const SplitArgs p) {
  constexpr int S = 12, NB = 3;
  // one array, the exp table first: both tables' LDS offsets fit ds_read's offset field
  __shared__ __attribute__((aligned(16))) double tabs[2048 + 2 * 8192];
  double *const etab = tabs;           // 2^(i/2048 - 1010)
  double *const ltab8 = tabs + 2048;   // {2^1023/c, -log(1/c)} (stage_log8k_x)
  __shared__ double amax[S], lpi[S];
  const int tid = threadIdx.x;
  for (int x = tid; x < 2048; x += 64 * kNWB12) etab[x] = kExpTab4[x] * 0x1p-1010;
  stage_log8k_x(ltab8, tid, 64 * kNWB12);
  const int SB = p.SB, K = p.K, T = p.T;
  // persistent: NB blocks per cluster; XCD-aware when NBk % 8 == 0 (as fb_bwd4_kernel)
  const int bk = blockIdx.x, NBk = (int)gridDim.x / K;
  int j, t0;
  if (NBk % 8 == 0) {
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
  double AT[NB][NB];
#pragma unroll
  for (int k2 = 0; k2 < NB; ++k2)
#pragma unroll
    for (int i2 = 0; i2 < NB; ++i2) AT[k2][i2] = p.Atg[(size_t)j * S * S + (4 * i2 + c) * S + 4 * k2 + r];
  bool cl_nf = false;
#pragma unroll
  for (int x = 0; x < S; ++x) cl_nf |= isnan(amax[x]) || isnan(lpi[x]);
  bool zsafe;
  {
    double am = AT[0][0];
#pragma unroll
    for (int k2 = 0; k2 < NB; ++k2)
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2) am = fmin(am, AT[k2][i2]);
    for (int o = 32; o >= 1; o >>= 1) am = fmin(am, __shfl_xor(am, o, 64));
    zsafe = am >= 0x1p-600;  // NaN: not safe
  }
  zsafe = __builtin_amdgcn_readfirstlane((int)zsafe) != 0;
  // ds_bpermute sources of the log's column maxima (the log's Z^T row 4J + r): blocks
  // 0 / 1 from rows 0 / 1 of colmax3's w01, block 2 from any row of w2
  const int qsrc0 = (0 * 16 + 4 * b + r) << 2, qsrc1 = (1 * 16 + 4 * b + r) << 2;
  const unsigned long long pmask = 0x000F000F000F000Full << (4 * b);
  const double vlim = kVMax / (double)T - 3.0;
  const int ntile = (p.i_end - p.i_begin + 3) / 4;

  // versioned on SB == 12 too (F12: no clamp or zero select in the tile's addresses and
  // operands), as fb_bwd4_kernel
  auto tiles = [&](auto zs_tag, auto f12_tag) {
    constexpr bool ZS = decltype(zs_tag)::value;
    constexpr bool F12 = decltype(f12_tag)::value;
    const int SBk = F12 ? 12 : SB;
    // O32: 32-bit element offsets from the uniform base pointers (launch_bwd12 checks
    // that A, the prior and E stay below 4 GB), as fb_bwd4_kernel
    using off_t_ = typename std::conditional<O32, unsigned, size_t>::type;
    auto ld = [](const double *base, off_t_ x) {
      if constexpr (O32)
        return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + x * 8u);
      else
        return base[x];
    };
    const int tstride = NBk * kNWB12;
    // a tile's global inputs, loaded one tile ahead (as fb_bwd4_kernel): clamped
    // addresses, the selects on the values only when the tile is processed
    struct TileIn {
      double a[NB][NB], e[NB][NB], pr[NB];
    };
    auto load_tile = [&](int tile, TileIn &in) {
      const int i = p.i_begin + tile * 4 + b;
      const int ic = i < p.i_end ? i : p.i_end - 1;
#pragma unroll
      for (int j2 = 0; j2 < NB; ++j2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const int be = 4 * jj + c, bp = 4 * j2 + r;
          in.a[j2][jj] = ld(p.A, ((off_t_)ic * SBk + (be < SBk ? be : SBk - 1)) * SBk + (bp < SBk ? bp : SBk - 1));
        }
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const int be = 4 * jj + c;
          in.e[i2][jj] = ld(p.E, (off_t_)(j * S + 4 * i2 + r) * (off_t_)p.e_ld + (off_t_)(ic - p.i_buf0) * SBk +
                                     (be < SBk ? be : SBk - 1));
        }
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const int be = 4 * jj + c;
        in.pr[jj] = ld(p.prior, (off_t_)ic * SBk + (be < SBk ? be : SBk - 1));
      }
    };
    TileIn cur;
    if (wave * NBk + t0 < ntile) load_tile(wave * NBk + t0, cur);
    for (int tile = wave * NBk + t0; tile < ntile; tile += tstride) {
      const int i0 = p.i_begin + tile * 4;
      const int i = i0 + b;
      TileIn nxt;
      load_tile(min(tile + tstride, ntile - 1), nxt);  // (past the last tile: a repeat)
      double Ef[NB][NB], V[NB][NB], AbT[NB][NB];
      // B operand of V = sv Ab^T + Ef, block (J', J): Ab[4J + c][4J' + r] (zero past SB)
#pragma unroll
      for (int j2 = 0; j2 < NB; ++j2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const int be = 4 * jj + c, bp = 4 * j2 + r;
          AbT[j2][jj] = (be < SBk && bp < SBk) ? cur.a[j2][jj] : 0.0;
        }
      bool nf = false;
      uint64_t bigm = 0;  // the lanes failing the range check
      // row sums of Ab first (P layout: column 4J + c's sum in every lane row), then
      // Ef = E + amax[sigma] rowsum(Ab)[beta] as one fma per element (row sigma = 4I + r);
      // the range check (|E|, |Ef| < vlim, row sums <= 1) as ordered compares into a mask
      double rsj[NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        double x = 0.0;
#pragma unroll
        for (int k2 = 0; k2 < NB; ++k2) x = mfma4(1.0, AbT[k2][jj], x);
        rsj[jj] = x;
        bigm |= gt_mask(x, 1.0 + 1e-6);
      }
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2) {
        const double amr = amax[4 * i2 + r];
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const double e = cur.e[i2][jj];
          V[i2][jj] = e;
          const double ef = fma(amr, rsj[jj], e);
          Ef[i2][jj] = ef;
          bigm |= ge_mask(fabs(e), vlim) | ge_mask(fabs(ef), vlim);
          nf |= !isfinite(ef);
        }
      }
      const bool rbad = lane_in(bigm);
      int zmin = 0x7fffffff;

      // ---- K2: backward recursion, t = T-1 .. 1 ----
      for (int t = T - 1; t >= 1; --t) {
        constexpr int NE = NB * NB;  // elements per lane, (I, J) flattened
        double sf[NE], tv[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) sf[x] = red_s(V[x / NB][x % NB]);
        // the exp table values need no maximum: their reads go out first
#pragma unroll
        for (int x = 0; x < NE; ++x) tv[x] = etab_at(etab, sf[x]);
        unsigned xm[NB];
#pragma unroll
        for (int jj = 0; jj < NB; ++jj)
          xm[jj] = max(max(lo_u(sf[0 * NB + jj]), lo_u(sf[1 * NB + jj])), lo_u(sf[2 * NB + jj]));
        unsigned w01, w2;
        colmax3(xm[0], xm[1], xm[2], w01, w2);
        w01 >>= 11;
        w2 >>= 11;
        const int wq01 = (int)w01 - (1 << 20) - 1023, wq2 = (int)w2 - (1 << 20) - 1023;
        int mq[NB];
        mq[0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq01);
        mq[1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq01);
        mq[2] = __builtin_amdgcn_ds_bpermute(qsrc0, wq2);  // every row holds block 2
        unsigned wph[NB];
        split_rows(w01 - 1010u, wph[0], wph[1]);
        wph[2] = w2 - 1010u;
        double G[NB][NB];
        {
          double vv[NE], gg[NE];
          unsigned wpf[NE];
#pragma unroll
          for (int x = 0; x < NE; ++x) {
            vv[x] = V[x / NB][x % NB];
            wpf[x] = wph[x % NB];
          }
          exp_d_n<NE>(gg, vv, sf, tv, wpf);
#pragma unroll
          for (int x = 0; x < NE; ++x) G[x / NB][x % NB] = gg[x];
        }
        // Z^T block (J, I') = sum_K G^T(J, K) A'^T(K, I'); G^T(J, K) is V's block (K, J)
        double Z[NB][NB];
#pragma unroll
        for (int jj = 0; jj < NB; ++jj)
#pragma unroll
          for (int i2 = 0; i2 < NB; ++i2) Z[jj][i2] = mfma4(G[0][jj], AT[0][i2], 0.0);
#pragma unroll
        for (int k2 = 1; k2 < NB; ++k2)
#pragma unroll
          for (int jj = 0; jj < NB; ++jj)
#pragma unroll
            for (int i2 = 0; i2 < NB; ++i2) Z[jj][i2] = mfma4(G[k2][jj], AT[k2][i2], Z[jj][i2]);
        double sv[NB][NB];
        {
          double zf[NE], yf[NE];
          int wqf[NE];
#pragma unroll
          for (int x = 0; x < NE; ++x) {
            zf[x] = Z[x / NB][x % NB];
            wqf[x] = mq[x / NB];   // Z^T block (J, I'): row 4J + r, column block J's maximum
          }
          if constexpr (!ZS) {
#pragma unroll
            for (int x = 0; x < NE; ++x) zmin = min(zmin, __double2hiint(zf[x]));
          }
          log_x_n<NE, true>(yf, zf, wqf, ltab8);
#pragma unroll
          for (int x = 0; x < NE; ++x) sv[x / NB][x % NB] = yf[x];
        }
        // V block (I, J) = Ef + sum_J' sv(I, J') Ab^T(J', J); sv(I, J') is Z^T's block (J', I)
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
          for (int jj = 0; jj < NB; ++jj) V[i2][jj] = mfma4(sv[0][i2], AbT[0][jj], Ef[i2][jj]);
#pragma unroll
        for (int j2 = 1; j2 < NB; ++j2)
#pragma unroll
          for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
            for (int jj = 0; jj < NB; ++jj) V[i2][jj] = mfma4(sv[j2][i2], AbT[j2][jj], V[i2][jj]);
      }

      // ---- K3: termination, L_elbo = sum_beta prior_beta log sum_sigma exp(lpi + E + L) ----
      {
        double W[NB][NB], sf[NB * NB];
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
          for (int jj = 0; jj < NB; ++jj) {
            // (a state of zero initial probability: lpi = -inf, kept in the integer range)
            W[i2][jj] = fmax(lpi[4 * i2 + r] + V[i2][jj], -7.2e5);
            sf[i2 * NB + jj] = red_s(W[i2][jj]);
          }
        // maxima of all three column blocks in every row (full row reductions; the
        // old-style maxima: M = m ln2/2048, kk = (e << 11) + m - 1023 * 2048)
        unsigned wc[NB];
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const unsigned x = max(max(lo_u(sf[jj]), lo_u(sf[NB + jj])), lo_u(sf[2 * NB + jj]));
          const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
          const unsigned u = max((unsigned)a[0], (unsigned)a[1]);
          const auto bb = __builtin_amdgcn_permlane32_swap(u, u, false, false);
          wc[jj] = max((unsigned)bb[0], (unsigned)bb[1]);
        }
        double ef[NB * NB];
        {
          double wf[NB * NB];
          unsigned wpf[NB * NB];
#pragma unroll
          for (int x = 0; x < NB * NB; ++x) {
            wf[x] = W[x / NB][x % NB];
            wpf[x] = wc[x % NB] - kBias;
          }
          exp_m_n<NB * NB>(ef, wf, sf, wpf, etab);
        }
        double y = 0.0;
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          const double zs = rowsum_all(ef[jj] + ef[NB + jj] + ef[2 * NB + jj]);
          double lse1[1];
          const double zsf[1] = {zs};
          const int wqf[1] = {(int)(wc[jj] + kWq0)};
          log_x_n<1, false>(lse1, zsf, wqf, ltab8);
          const int be = 4 * jj + c;
          const double pr = be < SBk ? cur.pr[jj] : 0.0;
          y += pr * lse1[0];
        }
        const bool bad = zmin < kZMinHi || !isfinite(y) || rbad;
        y += shfl_xor_d(y, 1);
        y += shfl_xor_d(y, 2);
        const bool pbad = (__ballot(bad) & pmask) != 0;
        const bool pnf = cl_nf || (__ballot(nf) & pmask) != 0;
        if (lane == 4 * b && i < p.i_end) {   // row 0, c = 0: the quad's pair b
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
  if (SB == 12) {
    if (zsafe) tiles(std::true_type{}, std::true_type{});
    else tiles(std::false_type{}, std::true_type{});
  } else {
    if (zsafe) tiles(std::true_type{}, std::false_type{});
    else tiles(std::false_type{}, std::false_type{});
  }
}

// ---------------------------------------------------------------------------
bool bwd12_supported(int S, int SB) { return S == 12 && SB >= 1 && SB <= 12; }
int bwd12_ppb() { return kNWB12 * 4; }
int bwd12_resident_blocks() {
  return resident_per_cu(reinterpret_cast<const void *>(&fb_bwd12_kernel<true>), 64 * kNWB12, 0);
}

// the O32 version when every byte offset of A, the prior and E fits 32 bits
bool bwd12_o32(const SplitArgs &a) {
  const unsigned long long lim = 0xffffffffull / 8;
  return (unsigned long long)a.i_end * a.SB * a.SB < lim &&
         (unsigned long long)a.K * a.S * (unsigned long long)a.e_ld < lim;
}

hipError_t launch_bwd12(const SplitArgs &a, unsigned grid, hipStream_t st, hipEvent_t t0,
                        hipEvent_t t1) {
  if (!bwd12_supported(a.S, a.SB) || !a.Atg) return hipErrorInvalidValue;
  if (t0)  // timing events recorded by the dispatch itself (the bench's roofline)
    hipExtLaunchKernelGGL(bwd12_o32(a) ? &fb_bwd12_kernel<true> : &fb_bwd12_kernel<false>, dim3(grid),
                          dim3(64 * kNWB12), 0, st, t0, t1, 0, a);
  else
    hipLaunchKernelGGL(bwd12_o32(a) ? &fb_bwd12_kernel<true> : &fb_bwd12_kernel<false>, dim3(grid),
                       dim3(64 * kNWB12), 0, st, a);
  return hipGetLastError();
}

}  // namespace vbhem

// vbhem_fb_list12.hip -- the gated schedule's second pass (both sweeps, K2-K4 of
// mex.c:915-1298, for the pairs of the gate lists) for S = 12 cluster states, SB <= 12
// and T = 10 (C5's shape), every contraction on v_mfma_f64_4x4x4f64: fb_list4_kernel's
// scheme (vbhem_fb_list4.hip) on 3 x 3 blocks of 4 x 4, with
// fb_bwd12_kernel's backward step (vbhem_fb_bwd12.hip).
//
// One wavefront takes a quad: 4 consecutive entries of one cluster's gate list (4
// bases, the 4 MFMA blocks); a lane holds 9 elements (3 x 3 blocks) of each 12 x 12
// per-pair matrix in the P layout of vbhem_mfma4.h.  Per quad:
//   backward  G = exp(V - M), Z^T = G^T A'^T (27 MFMAs), sv = M + log Z,
//             V = Ef + sv Ab^T (27 MFMAs); G_t of every step is kept for the forward
//             sweep (the lattice: T - 1 slices of 9 doubles per lane, 162 registers);
//   K3        nu_1 = prior exp(lpi + V - logsumexp_sigma), sum_nu_1 = sum_beta nu_1;
//   forward   beta-first, as fb_list4_kernel:
//               f^T = Ab^T nu^T, Z^T = G^T A'^T (recomputed), g^T = f^T / Z^T,
//               H += g G^T, Qm^T = g^T A', nu^T = G^T o Qm^T, sum_t nu^T += nu^T
//             -- 108 MFMAs per quad and step, two per-pair transposes (ds_bpermute);
//   outputs   sum_nu_1 [S], sum_t_nu [S][SB], sum_xi = A' o H [S][S] per pair.
// The lattice lives in registers, so a wavefront needs ~400 of them: one wave per SIMD
// (4-wave blocks, one per CU), the registers past 256 in the accumulation file.  The
// fallback flags are fb_bwd12_kernel's (underflow of Z, |V| range, non-finite inputs);
// a flagged pair is recomputed by the exact kernel after the pass.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "vbhem_internal.h"
#include "vbhem_math.h"
#include "vbhem_mfma4.h"


namespace vbhem {

namespace {
using namespace m4;
constexpr int kL12NWB = 4;   // waves per block: one per SIMD, one block per CU
constexpr int kL12T = 10;    // the tau this kernel is built for (C3 - C5)
constexpr int NB = 3;        // 4 x 4 blocks per dimension (S = 12)
constexpr int NE = NB * NB;  // elements per lane and matrix

// row r of the 4 lane rows -> the maximum of every row (both permlane swaps)
__device__ __forceinline__ unsigned rowmax_all(unsigned x) {
  const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  const unsigned u = max((unsigned)a[0], (unsigned)a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return max((unsigned)b[0], (unsigned)b[1]);
}
__device__ __forceinline__ double rowsum_all12(double x) {
  const auto al = __builtin_amdgcn_permlane16_swap(lo_u(x), lo_u(x), false, false);
  const auto ah = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x),
                                                   (unsigned)__double2hiint(x), false, false);
  const double u = __hiloint2double((int)ah[0], (int)al[0]) + __hiloint2double((int)ah[1], (int)al[1]);
  const auto bl = __builtin_amdgcn_permlane32_swap(lo_u(u), lo_u(u), false, false);
  const auto bh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(u),
                                                   (unsigned)__double2hiint(u), false, false);
  return __hiloint2double((int)bh[0], (int)bl[0]) + __hiloint2double((int)bh[1], (int)bl[1]);
}
// per-pair transpose of a P-layout 12 x 12 matrix: blocks (I, J) -> (J, I), lanes
// (r, b, c) <- (c, b, r)
__device__ __forceinline__ void transpose12(const double (&x)[NB][NB], double (&y)[NB][NB], int taddr) {
#pragma unroll
  for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
    for (int jj = 0; jj < NB; ++jj) y[jj][i2] = bperm_d(taddr, x[i2][jj]);
}
}  // namespace

// FAST: SB == 12 (no clamp or zero select in the item's addresses and operands) and
// 32-bit load offsets (A, the prior and E below 4 GB), as fb_list4_kernel<T, FAST>
template <int T, bool FAST>
__global__ __launch_bounds__(64 * kL12NWB) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fb_list12_kernel(const SplitArgs p) {
  constexpr int S = 12;
  // one array, the exp table first (ds_read offsets), as fb_bwd12_kernel
  __shared__ __attribute__((aligned(16))) double tabs[2048 + 2 * 8192];
  double *const etab = tabs;           // 2^(i/2048 - 1010)
  double *const ltab8 = tabs + 2048;   // {1/c, -log(1/c)}
  __shared__ int pre[kList4MaxK + 1];  // first quad item of every cluster
  __shared__ int tots[kList4MaxK];     // the gate lists' lengths
  const int tid = threadIdx.x;
  for (int x = tid; x < 2048; x += 64 * kL12NWB) etab[x] = kExpTab4[x] * 0x1p-1010;
  stage_log8k(ltab8, tid, 64 * kL12NWB);
  const int K = p.K, SB = FAST ? 12 : p.SB;
  using off_t_ = typename std::conditional<FAST, unsigned, size_t>::type;
  auto ld = [](const double *base, off_t_ x) {
    if constexpr (FAST)
      return *reinterpret_cast<const double *>(reinterpret_cast<const char *>(base) + x * 8u);
    else
      return base[x];
  };
  if (tid == 0) {
    int s = 0;
    for (int jj = 0; jj < K; ++jj) {
      const int t = p.list_tot[jj];
      pre[jj] = s;
      tots[jj] = t;
      s += (t + 3) / 4;
    }
    pre[K] = s;
  }
  __syncthreads();
  const int nitem = __builtin_amdgcn_readfirstlane(pre[K]);
  const double vlim = kVMax / (double)T - 3.0;
  const int gw = (int)blockIdx.x * kL12NWB + (tid >> 6), nw = (int)gridDim.x * kL12NWB;
  const int lane = tid & 63;
  const int r = lane >> 4, b = (lane >> 2) & 3, c = lane & 3;
  // ds_bpermute sources of the log's column maxima (Z^T row 4J + r): blocks 0 / 1 from
  // rows 0 / 1 of colmax_rows' result, block 2 from any row of its full reduction
  const int qsrc0 = (4 * b + r) << 2, qsrc1 = (16 + 4 * b + r) << 2;
  const int taddr = (16 * c + 4 * b + r) << 2;
  const unsigned long long pmask = 0x000F000F000F000Full << (4 * b);

  // An item's global inputs (A in both layouts, E, the prior) are loaded during the
  // previous item's forward sweep, into the registers of lattice slices that are dead
  // by then, and its gate-list entries at the previous item's start (as
  // fb_list4_kernel): with one wave per SIMD nothing else hides an item's start-up
  // latency (C5: 0.588 -> 0.523 ms per group, profiles/r05w_ab_c5_list12_prefetch.txt).
  // Clamped addresses; the selects on the values where the item uses them.
  struct ItemIn {
    double ab[NB][NB], af[NB][NB], e[NB][NB], pr[NB];
  };
  auto load_in = [&](int i, int jj, ItemIn &in) {
#pragma unroll
    for (int j2 = 0; j2 < NB; ++j2)
#pragma unroll
      for (int j3 = 0; j3 < NB; ++j3) {
        const int be = 4 * j3 + c, bp = 4 * j2 + r;
        const int bec = be < SB ? be : SB - 1, bpc = bp < SB ? bp : SB - 1;
        in.ab[j2][j3] = ld(p.A, ((off_t_)i * SB + bec) * SB + bpc);
        in.af[j2][j3] = ld(p.A, ((off_t_)i * SB + bpc) * SB + bec);
      }
#pragma unroll
    for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
      for (int j3 = 0; j3 < NB; ++j3) {
        const int be = 4 * j3 + c;
        in.e[i2][j3] = ld(p.E, (off_t_)(jj * S + 4 * i2 + r) * (off_t_)p.e_ld + (off_t_)(i - p.i_buf0) * SB +
                                   (be < SB ? be : SB - 1));
      }
#pragma unroll
    for (int j3 = 0; j3 < NB; ++j3) {
      const int be = 4 * j3 + c;
      in.pr[j3] = ld(p.prior, (off_t_)i * SB + (be < SB ? be : SB - 1));
    }
  };
  // the base of pair b of item it (cluster jj; past the list's end: the quad's first)
  auto base_of = [&](int it, int jj) -> int {
    const int n0 = (it - pre[jj]) * 4;
    const int tot = tots[jj];
    return p.list[(size_t)jj * p.list_cap + (n0 + b < tot ? n0 + b : n0)];
  };
  int js = 0, jsn = 0;
  ItemIn cur;
  int icur = 0;
  if (gw < nitem) {
    while (pre[js + 1] <= gw) ++js;
    jsn = js;
    icur = base_of(gw, __builtin_amdgcn_readfirstlane(js));
    load_in(icur, __builtin_amdgcn_readfirstlane(js), cur);
  }
  for (int it = gw; it < nitem; it += nw) {
    const int j = __builtin_amdgcn_readfirstlane(js);  // (js: advanced to it)
    // the next item (a repeat of this one past the end): its cluster and list entry now
    const int itn = min(it + nw, nitem - 1);
    while (pre[jsn + 1] <= itn) ++jsn;
    const int jn = __builtin_amdgcn_readfirstlane(jsn);
    const int inext = base_of(itn, jn);
    // the cluster's constants, per item (cache hits): A'^T as the B operand of Z^T
    // (block (K, I'): A'[4I' + c][4K + r]), A' in P (A'[4I + r][4I' + c]), amax (rows
    // 4I + c), lpi (rows 4I + r)
    double AT[NB][NB], amQ[NB], lpP[NB];
    bool cl_nf;
    const double *At = p.Atg + (size_t)j * S * S;
    {
      bool nf = false;
#pragma unroll
      for (int x = 0; x < NB; ++x)
#pragma unroll
        for (int y = 0; y < NB; ++y) AT[x][y] = At[(4 * y + c) * S + 4 * x + r];
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2) {
        const double *la = p.logA + ((size_t)j * S + 4 * i2 + r) * S;  // (P rows: the fma below)
        double mx = la[0];
#pragma unroll
        for (int s2 = 1; s2 < S; ++s2) mx = fmax(mx, la[s2]);
        amQ[i2] = mx;
        lpP[i2] = p.logPi[(size_t)j * S + 4 * i2 + r];
        nf |= isnan(mx) || isnan(lpP[i2]);
      }
      cl_nf = __ballot(nf) != 0;
    }
    const int n0 = (it - pre[j]) * 4;
    const int tot = tots[j];
    const bool act = n0 + b < tot;
    const int i = icur;
    const size_t lp = (size_t)(i - p.i_buf0) * K + j;

    // ---- per-pair inputs: Ab^T as the backward's B operand, E, Ef ----
    double AbT[NB][NB], Ef[NB][NB], V[NB][NB];
#pragma unroll
    for (int j2 = 0; j2 < NB; ++j2)
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const int be = 4 * jj + c, bp = 4 * j2 + r;
        AbT[j2][jj] = (be < SB && bp < SB) ? cur.ab[j2][jj] : 0.0;
      }
    bool nfp = false;
    uint64_t bigm = 0;  // the lanes failing the range check (ordered compares into a mask)
    // Ef = E + amax[sigma] rowsum(Ab)[beta]: one fma per element from the row sums
    // (as fb_bwd12_kernel; amQ holds the P rows 4I + r here)
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
    for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const double e = cur.e[i2][jj];
        V[i2][jj] = e;
        const double ef = fma(amQ[i2], rsj[jj], e);
        Ef[i2][jj] = ef;
        bigm |= ge_mask(fabs(e), vlim) | ge_mask(fabs(ef), vlim);
        nfp |= !isfinite(ef);
      }
    const bool rbad = lane_in(bigm);
    int zmin = 0x7fffffff;

    // ---- K2: backward recursion (fb_bwd12_kernel's step), G_t kept for the forward ----
    // (the log keeps log_q_n's form on the unscaled table: with fb_bwd12_kernel's
    // log_x_n this kernel, at one wave per SIMD and 512 registers, spilled 92 bytes)
    double lat[T][NB][NB];
#pragma unroll
    for (int t = T - 1; t >= 1; --t) {
      double sf[NE], tv[NE];
#pragma unroll
      for (int x = 0; x < NE; ++x) sf[x] = red_s(V[x / NB][x % NB]);
#pragma unroll
      for (int x = 0; x < NE; ++x) tv[x] = etab_at(etab, sf[x]);
      unsigned xm[NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
        xm[jj] = max(max(lo_u(sf[0 * NB + jj]), lo_u(sf[1 * NB + jj])), lo_u(sf[2 * NB + jj]));
      unsigned w01 = colmax_rows(xm[0], xm[1]) >> 11;
      unsigned w2 = rowmax_all(xm[2]) >> 11;
      const int wq01 = (int)w01 - (1 << 20) - 1023, wq2 = (int)w2 - (1 << 20) - 1023;
      int mq[NB];
      mq[0] = __builtin_amdgcn_ds_bpermute(qsrc0, wq01);
      mq[1] = __builtin_amdgcn_ds_bpermute(qsrc1, wq01);
      mq[2] = __builtin_amdgcn_ds_bpermute(qsrc0, wq2);  // every row holds block 2's
      unsigned wph[NB];
      split_rows(w01 - 1010u, wph[0], wph[1]);
      wph[2] = w2 - 1010u;
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
        for (int x = 0; x < NE; ++x) lat[t][x / NB][x % NB] = gg[x];
      }
      double Z[NB][NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) Z[jj][i2] = mfma4(lat[t][0][jj], AT[0][i2], 0.0);
#pragma unroll
      for (int k2 = 1; k2 < NB; ++k2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj)
#pragma unroll
          for (int i2 = 0; i2 < NB; ++i2) Z[jj][i2] = mfma4(lat[t][k2][jj], AT[k2][i2], Z[jj][i2]);
      double sv[NB][NB];
      {
        double zf[NE], yf[NE];
        int wqf[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) {
          zf[x] = Z[x / NB][x % NB];
          wqf[x] = mq[x / NB];  // Z^T block (J, I'): row 4J + r, column block J's maximum
        }
#pragma unroll
        for (int x = 0; x < NE; ++x) zmin = min(zmin, __double2hiint(zf[x]));
        log_q_n<NE, true>(yf, zf, wqf, ltab8);
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

    // ---- K3: nu_1 = prior exp(lpi + V - logsumexp over sigma), sum_nu_1 ----
    double nu[NB][NB];
    bool bad = zmin < kZMinHi || rbad;
    {
      double W[NB][NB], sf[NE];
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj) {
          // (a state of zero initial probability: lpi = -inf, kept in the integer range)
          W[i2][jj] = fmax(lpP[i2] + V[i2][jj], -7.2e5);
          sf[i2 * NB + jj] = red_s(W[i2][jj]);
        }
      // the maxima of every column block in every row (M = m ln2/2048)
      unsigned wc[NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
        wc[jj] = rowmax_all(max(max(lo_u(sf[jj]), lo_u(sf[NB + jj])), lo_u(sf[2 * NB + jj])));
      double ef[NE];
      {
        double wf[NE];
        unsigned wpf[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) {
          wf[x] = W[x / NB][x % NB];
          wpf[x] = wc[x % NB] - kBias;
        }
        exp_m_n<NE>(ef, wf, sf, wpf, etab);
      }
      double lse[NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const double zsf[1] = {rowsum_all12(ef[jj] + ef[NB + jj] + ef[2 * NB + jj])};
        const int wqf[1] = {(int)(wc[jj] + kWq0)};
        double l1[1];
        log_q_n<1, false>(l1, zsf, wqf, ltab8);
        lse[jj] = l1[0];
        bad |= !isfinite(l1[0]);
      }
      double xf[NE], s2[NE], e2[NE];
      unsigned wp0[NE];
#pragma unroll
      for (int x = 0; x < NE; ++x) {
        xf[x] = fmax(W[x / NB][x % NB] - lse[x % NB], -7.0e5);  // (in the integer range)
        s2[x] = red_s(xf[x]);
        wp0[x] = 2147483648u - kBias;  // m = 0
      }
      exp_m_n<NE>(e2, xf, s2, wp0, etab);
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const int be = 4 * jj + c;
        const double pb = be < SB ? cur.pr[jj] : 0.0;
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) nu[i2][jj] = pb * e2[i2 * NB + jj];
      }
      // sum_nu_1[sigma = 4I + r]: over the column blocks, then the 4 lanes c
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2) {
        double a = nu[i2][0] + nu[i2][1] + nu[i2][2];
        a += shfl_xor_d(a, 1);
        a += shfl_xor_d(a, 2);
        if (act && c == 0) p.nu1[lp * S + 4 * i2 + r] = a;
      }
    }

    // ---- K4: forward recursion, beta-first ----
    double AbF[NB][NB];  // Ab in P (Ab[4J' + r][4J + c]): f^T = Ab^T nu^T
#pragma unroll
    for (int j2 = 0; j2 < NB; ++j2)
#pragma unroll
      for (int jj = 0; jj < NB; ++jj) {
        const int bp = 4 * j2 + r, be = 4 * jj + c;
        AbF[j2][jj] = (be < SB && bp < SB) ? cur.af[j2][jj] : 0.0;
      }
    ItemIn nxt;
    // A' in P (A'[4I + r][4I' + c]), loaded only now: not live across the backward sweep
    double Ap[NB][NB];
#pragma unroll
    for (int x = 0; x < NB; ++x)
#pragma unroll
      for (int y = 0; y < NB; ++y) Ap[x][y] = At[(4 * x + r) * S + 4 * y + c];
    double nuT[NB][NB], tnT[NB][NB], H[NB][NB];
    transpose12(nu, nuT, taddr);
#pragma unroll
    for (int x = 0; x < NB; ++x)
#pragma unroll
      for (int y = 0; y < NB; ++y) {
        tnT[x][y] = nuT[x][y];
        H[x][y] = 0.0;
      }
#pragma unroll
    for (int t = 1; t < T; ++t) {
      // the next item's inputs, into the registers of the lattice slices 1 .. T/2 - 1
      if (t == T / 2) load_in(inext, jn, nxt);
      double Gt[NB][NB];
      transpose12(lat[t], Gt, taddr);
      // f^T block (J, I) = sum_J' Ab(J', J)^T nu^T(J', I); Z^T block (J, I') as the backward's
      double fT[NB][NB], ZT[NB][NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) {
          fT[jj][i2] = mfma4(AbF[0][jj], nuT[0][i2], 0.0);
          ZT[jj][i2] = mfma4(lat[t][0][jj], AT[0][i2], 0.0);
        }
#pragma unroll
      for (int k2 = 1; k2 < NB; ++k2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj)
#pragma unroll
          for (int i2 = 0; i2 < NB; ++i2) {
            fT[jj][i2] = mfma4(AbF[k2][jj], nuT[k2][i2], fT[jj][i2]);
            ZT[jj][i2] = mfma4(lat[t][k2][jj], AT[k2][i2], ZT[jj][i2]);
          }
      double gT[NB][NB];
      {
        double zf[NE], rz[NE];
#pragma unroll
        for (int x = 0; x < NE; ++x) zf[x] = ZT[x / NB][x % NB];
        rcp_pos_n<NE>(rz, zf);
#pragma unroll
        for (int x = 0; x < NE; ++x) gT[x / NB][x % NB] = fT[x / NB][x % NB] * rz[x];
      }
      // H block (I, I') += sum_J gT(J, I)^T G^T(J, I')
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
          for (int i3 = 0; i3 < NB; ++i3) H[i2][i3] = mfma4(gT[jj][i2], Gt[jj][i3], H[i2][i3]);
      double g[NB][NB];
      transpose12(gT, g, taddr);
      // Qm^T block (J, I') = sum_I g(I, J)^T A'(I, I'); nu^T = G^T o Qm^T
      double qm[NB][NB];
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i3 = 0; i3 < NB; ++i3) qm[jj][i3] = mfma4(g[0][jj], Ap[0][i3], 0.0);
#pragma unroll
      for (int i2 = 1; i2 < NB; ++i2)
#pragma unroll
        for (int jj = 0; jj < NB; ++jj)
#pragma unroll
          for (int i3 = 0; i3 < NB; ++i3) qm[jj][i3] = mfma4(g[i2][jj], Ap[i2][i3], qm[jj][i3]);
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i3 = 0; i3 < NB; ++i3) {
          nuT[jj][i3] = Gt[jj][i3] * qm[jj][i3];
          tnT[jj][i3] += nuT[jj][i3];
        }
    }

    wait_vm_prefetch();  // (the next item's inputs: before this item's stores)
    // ---- outputs and fallback flags ----
    const bool pbad = (__ballot(bad) & pmask) != 0;
    const bool pnf = cl_nf || (__ballot(nfp) & pmask) != 0;
    if (act) {
      // sum_t_nu[sigma][beta]: tnT block (J, I) lane (r, b, c) = tn[4I + c][4J + r]
#pragma unroll
      for (int jj = 0; jj < NB; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < NB; ++i2) {
          const int be = 4 * jj + r;
          if (be < SB) p.tnu[(lp * S + 4 * i2 + c) * SB + be] = tnT[jj][i2];
        }
      // sum_xi = A' o H: H block (I, I') lane (r, b, c) = H[4I + r][4I' + c], as Ap
#pragma unroll
      for (int i2 = 0; i2 < NB; ++i2)
#pragma unroll
        for (int i3 = 0; i3 < NB; ++i3) p.xi[(lp * S + 4 * i2 + r) * S + 4 * i3 + c] = Ap[i2][i3] * H[i2][i3];
      if (pbad && !pnf && lane == 4 * b) {
        // underflow or range with finite inputs: the exact kernel recomputes the pair
        const int slot = atomicAdd(p.flag_count, 1);
        atomicAdd(p.flag_count + 1, 1);
        p.flag_list[slot] = (int)((size_t)i * K + j);
      }
    }
    cur = nxt;
    icur = inext;
    js = jsn;
  }
}

// ---------------------------------------------------------------------------
bool list12_supported(int S, int SB, int T, int K) {
  return S == 12 && SB >= 1 && SB <= 12 && T == kL12T && K >= 1 && K <= kList4MaxK;
}
bool list12_fast(const SplitArgs &a) {
  const unsigned long long lim = 0xffffffffull / 8;
  return a.SB == 12 && (unsigned long long)a.i_end * a.SB * a.SB < lim &&
         (unsigned long long)a.K * a.S * (unsigned long long)a.e_ld < lim;
}
int list12_resident_blocks() {
  auto *fn = &fb_list12_kernel<kL12T, true>;
  return resident_per_cu(reinterpret_cast<const void *>(fn), 64 * kL12NWB, 0);
}
hipError_t launch_list12(const SplitArgs &a, unsigned grid, hipStream_t st) {
  if (!list12_supported(a.S, a.SB, a.T, a.K) || !a.Atg || !a.list || !a.list_tot)
    return hipErrorInvalidValue;
  auto *fn = list12_fast(a) ? &fb_list12_kernel<kL12T, true> : &fb_list12_kernel<kL12T, false>;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * kL12NWB), 0, st, a);
  return hipGetLastError();
}

}  // namespace vbhem

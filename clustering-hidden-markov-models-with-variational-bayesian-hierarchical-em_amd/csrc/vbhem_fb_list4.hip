// vbhem_fb_list4.hip -- the gated schedule's second pass (both sweeps, K2-K4 of
// mex.c:915-1298, for the pairs of the gate lists) for S = 8 cluster states, SB <= 8
// and T = 10, with every contraction on the fp64 matrix cores
// (v_mfma_f64_4x4x4f64) in the P / Q layouts of vbhem_mfma4.h.
//
// One wavefront takes a quad: 4 consecutive entries of one cluster's gate list (4
// bases, the 4 MFMA blocks).  Per quad:
//   backward  as fb_bwd4_kernel (G = exp(V - M), Z^T = G^T A'^T, sv = M + log Z,
//             V = Ef + sv Ab^T), keeping G_t of every step in registers (the lattice:
//             T - 1 slices of 4 doubles per lane);
//   K3        nu_1 = prior exp(lpi + V - logsumexp_sigma), sum_nu_1 = sum_beta nu_1;
//   forward   with nu and the other per-step matrices kept transposed (beta-first):
//               f^T = Ab^T nu^T             (nu Ab, the base transitions)
//               Z^T = G^T A'^T              (recomputed: the backward's Z)
//               g^T = f^T / Z^T
//               H  += g G^T                 (sum_xi before the A' factor)
//               Qm^T = g^T A'               (g transposed once per step)
//               nu^T = G^T o Qm^T,  sum_t nu^T += nu^T
//             -- 32 MFMAs per quad and step, two per-pair transposes (G -> G^T,
//             g^T -> g) through ds_bpermute, and a reciprocal;
//   outputs   sum_nu_1 [S], sum_t_nu [S][SB], sum_xi = A' o H [S][S] per pair.
// An item's inputs are loaded during the previous item's forward sweep (C4 list pass
// 0.240 -> 0.206 ms, profiles/r05v_ab_c4_list4_prefetch.txt).
// The fallback flags are fb_bwd4_kernel's (underflow of Z, |V| range, non-finite
// inputs); a flagged pair is recomputed by the wave itself after its item loop
// (xinline: queued in LDS; no fb_exact_kernel launch after the pass) or by the exact
// kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "vbhem_exact.h"
#include "vbhem_internal.h"
#include "vbhem_math.h"
#include "vbhem_mfma4.h"

// (The backward half keeps the round-3 step on 32 KB of tables -- 2^(j/2048) and the
// 1024-interval log -- two 4-wave blocks per CU: fb_bwd4_kernel's larger-table step
// measured no gain here, 0.242 vs 0.244 ms at C4 (profiles/r04e_ab_l4r4_c4.txt), since
// the forward sweep sets this kernel's time.)

namespace vbhem {

namespace {
using namespace m4;
constexpr int kL4Waves = 2;   // waves per SIMD (the lattice is 72 VGPRs)
constexpr int kL4NWB = 4;    // waves per block
constexpr int kL4T = 10;      // the tau this kernel is built for (C3 - C5)
}  // namespace
constexpr int kL4XQ = 1024;   // flagged pairs queued per wave (xinline; list4_xq_fits)
namespace {
}  // namespace

// FAST: SB == 8 (no clamp or zero select in the item's addresses and operands) and
// 32-bit load offsets (A, the prior and E below 4 GB), as fb_bwd4_kernel<O32>
template <int T, bool FAST>
__global__ __launch_bounds__(64 * kL4NWB) __attribute__((amdgpu_waves_per_eu(kL4Waves)))
void fb_list4_kernel(const SplitArgs p) {
  constexpr int S = 8;
  __shared__ __attribute__((aligned(16))) double etab[2048];
  __shared__ __attribute__((aligned(16))) double ltab[2 * 1024];
  __shared__ int pre[kList4MaxK + 1];  // first quad item of every cluster
  __shared__ int tots[kList4MaxK];     // the gate lists' lengths
  __shared__ int xq[kL4NWB * kL4XQ];   // per wave: its flagged pairs (xinline)
  const int tid = threadIdx.x;
  stage_tables(etab, ltab, tid, 64 * kL4NWB);
  const int K = p.K, SB = FAST ? 8 : p.SB;
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
  const int gw = (int)blockIdx.x * kL4NWB + (tid >> 6), nw = (int)gridDim.x * kL4NWB;

  // An item's global inputs (A in both layouts, E, the prior) are loaded during the
  // previous item's forward sweep, once its first lattice slices are dead (no extra
  // registers), and the item's gate-list entries at the previous item's start: an
  // item starts with its inputs in registers instead of two dependent memory
  // latencies (list entry, then inputs).  Clamped addresses; the selects on the loaded
  // values only where the item uses them.
  struct ItemIn {
    double ab[2][2], e[2][2], pr[2], af[2][2];
  };
  auto load_in = [&](int i, int jj, int r_, int c_, ItemIn &in) {
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
      for (int j3 = 0; j3 < 2; ++j3) {
        const int be = 4 * j3 + c_, bp = 4 * j2 + r_;
        const int bec = be < SB ? be : SB - 1, bpc = bp < SB ? bp : SB - 1;
        in.ab[j2][j3] = ld(p.A, ((off_t_)i * SB + bec) * SB + bpc);
        in.af[j2][j3] = ld(p.A, ((off_t_)i * SB + bpc) * SB + bec);
      }
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j3 = 0; j3 < 2; ++j3) {
        const int be = 4 * j3 + c_;
        in.e[i2][j3] = ld(p.E, (off_t_)(jj * S + 4 * i2 + r_) * (off_t_)p.e_ld + (off_t_)(i - p.i_buf0) * SB +
                                   (be < SB ? be : SB - 1));
      }
#pragma unroll
    for (int j3 = 0; j3 < 2; ++j3) {
      const int be = 4 * j3 + c_;
      in.pr[j3] = ld(p.prior, (off_t_)i * SB + (be < SB ? be : SB - 1));
    }
  };
  // the base of pair b of item it (cluster jj; past the list's end: the quad's first)
  auto base_of = [&](int it, int jj, int b_) -> int {
    const int n0 = (it - pre[jj]) * 4;
    const int tot = tots[jj];
    return p.list[(size_t)jj * p.list_cap + (n0 + b_ < tot ? n0 + b_ : n0)];
  };
  int js = 0, jsn = 0, nq = 0;
  ItemIn cur;
  int icur = 0;
  if (gw < nitem) {
    const int lane = tid & 63;
    while (pre[js + 1] <= gw) ++js;
    jsn = js;
    icur = base_of(gw, __builtin_amdgcn_readfirstlane(js), (lane >> 2) & 3);
    load_in(icur, __builtin_amdgcn_readfirstlane(js), lane >> 4, lane & 3, cur);
  }
  for (int it = gw; it < nitem; it += nw) {
    // lane geometry recomputed per item from an opaque copy of the thread id, so that
    // no lane-invariant address is hoisted out of the item loop (such live ranges
    // spilled to scratch at 256 VGPRs)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int lane = tq & 63;
    const int r = lane >> 4, b = (lane >> 2) & 3, c = lane & 3;
    const int qsrc0 = (4 * b + r) << 2, qsrc1 = (16 + 4 * b + r) << 2;
    const int taddr = (16 * c + 4 * b + r) << 2;
    const unsigned long long pmask = 0x000F000F000F000Full << (4 * b);
    const int j = __builtin_amdgcn_readfirstlane(js);  // (js: advanced to it)
    // the next item (a repeat of this one past the end): its cluster and list entry now
    const int itn = min(it + nw, nitem - 1);
    while (pre[jsn + 1] <= itn) ++jsn;
    const int jn = __builtin_amdgcn_readfirstlane(jsn);
    const int inext = base_of(itn, jn, b);
    // the cluster's constants, loaded per item (cache hits; holding them across items
    // spilled 17 values to scratch): A'^T as the B operand of Z^T (block (K, I'):
    // A'[4I' + c][4K + r]), A' in P (A'[4I + r][4I' + c]), amax (rows 4I + c), lpi
    double AT[2][2], Ap[2][2], amQ[2], lpP[2];
    bool cl_nf;
    {
      const double *At = p.Atg + (size_t)j * S * S;
      bool nf = false;
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          AT[x][y] = At[(4 * y + c) * S + 4 * x + r];
          Ap[x][y] = At[(4 * x + r) * S + 4 * y + c];
        }
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
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
    double AbT[2][2], Ef[2][2], V[2][2];
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int be = 4 * jj + c, bp = 4 * j2 + r;
        AbT[j2][jj] = (be < SB && bp < SB) ? cur.ab[j2][jj] : 0.0;
      }
    bool nfp = false;
    uint64_t bigm = 0;  // the lanes failing the range check (ordered compares into a mask)
    // Ef = E + amax[sigma] rowsum(Ab)[beta]: one fma per element from the row sums
    // (as fb_bwd4_kernel; amQ holds the P rows 4I + r here)
    double rsj[2];
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) rsj[jj] = mfma4(1.0, AbT[1][jj], mfma4(1.0, AbT[0][jj], 0.0));
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const double e = cur.e[i2][jj];
        V[i2][jj] = e;
        Ef[i2][jj] = fma(amQ[i2], rsj[jj], e);
        bigm |= ge_mask(fabs(e), vlim) | ge_mask(fabs(Ef[i2][jj]), vlim);
        nfp |= !isfinite(Ef[i2][jj]);
      }
    bigm |= gt_mask(rsj[0], 1.0 + 1e-6) | gt_mask(rsj[1], 1.0 + 1e-6);
    const bool rbad = lane_in(bigm);
    int zmin = 0x7fffffff;

    // ---- K2: backward recursion (fb_bwd4_kernel's round-3 step), G_t kept for the forward ----
    double lat[T][2][2];
#pragma unroll
    for (int t = T - 1; t >= 1; --t) {
      double s[2][2];
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) s[i2][jj] = red_s(V[i2][jj]);
      const unsigned w = colmax_rows(max(lo_u(s[0][0]), lo_u(s[1][0])), max(lo_u(s[0][1]), lo_u(s[1][1])));
      const int wq = (int)(w + kWq0);
      const int mq[2] = {__builtin_amdgcn_ds_bpermute(qsrc0, wq), __builtin_amdgcn_ds_bpermute(qsrc1, wq)};
      unsigned wp[2];
      split_rows(w - kBias, wp[0], wp[1]);
      {
        const double vf[4] = {V[0][0], V[0][1], V[1][0], V[1][1]};
        const double sf[4] = {s[0][0], s[0][1], s[1][0], s[1][1]};
        const unsigned wpf[4] = {wp[0], wp[1], wp[0], wp[1]};
        double gf[4];
        exp_m_n<4>(gf, vf, sf, wpf, etab);
        lat[t][0][0] = gf[0]; lat[t][0][1] = gf[1]; lat[t][1][0] = gf[2]; lat[t][1][1] = gf[3];
      }
      double z[4];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2)
          z[2 * jj + i2] = mfma4(lat[t][1][jj], AT[1][i2], mfma4(lat[t][0][jj], AT[0][i2], 0.0));
      zmin = min(zmin, min(min(__double2hiint(z[0]), __double2hiint(z[1])),
                           min(__double2hiint(z[2]), __double2hiint(z[3]))));
      double svf[4];
      {
        const int wqf[4] = {mq[0], mq[0], mq[1], mq[1]};
        log_m_n<4>(svf, z, wqf, ltab);
      }
      // sv(I, J') is Z^T's block (J', I) = svf[2 J' + I]
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          V[i2][jj] = mfma4(svf[2 + i2], AbT[1][jj], mfma4(svf[i2], AbT[0][jj], Ef[i2][jj]));
    }

    // ---- K3: nu_1 = prior exp(lpi + V - logsumexp over sigma), sum_nu_1 ----
    double nu[2][2];
    bool bad;
    {
      double W[2][2], s[2][2];
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          W[i2][jj] = fmax(lpP[i2] + V[i2][jj], -7.2e5);
          s[i2][jj] = red_s(W[i2][jj]);
        }
      const unsigned w = colmax_rows(max(lo_u(s[0][0]), lo_u(s[1][0])), max(lo_u(s[0][1]), lo_u(s[1][1])));
      unsigned wp[2];
      split_rows(w - kBias, wp[0], wp[1]);
      double ev[4];
      {
        const double wf[4] = {W[0][0], W[0][1], W[1][0], W[1][1]};
        const double sf[4] = {s[0][0], s[0][1], s[1][0], s[1][1]};
        const unsigned wpf[4] = {wp[0], wp[1], wp[0], wp[1]};
        exp_m_n<4>(ev, wf, sf, wpf, etab);
      }
      // row r: column 4 (r & 1) + c (w's layout), then both column blocks in every row
      const double zs = colsum_rows(ev[0] + ev[2], ev[1] + ev[3]);
      double lser[1];
      {
        const double zsf[1] = {zs};
        const int wqf[1] = {(int)(w + kWq0)};
        log_m_n<1>(lser, zsf, wqf, ltab);
      }
      bad = zmin < kZMinHi || rbad || !isfinite(lser[0]);
      const auto sl = __builtin_amdgcn_permlane16_swap(lo_u(lser[0]), lo_u(lser[0]), false, false);
      const auto sh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(lser[0]),
                                                       (unsigned)__double2hiint(lser[0]), false, false);
      const double lse[2] = {__hiloint2double((int)sh[0], (int)sl[0]), __hiloint2double((int)sh[1], (int)sl[1])};
      double xf[4], sf[4], ef[4];
      unsigned wpf[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        xf[x] = fmax(W[x / 2][x % 2] - lse[x % 2], -7.0e5);  // (in the integer range)
        sf[x] = red_s(xf[x]);
        wpf[x] = 2147483648u - kBias;  // m = 0
      }
      exp_m_n<4>(ef, xf, sf, wpf, etab);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int be = 4 * jj + c;
        const double pb = be < SB ? cur.pr[jj] : 0.0;
        nu[0][jj] = pb * ef[jj];
        nu[1][jj] = pb * ef[2 + jj];
      }
      // sum_nu_1[sigma = 4I + r]: over the column blocks, then the 4 lanes c
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2) {
        double a = nu[i2][0] + nu[i2][1];
        a += shfl_xor_d(a, 1);
        a += shfl_xor_d(a, 2);
        if (act && c == 0) p.nu1[lp * S + 4 * i2 + r] = a;
      }
    }

    // ---- K4: forward recursion, beta-first ----
    double AbF[2][2];  // Ab in P (Ab[4J' + r][4J + c]): f^T = Ab^T nu^T
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int bp = 4 * j2 + r, be = 4 * jj + c;
        AbF[j2][jj] = (be < SB && bp < SB) ? cur.af[j2][jj] : 0.0;
      }
    ItemIn nxt;
    double nuT[2][2], tnT[2][2], H[2][2];
    transpose8(nu, nuT, taddr);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        tnT[x][y] = nuT[x][y];
        H[x][y] = 0.0;
      }
#pragma unroll
    for (int t = 1; t < T; ++t) {
      // the next item's inputs, into the registers of the lattice slices 1 .. T/2 - 1
      if (t == T / 2) load_in(inext, jn, r, c, nxt);
      double Gt[2][2];
      transpose8(lat[t], Gt, taddr);
      // f^T block (J, I) = sum_J' Ab(J', J)^T nu^T(J', I); Z^T block (J, I') as the backward's
      double fT[2][2], ZT[2][2];
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
          fT[jj][i2] = mfma4(AbF[1][jj], nuT[1][i2], mfma4(AbF[0][jj], nuT[0][i2], 0.0));
          ZT[jj][i2] = mfma4(lat[t][1][jj], AT[1][i2], mfma4(lat[t][0][jj], AT[0][i2], 0.0));
        }
      double gT[2][2];
      {
        const double zf[4] = {ZT[0][0], ZT[0][1], ZT[1][0], ZT[1][1]};
        double rz[4];
        rcp_pos_n<4>(rz, zf);
        gT[0][0] = fT[0][0] * rz[0]; gT[0][1] = fT[0][1] * rz[1];
        gT[1][0] = fT[1][0] * rz[2]; gT[1][1] = fT[1][1] * rz[3];
      }
      // H block (I, I') += sum_J gT(J, I)^T G^T(J, I')
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int i3 = 0; i3 < 2; ++i3) H[i2][i3] = mfma4(gT[1][i2], Gt[1][i3], mfma4(gT[0][i2], Gt[0][i3], H[i2][i3]));
      double g[2][2];
      transpose8(gT, g, taddr);
      // Qm^T block (J, I') = sum_I g(I, J)^T A'(I, I'); nu^T = G^T o Qm^T
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i3 = 0; i3 < 2; ++i3) {
          const double qm = mfma4(g[1][jj], Ap[1][i3], mfma4(g[0][jj], Ap[0][i3], 0.0));
          nuT[jj][i3] = Gt[jj][i3] * qm;
          tnT[jj][i3] += nuT[jj][i3];
        }
    }

    // ---- outputs and fallback flags ----
    const bool pbad = (__ballot(bad) & pmask) != 0;
    const bool pnf = cl_nf || (__ballot(nfp) & pmask) != 0;
    if (act) {
      // sum_t_nu[sigma][beta]: tnT block (J, I) lane (r, b, c) = tn[4I + c][4J + r]
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
          const int be = 4 * jj + r;
          if (be < SB) p.tnu[(lp * S + 4 * i2 + c) * SB + be] = tnT[jj][i2];
        }
      // sum_xi = A' o H: H block (I, I') lane (r, b, c) = H[4I + r][4I' + c], as Ap
#pragma unroll
      for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
        for (int i3 = 0; i3 < 2; ++i3) p.xi[(lp * S + 4 * i2 + r) * S + 4 * i3 + c] = Ap[i2][i3] * H[i2][i3];
      if (pbad && !pnf && lane == 4 * b) {
        // underflow or range with finite inputs: the pair is recomputed by the exact
        // recursion -- below, by this wave (xinline), or by the exact kernel
        atomicAdd(p.flag_count + 1, 1);
        if (!p.xinline) {
          const int slot = atomicAdd(p.flag_count, 1);
          p.flag_list[slot] = (int)((size_t)i * K + j);
        }
      }
    }
    if (p.xinline) {
      // the wave's flagged pairs into its LDS queue (recomputed after the item loop)
      const unsigned long long fm = __ballot(act && pbad && !pnf && lane == 4 * b);
      if (fm) {
        const int l = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(fm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fm, 0u));
        if (fm >> lane & 1) xq[(tid >> 6) * kL4XQ + nq + l] = (int)((size_t)i * K + j);
        nq += __builtin_popcountll(fm);
      }
    }
    cur = nxt;
    icur = inext;
    js = jsn;
  }
  // the exact recursion of the wave's flagged pairs (SplitArgs::xinline: the host
  // inlines when every wave's queue bound fits and the grid has a scratch slot per
  // wave), after the item loop, where none of the loop's registers are live
  if (p.xinline) {
    const int *q = xq + (tid >> 6) * kL4XQ;
    for (int x = 0; x < nq; ++x)
      exact_pair_wave<true>(p.xf, __builtin_amdgcn_readfirstlane(q[x]), p.xscr + (size_t)gw * p.xstride, nullptr);
  }
}

// ---------------------------------------------------------------------------
bool list4_supported(int S, int SB, int T, int K) {
  return S == 8 && SB >= 1 && SB <= 8 && T == kL4T && K >= 1 && K <= kList4MaxK;
}
bool list4_fast(const SplitArgs &a) {
  const unsigned long long lim = 0xffffffffull / 8;
  return a.SB == 8 && (unsigned long long)a.i_end * a.SB * a.SB < lim &&
         (unsigned long long)a.K * a.S * (unsigned long long)a.e_ld < lim;
}
long long list4_inline_waves(const SplitArgs &a, unsigned grid) {
  const long long nw = (long long)grid * kL4NWB;
  const long long items = (long long)a.K * ((a.i_end - a.i_begin + 3) / 4);  // all lists full
  if (nw < 1 || 4 * ((items + nw - 1) / nw) > kL4XQ) return 1ll << 40;
  return nw;
}
int list4_resident_blocks() {
  auto *fn = &fb_list4_kernel<kL4T, true>;
  return resident_per_cu(reinterpret_cast<const void *>(fn), 64 * kL4NWB, 0);
}
hipError_t launch_list4(const SplitArgs &a, unsigned grid, hipStream_t st) {
  if (!list4_supported(a.S, a.SB, a.T, a.K) || !a.Atg || !a.list || !a.list_tot) return hipErrorInvalidValue;
  auto *fn = list4_fast(a) ? &fb_list4_kernel<kL4T, true> : &fb_list4_kernel<kL4T, false>;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * kL4NWB), 0, st, a);
  return hipGetLastError();
}

}  // namespace vbhem

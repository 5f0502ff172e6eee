// vbhem_mfma4.h -- shared device helpers of the MFMA recursion kernels for S = 8
// (fb_bwd4_kernel, vbhem_fb_bwd4.hip; fb_list4_kernel, vbhem_fb_list4.hip): the P / Q
// lane layouts of v_mfma_f64_4x4x4f64, the integer column maxima folded into a
// table exp / log, and the cross-row reductions.  Internal.
//
// Layouts (one quad = 4 pairs = the 4 blocks of every MFMA; lane = 16 r + 4 b + c):
//   P:  X[i][j] of 4x4 block (I, J) in lane 16 (i - 4I) + 4 pair + (j - 4J)
//   Q:  X[i][j] of 4x4 block (I, J) in lane 16 (j - 4J) + 4 pair + (i - 4I)
// mfma4(x, y, c) with x, y read as P-layout blocks returns x^T y + c in P: D block
// (M, N) = sum_K mfma4(X block (K, M), Y block (K, N)) -- it contracts the FIRST
// index of both operands (scripts/ubench_valu.hip probes the lane maps).
#pragma once
#include <hip/hip_runtime.h>

#include "vbhem_log_table.h"

namespace vbhem {
namespace m4 {

// underflow guard of the column sums Z (as fb_bwd2_kernel): Z < 2^-665
constexpr int kZMinHi = 0x16600000;
constexpr double kInvLn2N = 2954.639443740597;        // 2048 / ln 2
constexpr double kLn2N = 0x1.62e42fefa39efp-12;       // ln 2 / 2048 (2048 kLn2N = ln 2 exactly)
constexpr double kShiftU = 0x1.8p52 + 2147483648.0;   // low word of s = n + 2^31
constexpr unsigned kBias = 1010u * 2048u;             // exp: 2^(-1010) folded into the table
constexpr unsigned kWq0 = 0u - 2147483648u - 1023u * 2048u;  // log: m + 2^31 -> m - 1023*2048
constexpr double kVMax = 7.0e5;                       // |V| limit of the integer maxima
namespace {  // one copy per translation unit
alignas(16) __device__ const double kExpTab4[2048] = VBHEM_EXP2048_TABLE_INIT;
alignas(16) __device__ const double kLogTab4[2 * 1024] = VBHEM_LOG12_TABLE_INIT;
alignas(16) __device__ const double kLogTab8k[2 * 8192] = VBHEM_LOG8K_TABLE_INIT;
}  // namespace

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// The per-tile range check (|E|, |Ef| < vlim, Ab row sums <= 1) as one ordered compare
// per element into a wave mask instead of an fmax chain, which the compiler emits with
// NaN canonicalisation (three maxes per pair) and, written as per-lane compares, folds
// back into that chain.  Ordered, so a NaN element is skipped exactly as fmax skips it.
// fb_bwd4_kernel at C4: 1.252-1.264 vs 1.277-1.292 ms (4 interleaved repeats on one box,
// profiles/r05ax_ab_range_cmp.txt); C5 within noise
__device__ __forceinline__ uint64_t ge_mask(double x, double lim) {
  return __builtin_amdgcn_fcmp(x, lim, 3);  // FCMP_OGE
}
__device__ __forceinline__ uint64_t gt_mask(double x, double lim) {
  return __builtin_amdgcn_fcmp(x, lim, 2);  // FCMP_OGT
}
__device__ __forceinline__ bool lane_in(uint64_t m) { return (m >> __lane_id()) & 1; }

// s_waitcnt vmcnt(0) alone (expcnt 7, lgkmcnt 15 on gfx9), issued where the only vector
// memory operations in flight are a prefetch that has had most of an item to land: the
// compiler's own wait before the prefetched registers are copied would otherwise come
// after the item's output stores and wait for those as well (they count in vmcnt, and
// the stores sit behind lane branches, so the compiler cannot count past them).
// fb_list12_kernel (one wave per SIMD): 0.522 -> 0.512 ms per C5 group; in
// fb_list4_kernel it measured 0.206 -> 0.215 ms and in the backward kernels no change
// (profiles/r05z_ab_*), so only there
__device__ __forceinline__ void wait_vm_prefetch() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// s = V 2048/ln2 + 1.5 2^52 + 2^31: n + 2^31 in the low word (exact for |V| < 7.3e5)
__device__ __forceinline__ double red_s(double v) { return fma(v, kInvLn2N, kShiftU); }
__device__ __forceinline__ unsigned lo_u(double x) { return (unsigned)__double2loint(x); }

// exp(V - m ln2/2048) for wp = m + 2^31 - kBias, N elements stage by stage (the
// chains interleave: the kernel's latency is hidden by ILP, not by more waves):
// d = max(0, n - m + kBias) (the clamp sends anything below exp(-700) to
// ~exp(-700)); 2^(d/2048 - 1010) from the table (scaled by 2^-1010) and the
// exponent add, exp(r) as a quadratic, |r| <= ln2/4096
template <int N>
__device__ __forceinline__ void exp_m_n(double (&g)[N], const double (&v)[N], const double (&s)[N],
                                        const unsigned (&wp)[N], const double *etab) {
  double r[N], t[N];
  unsigned d[N];
#pragma unroll
  for (int x = 0; x < N; ++x) {
    d[x] = __builtin_elementwise_sub_sat(lo_u(s[x]), wp[x]);
    t[x] = *reinterpret_cast<const double *>(
        __builtin_assume_aligned(reinterpret_cast<const char *>(etab) + ((d[x] << 3) & 0x3ff8u), 8));
  }
#pragma unroll
  for (int x = 0; x < N; ++x) r[x] = fma(-(s[x] - kShiftU), kLn2N, v[x]);
#pragma unroll
  for (int x = 0; x < N; ++x) {
    // exp(r) - 1 to second order: |r| <= ln2/4096, the dropped r^3/6 <= 8.1e-13
    // relative -- an absolute 8e-13 in log Z per step, far below the recursion's
    // 1e-10 (pairs) and 1e-5 (ELBO) tolerances; one fp64 operation less than cubic
    const double pp = fma(0.5 * r[x], r[x], r[x]);
    const double m = fma(t[x], pp, t[x]);
    // hi(m) + (d >> 11) << 20 as shift + shift-add: the shifted value is laundered
    // through an empty asm so the combiner cannot merge the two shifts into a
    // shift-and-mask (three ops).  No instruction is written in asm here: the
    // compiler's hazard recognizer does not see operands of inline asm, and a VALU
    // read of an MFMA result needs wait states it would not insert.
    unsigned e = d[x] >> 11;
    asm("" : "+v"(e));
    g[x] = __hiloint2double((int)((e << 20) + (unsigned)__double2hiint(m)), __double2loint(m));
  }
}

// log(Z) + m ln2/2048 for wq = m - 1023*2048 (int32), N elements stage by stage:
// Z = 2^e zz, zz in [1, 2), 1024 intervals {1/(2c), -log(1/c)}, log1p(r) to r^3 in
// s = r/2; (e 2048 + m) ln2/2048 is one fma against the table constant (the
// integer sum is exact)
template <int N>
__device__ __forceinline__ void log_m_n(double (&y)[N], const double (&z)[N], const int (&wq)[N],
                                        const double *ltab) {
  double zz[N], ic[N], w[N];
  // exponent word of 1.0 in a register the combiner cannot see through: the
  // mantissa insert below becomes one v_bfi_b32
  unsigned one_hi = 0x3ff00000u;
  asm("" : "+v"(one_hi));
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const unsigned hi = (unsigned)__double2hiint(z[x]);
    // zz = mantissa with exponent 0, kk = (hi >> 20) 2048 + wq (shift + shift-add)
    const unsigned zh = (hi & 0x000fffffu) | (one_hi & 0xfff00000u);
    unsigned ex = hi >> 20;
    asm("" : "+v"(ex));
    const int kk = (int)(ex << 11) + wq[x];
    zz[x] = __hiloint2double((int)zh, __double2loint(z[x]));
    const double2 e = *reinterpret_cast<const double2 *>(
        __builtin_assume_aligned(reinterpret_cast<const char *>(ltab) + ((hi >> 6) & 0x3ff0u), 16));
    ic[x] = e.x;
    w[x] = fma((double)kk, kLn2N, e.y);
  }
#pragma unroll
  for (int x = 0; x < N; ++x) {
    // log1p(r) = 2 (s - s^2 + 4/3 s^3) with s = r/2, |s| <= 2^-12: the dropped -4 s^4
    // is <= 1.4e-14 absolute
    const double sh = fma(zz[x], ic[x], -0.5);
    const double s2 = sh * sh;
    const double q = fma(sh, 4.0 / 3.0, -1.0);
    y[x] = fma(fma(q, s2, sh), 2.0, w[x]);
  }
}

// column maxima of a quad's two column blocks: x0 / x1 = this lane row's maximum of
// block J = 0 / 1; the result's lane row r holds block J = r & 1 (over all 4 rows)
__device__ __forceinline__ unsigned colmax_rows(unsigned x0, unsigned x1) {
  const auto a = __builtin_amdgcn_permlane16_swap(x0, x1, false, false);
  const unsigned u = max((unsigned)a[0], (unsigned)a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return max((unsigned)b[0], (unsigned)b[1]);
}
// row r holds block r & 1 -> block 0 / block 1 in every row
__device__ __forceinline__ void split_rows(unsigned w, unsigned &w0, unsigned &w1) {
  const auto a = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  w0 = a[0];
  w1 = a[1];
}
// the same row reduction as sums of doubles (the termination's column sums)
__device__ __forceinline__ double colsum_rows(double x0, double x1) {
  const auto al = __builtin_amdgcn_permlane16_swap(lo_u(x0), lo_u(x1), false, false);
  const auto ah = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(x0),
                                                   (unsigned)__double2hiint(x1), false, false);
  const double u = __hiloint2double((int)ah[0], (int)al[0]) + __hiloint2double((int)ah[1], (int)al[1]);
  const auto bl = __builtin_amdgcn_permlane32_swap(lo_u(u), lo_u(u), false, false);
  const auto bh = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(u),
                                                   (unsigned)__double2hiint(u), false, false);
  return __hiloint2double((int)bh[0], (int)bl[0]) + __hiloint2double((int)bh[1], (int)bl[1]);
}

__device__ __forceinline__ double shfl_xor_d(double x, int m) {
  const int l = (int)__lane_id() ^ m;
  const int lo = __builtin_amdgcn_ds_bpermute(l << 2, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(l << 2, __double2hiint(x));
  return __hiloint2double(hi, lo);
}

// the per-pair transpose of a P-layout 8 x 8 matrix (blocks (I, J) -> (J, I), lanes
// (r, b, c) <- (c, b, r)) through the LDS crossbar (ds_bpermute: no LDS memory,
// no VALU); taddr = ((16 c + 4 b + r) << 2) of this lane
__device__ __forceinline__ double bperm_d(int taddr, double x) {
  const int lo = __builtin_amdgcn_ds_bpermute(taddr, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(taddr, __double2hiint(x));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void transpose8(const double (&x)[2][2], double (&y)[2][2], int taddr) {
#pragma unroll
  for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) y[jj][i2] = bperm_d(taddr, x[i2][jj]);
}

// the exp / log tables of exp_m_n / log_m_n in LDS: 2^(i/2048 - 1010) and {1/(2c), -log(1/c)}
__device__ __forceinline__ void stage_tables(double *etab, double *ltab, int tid, int nt) {
  for (int x = tid; x < 2048; x += nt) {
    etab[x] = kExpTab4[x] * 0x1p-1010;
    ltab[x] = kLogTab4[x];
  }
}

// ---- the round-4 step helpers (fb_bwd4_kernel, fb_bwd12_kernel) ----
// the 8192-interval log table, {1/c, -log(1/c)} with c the centre of [1 + k/8192,
// 1 + (k+1)/8192) and 1/c rounded to a double (the table need not hold 1/c exactly:
// log zz = -log(ic) + log1p(zz ic - 1) for any ic), generated with correctly rounded
// logs (scripts/gen_log_table.py) and copied into each block's LDS: 16-byte loads from
// L2 instead of a division and a libm log per entry (computing it took ~6 us of every
// fb_bwd4_kernel launch, profiles/r05ah_ab_shard_cheap_stage.txt)
__device__ __forceinline__ void stage_log8k(double *ltab, int tid, int nt) {
  const double2 *src = reinterpret_cast<const double2 *>(kLogTab8k);
  double2 *dst = reinterpret_cast<double2 *>(ltab);
  // (unrolled: a 4-wave block's 32 copies per thread go out in two batches, not one
  // memory latency after another)
#pragma unroll 16
  for (int k = tid; k < 8192; k += nt) dst[k] = src[k];
}

// log(Z) + M, 8192-interval table, log1p(r) = r - r^2/2 (|r| <= 2^-14): kk = the
// binary exponent of Z plus the maximum's term (integer, exact), then one fma
template <int N, bool DEC>
__device__ __forceinline__ void log_q_n(double (&y)[N], const double (&z)[N], const int (&wq)[N],
                                        const double *ltab) {
  double zz[N], ic[N], w[N];
  unsigned one_hi = 0x3ff00000u;
  asm("" : "+v"(one_hi));
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const unsigned hi = (unsigned)__double2hiint(z[x]);
    const unsigned zh = (hi & 0x000fffffu) | (one_hi & 0xfff00000u);
    unsigned ex = hi >> 20;
    asm("" : "+v"(ex));
    const int kk = DEC ? (int)ex + wq[x] : (int)(ex << 11) + wq[x];
    zz[x] = __hiloint2double((int)zh, __double2loint(z[x]));
    const double2 e = *reinterpret_cast<const double2 *>(
        __builtin_assume_aligned(reinterpret_cast<const char *>(ltab) + ((hi >> 3) & 0x1fff0u), 16));
    ic[x] = e.x;
    w[x] = fma((double)kk, DEC ? 0x1.62e42fefa39efp-1 : kLn2N, e.y);
  }
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const double r = fma(zz[x], ic[x], -1.0);
    const double h = fma(r, -0.5, 1.0);
    y[x] = fma(r, h, w[x]);
  }
}

// ---- round 6 (fb_bwd4_kernel, fb_bwd12_kernel) ----
// The 8192-interval log table with 1/c scaled by 2^1023 (stage_log8k_x): for Z = 2^(ex -
// 1023) zz the remainder r = zz / c - 1 is Z (2^1023/c) 2^-ex - 1, and 2^-ex goes into
// the table value's exponent field by one integer op (v_mad_i32_i24 ex, -2^20, hi), where
// log_q_n inserted 1.0's exponent into Z (a v_bfi_b32 and, as allocated, a v_mov_b32 for
// the low word).  Both scalings are exact, so r is the same bit for bit.  ic 2^1023 is
// finite (c > 1, so 1/c < 1), and ic 2^(1023 - ex) stays normal for every Z the kernels
// accept (2^-665 <= Z <= S; a Z outside that is flagged or non-finite anyway).
__device__ __forceinline__ void stage_log8k_x(double *ltab, int tid, int nt) {
  const double2 *src = reinterpret_cast<const double2 *>(kLogTab8k);
  double2 *dst = reinterpret_cast<double2 *>(ltab);
#pragma unroll 16
  for (int k = tid; k < 8192; k += nt) {
    const double2 v = src[k];
    dst[k] = make_double2(v.x * 0x1p1023, v.y);
  }
}
// log(Z) + M on stage_log8k_x's table: kk = Z's biased exponent + wq (DEC: M a multiple
// of ln 2, wq = k - 1023; otherwise M = m ln2/2048, wq = m - 1023 2048 and kk = ex 2048 + wq)
template <int N, bool DEC>
__device__ __forceinline__ void log_x_n(double (&y)[N], const double (&z)[N], const int (&wq)[N],
                                        const double *ltab) {
  double ic[N], w[N];
  // -2^20 in an SGPR the combiner cannot see: __mul24 by a known power of two would
  // become a shift and a subtraction (two ops, measured 4 % slower); this way it is one
  // v_mad_i32_i24
  int m20 = -1048576;
  asm("" : "+s"(m20));
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const unsigned hi = (unsigned)__double2hiint(z[x]);
    unsigned ex = hi >> 20;
    asm("" : "+v"(ex));
    const int kk = DEC ? (int)ex + wq[x] : (int)(ex << 11) + wq[x];
    const double2 e = *reinterpret_cast<const double2 *>(
        __builtin_assume_aligned(reinterpret_cast<const char *>(ltab) + ((hi >> 3) & 0x1fff0u), 16));
    // ic 2^(1023 - ex): one 24-bit multiply-add on the high word
    const int ich = __mul24((int)ex, m20) + __double2hiint(e.x);
    ic[x] = __hiloint2double(ich, __double2loint(e.x));
    w[x] = fma((double)kk, DEC ? 0x1.62e42fefa39efp-1 : kLn2N, e.y);
  }
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const double r = fma(z[x], ic[x], -1.0);
    const double h = fma(r, -0.5, 1.0);
    y[x] = fma(r, h, w[x]);
  }
}

// exp(V - M) for M = (h - 2^20) ln 2, h = the column maximum of lo(s) >> 11: the table
// index is lo(s) mod 2048 (independent of M), the scale 2^(lo(s) >> 11 - h) clamped
// below at 2^-1010 (wph = h - 1010): table scaled by 2^-1010, exponent added
template <int N>
__device__ __forceinline__ void exp_d_n(double (&g)[N], const double (&v)[N], const double (&s)[N],
                                        const double (&t)[N], const unsigned (&wph)[N]) {
#pragma unroll
  for (int x = 0; x < N; ++x) {
    const double r = fma(-(s[x] - kShiftU), kLn2N, v[x]);
    const double pp = fma(0.5 * r, r, r);
    const double m = fma(t[x], pp, t[x]);
    unsigned e = __builtin_elementwise_sub_sat(lo_u(s[x]) >> 11, wph[x]);
    asm("" : "+v"(e));
    g[x] = __hiloint2double((int)((e << 20) + (unsigned)__double2hiint(m)), __double2loint(m));
  }
}
__device__ __forceinline__ double etab_at(const double *etab, double s) {
  return *reinterpret_cast<const double *>(
      __builtin_assume_aligned(reinterpret_cast<const char *>(etab) + ((lo_u(s) << 3) & 0x3ff8u), 8));
}

}  // namespace m4
}  // namespace vbhem

// vbhem_internal.h -- kernel argument blocks shared by the kernels and the
// C-ABI layer (not part of the public interface; see include/vbhem_estep.h).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

namespace vbhem {

// record `msg` for vbhem_last_error() and return `code` (vbhem_capi.hip)
int set_error(int code, const std::string &msg);

// Host-side launch helpers: the dynamic-LDS attribute, the occupancy query and
// the CU count are per (device, kernel, block, LDS) facts, so they are asked
// once per device and remembered (every fused E-step launches the same kernels
// with the same geometry).  Keyed by the caller's current device: a process that
// drives several GPUs gets each device's own answers.
inline int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return dev;
}
inline hipError_t set_dyn_lds(const void *fn, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void *>, size_t> done;  // largest LDS already allowed
  const auto key = std::make_pair(current_device(), fn);
  std::lock_guard<std::mutex> g(mu);
  auto it = done.find(key);
  if (it != done.end() && it->second >= lds) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) done[key] = lds;
  return e;
}
inline int resident_per_cu(const void *fn, int threads, size_t lds) {
  static std::mutex mu;
  static std::map<std::tuple<int, const void *, int, size_t>, int> memo;
  const auto key = std::make_tuple(current_device(), fn, threads, lds);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
  }
  int n = 0;
  if (set_dyn_lds(fn, lds) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, lds) != hipSuccess || n < 1)
    return 1;  // not remembered: ask again next time
  std::lock_guard<std::mutex> g(mu);
  memo[key] = n;
  return n;
}
inline int device_cus() {
  static std::mutex mu;
  static std::map<int, int> cus;
  const int dev = current_device();
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cus.find(dev);
    if (it != cus.end()) return it->second;
  }
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
    return 256;  // not remembered
  std::lock_guard<std::mutex> g(mu);
  cus[dev] = n;
  return n;
}

constexpr int kCovDiag = 0;
constexpr int kCovFull = 1;

// fb_pairs_kernel / fb_exact_kernel arguments.  All offsets are in doubles
// from the start of dynamic LDS.
struct FbArgs {
  int SB, d, covmode, K, S, T;
  int BI, BJ, NE, RS, AS, ABS, njb;
  int i_begin, i_end, i_buf0;  // bases processed [i_begin, i_end); buffers row 0 = i_buf0
  int np, MS, PS;              // packed-covariance count and LDS strides
  const double *prior, *A, *centres, *covars;
  const double *logA, *logPi, *m, *P, *c;
  double *LL, *nu1, *xi, *tnu;
  int *flag_count, *flag_list;
  int off_At, off_amax, off_lpi, off_Ab, off_pib, off_flag, off_reg;
  int off_k1m, off_k1P, off_k1c, off_k1mu, off_k1C;
  int pair_stride;
  double smooth;  // E /= smooth when != 1 (VHEM sibling, hem_hmm_bwd_fwd_mex.c:848-860)
};

struct EmitArgs {
  int SB, d, covmode, K, S;
  int i_begin, i_end;
  const double *centres, *covars, *tnu;
  double *emit_pr, *emit_mu, *emit_Mu;
};

struct StatsArgs {
  int K, S, SB, SBp, d, covmode, NU;
  int JG;   // clusters per row group (grid.y)
  int NBB;  // bases per batch (MFMA K-dim = NBB*SBp)
  int AST;  // LDS row stride of A = NBB*SBp + 1
  int UST;  // LDS row stride of U = 16*ceil(NU/16)
  int i_begin, i_end, i_buf0, slab_len;
  const double *centres, *covars, *LL, *nu1, *xi, *tnu, *tildeN, *logOmega;
  double *Z;  // [group][K] hat_Z * tilde_N (resp_kernel -> stats_kernel)
  double *hatZ, *slabs;
  // gated-pair lists (sparse path): per-chunk gate counts, per-cluster bases, totals
  int *gate_cnt;   // [nchunk][K]  (resp_kernel)
  int *list;       // [K][list_cap] bases i with Z(i, j) > 1e-8, ascending i
  int *list_tot;   // [K]
  int list_cap;
  int PB;          // pairs per batch of stats_list_kernel
  int assign;      // gated schedule, first group: write the slab entries instead of adding
  int KT, SL;      // batched trials: clusters per trial (K = R * KT) and the per-trial
                   // statistics length; slab = R sections of SL (KT = K, SL = slab_len: one)
  // the emission GEMM's prepared operand for the bases of this call (null: not built);
  // stats_list_u_kernel reads the emission moments from it instead of the covariances
  const double *U, *uz;  // operand, its shift z (d doubles)
  long long u_col0;      // first column of U
  int ukdp;              // k-extent of U (multiple of 4)
  int nzero;             // stats_list_u_kernel with assign: slabs [gridDim.x, nzero) get zeros
  const double *Us;      // the statistics copy of the prepared operand (us_doubles), or null
  int nzero_m;           // stats_list_m_kernel: at most this many parts (slabs) per cluster (0: nzero)
  // the backward pass's exact fallback folded into resp_kernel (the flagged pairs of
  // each block's bases) instead of a launch after the pass (fold != 0; one base group);
  // the gate-list pass's flagged pairs: recomputed by the list kernel itself (fold = 2,
  // SplitArgs::xinline) or an fb_exact_kernel launch from flag_count[3] in
  // launch_stats_list (fold = 1)
  int fold;
  FbArgs fx;                 // the exact recursion's arguments (outputs, flag counter / list)
  double *xscratch;          // its scratch: xslots slots of xstride doubles
  long long xstride;
  int xslots;
};

// fb_split_kernel (one base-state column per LPC lanes; S <= kSplitMaxS, SB <= S).
constexpr int kSplitMaxS = 16;
template <int S>
struct SplitLPC {
#ifdef VBHEM_SPLIT_LPC5   // A/B: lanes per column of the dense / list modes at S = 5
  static constexpr int value = S <= 4 ? 1 : S == 5 ? VBHEM_SPLIT_LPC5 : S <= 8 ? 2 : 4;
#else
  static constexpr int value = S <= 4 ? 1 : S <= 8 ? 2 : 4;
#endif
};
// the backward-only mode's alternative (no H / sum_t_nu registers: wider columns fit)
template <int S>
struct BwdLPC {
  static constexpr int value = S <= 8 ? 1 : 2;
};
template <int S, int LPC>
struct SplitLayout {
  static constexpr int SH = (S + LPC - 1) / LPC;           // rows per lane
  static constexpr int XCS = (LPC * SH + 1) / 2 * 2 + 2;   // slab column stride (even)
  static constexpr int XP = S * XCS + 2;                    // per-pair slab
  static constexpr int HEAD = 2 * S * S + 2 * S;            // At, AtT, amax, lpi
  static constexpr int OFF_X = (HEAD + 1) / 2 * 2;
};
// K1 emission GEMM (vbhem_emission.hip)
// W' / bias' padding of the emission GEMM: k-rows to a multiple of 4 (MFMA k-step),
// rows (j, s) to a multiple of 128 (a chunk of 8 MFMA row tiles)
inline int emission_kdp(int d, int covmode) {
  const int kd = covmode == kCovFull ? d * (d + 1) / 2 + d : 2 * d;
  return (kd + 3) / 4 * 4;
}
inline int emission_ksp(int ks) { return (ks + 127) / 128 * 128; }

struct EmissionArgs {
  int SB, d, covmode, K, S, KD, CB;
  int kdp, ksp;  // padded W' dims: [kdp][ksp], bias' [ksp]
  bool wfull;  // column tiles staged in LDS (d <= 8); else read through L1/L2
  bool wlds;   // W staged in LDS (8-wave blocks); else read through L1/L2 (4-wave blocks)
  int nwave;
  int i_begin, i_end, i_buf0;
  long long e_ld;  // row stride of E = (bases in the buffer) * SB
  const double *centres, *covars, *m, *P, *c;
  double *W, *bias, *shift;  // W' = -W/2 [kdp][ksp], bias' = -bias/2 [ksp], z [d] (emission_prep_kernel)
  double *E;                 // [K*S][(i - i_buf0) * SB + b]  (row stride e_ld)
  double smooth;             // E /= smooth when != 1 (VHEM sibling)
  // prepared-operand GEMM (emission_u_kernel): U in the u_prep layout, its tile 0 at
  // global column u_col0; zfix = the shift U was built with (emission_prep_kernel
  // then uses it for W', bias'), or null (z = mean of the finite cluster means)
  const double *U, *zfix;
  long long u_col0;
  int urc;    // row tiles per LDS chunk of W' (emission_u_kernel), 0: old kernels
  int ukqb;   // register bucket of the U tile (k-steps)
  // per-call side jobs of emission_prep_kernel
  const double *logA;        // [K][S][S]
  double *Atg;               // [K][S][S] A' = exp(logA - rowmax), or null
  int *zero_ints;            // fallback counters zeroed by block 0, or null
  int n_zero;
};
bool plan_emission(EmissionArgs &a, size_t &lds);
// emission_u_kernel's plan: row chunking and LDS; false when the shape needs the
// raw / generic kernels (k-steps > kUMaxKq).  launch_emission takes it when a.U is set.
bool plan_emission_u(EmissionArgs &a, size_t &lds);

// The base-set operand U of the K1 GEMM (vbhem_prepare_base): for column tile ct
// (16 columns (i,b), global column u_col0 + 16 ct + cl) and k-step t, the 64
// doubles of the MFMA B operand in lane order: U[(ct kq + t) 64 + 16 kl + cl] =
// u(e = 4t + kl, col), zero for e >= KD and for columns past the end.  Buffer:
// [kUHead doubles: z (d) | 0][ntile * kq * 64].
constexpr int kUHead = 64;
constexpr int kUMaxKq = 40;
inline long long u_tiles(long long ncols) { return (ncols + 15) / 16; }
inline size_t u_doubles(long long ncols, int d, int covmode) {
  return (size_t)kUHead + (size_t)u_tiles(ncols) * (emission_kdp(d, covmode) / 4) * 64;
}
struct UPrepArgs {
  int N, SB, d, covmode, kdp;
  int i_begin, i_end;         // bases whose columns are built
  long long u_col0;           // global column of tile 0 (a multiple of 16)
  const int *nstates;
  const double *centres, *covars;
  double *U;                  // the buffer (head + tiles)
  const double *z;            // the shift (device), or null: u_shift_kernel computes the
                              // mean of the valid base means of [0, N) into the head first
};
hipError_t launch_u_prep(const UPrepArgs &a, hipStream_t st);
// The statistics copy of the base-set operand (vbhem_prepare_base, right after U in
// the same buffer): per base i an [NUP / 16][SBP][16] block (SBP = SB rounded up to 4,
// NUP = NU rounded up to 16; feature tile, base state, feature within the tile) of the
// statistic features f of every base state b:
// 1 | mu'_a (d) | packed Sigma + mu' mu'^T (as U, off-diagonals Sigma_ab + Sigma_ba +
// 2 mu'_a mu'_b), mu' = mu - z, zero past SB and NU.  stats_list_m_kernel's MFMA B
// operand: a 16-feature tile of four consecutive states is one contiguous 512-byte
// segment (one load per k-slice; with [SBP][NUP] rows it was four 128-byte segments
// in four rows), a base's block is contiguous (the tile order of U splits it over two
// 16-column tiles' half lines).
__host__ __device__ inline int us_sbp(int SB) { return (SB + 3) / 4 * 4; }
__host__ __device__ inline int us_nup(int NU) { return (NU + 15) / 16 * 16; }
__host__ __device__ inline int us_nu(int d, int covmode) { return 1 + d + (covmode == kCovFull ? d * (d + 1) / 2 : d); }
inline size_t us_doubles(long long N, int SB, int d, int covmode) {
  return (size_t)N * us_sbp(SB) * us_nup(us_nu(d, covmode));
}
// builds Us for bases [0, a.N) with the shift in a.U's head (after launch_u_prep)
hipError_t launch_us_build(const UPrepArgs &a, double *Us, hipStream_t st);
hipError_t launch_emission_prep(const EmissionArgs &a, hipStream_t st);
hipError_t launch_emission(const EmissionArgs &a, size_t lds, hipStream_t st);

// fb_split_kernel modes:
//   kFbDense    every pair of [i_begin, i_end) x K: all outputs (K2-K4)
//   kFbBackward every pair: K2 + K3 log-likelihood only (no lattice, no forward sweep)
//   kFbList     the gated pairs list[j * list_cap + n], n < list_tot[j]: K2-K4 outputs
//               except LL (already written by the backward pass)
enum FbMode : int { kFbDense = 0, kFbBackward = 1, kFbList = 2 };

struct SplitArgs {
  int SB, d, covmode, K, S, T, nwb, lpc;
  int mode;  // FbMode
  int i_begin, i_end, i_buf0;
  int off_Y, off_F, off_R;  // LDS layout (doubles), depends on pairs per block
  int off_L;                // kFbList: [K + 1] ints of work-item prefix (after the lattice)
  int off_T;                // kFbBackward: log_tab_n table (kLogTabDoubles, after off_R + 2)
  const double *prior, *A;
  const double *logA, *logPi;
  const double *E;  // emission_kernel output, [K*S][(i - i_buf0) * SB + b], row stride e_ld
  long long e_ld;
  double *LL, *nu1, *xi, *tnu;
  int *flag_count, *flag_list;
  const int *list, *list_tot;  // kFbList: gated bases per cluster (gate_list_kernel)
  int list_cap;
  const double *Atg;           // kFbBackward, LPC 1: [K][S][S] A' (emission_prep_kernel),
                               // then [K][S] room for fb_bwd4_kernel's logA row maxima
  // K1 inside the recursion kernel (eU set; fb_bwd2_kernel and fb_split_kernel's list
  // mode, for a short GEMM inner dimension, kdp <= kK1InKernelMaxKdp): E = bias' + W'^T u
  // per entry from the prepared operand U (u_prep layout, tile 0 at column e_col0,
  // ekdp / 4 k-steps) and emission_prep_kernel's W' [ekdp][eksp], bias' [eksp],
  // instead of reading emission_kernel's E
  const double *eU, *eW, *ebias;
  long long e_col0;
  int ekdp, eksp;
  double esmooth;
  // the gate-list pass's exact fallback inline (xinline; fb_list4_kernel and
  // fb_split_kernel's list mode): a wavefront that flags a pair recomputes it itself
  // (exact_pair_wave, vbhem_exact.h; Theta and the small arrays in the wavefront's
  // scratch slot xscr + wave * xstride, one slot per wavefront of the persistent grid)
  // instead of listing it for an fb_exact_kernel launch after the pass -- at once
  // (fb_split_kernel, kSplitInlineMinS <= S <= kSplitInlineMaxS only) or from a
  // per-wave LDS queue after the item loop (fb_list4_kernel, list4_inline_waves)
  int xinline;
  double *xscr;
  long long xstride;
  FbArgs xf;
  // fb_bwd2_kernel with K1 inside and prep set: emission_prep_kernel's work in the
  // kernel (no launch of its own).  Every block computes its cluster's W' / bias' / A'
  // from the cluster constants with that kernel's arithmetic (em_* below), the first
  // block of each cluster writes them to eW / ebias / Atg for the gate-list pass, and
  // the fallback counters are zeroed in the kernel when the flag head's tag is not
  // ftag_val (kFlagPre)
  int prep;
  const double *pm, *pP, *pc, *pz;  // cluster means [K S][d], precisions, constants [K S], shift [d]
  double *pshift;                   // the shift, copied for the later kernels
  unsigned long long *ftag;
  unsigned long long ftag_val;
};

// emission_prep_kernel's per-row arithmetic, one definition for it and for
// fb_bwd2_kernel's in-kernel preparation (the same bits either way)
constexpr double kLog2PiE = 1.8378770664093454835606594728112353;
__device__ __forceinline__ double em_psym(const double *P, int a, int b, int d) {
  return 0.5 * (P[a * d + b] + P[b * d + a]);
}
// (P_sym m')_a, m' = m - z
__device__ __forceinline__ double em_pm_full(const double *P, const double *mr, const double *zs,
                                             int a, int d) {
  double v = 0.0;
  for (int b = 0; b < d; ++b) v = fma(em_psym(P, a, b, d), mr[b] - zs[b], v);
  return v;
}
// W' entry of packed (a, b) of the full-covariance quadratic term
__device__ __forceinline__ double em_w_full(const double *P, int a, int b, int d) {
  return -0.5 * ((a == b) ? P[a * d + a] : em_psym(P, a, b, d));
}
__device__ __forceinline__ double em_bias(int d, double c, double q) {
  return -0.5 * (d * kLog2PiE + c + q);
}

constexpr int kK1InKernelMaxKdp = 8;
constexpr int kSplitInlineMinS = 4, kSplitInlineMaxS = 6;  // SplitArgs::xinline: list kernels that take it  // d = 2 full / d <= 4 diag: at most 8 fmas per entry

// the kdp <= 8 operand values u_e of one column (i SB + b) of U (zero past kdp)
__device__ __forceinline__ void k1_column(const SplitArgs &p, long long col,
                                          double (&u)[kK1InKernelMaxKdp]) {
  const long long c = col - p.e_col0;
  const double *Ut = p.eU + kUHead + (size_t)(c >> 4) * (p.ekdp / 4) * 64 + (int)(c & 15);
#pragma unroll
  for (int e = 0; e < kK1InKernelMaxKdp; ++e)
    u[e] = e < p.ekdp ? Ut[(e >> 2) * 64 + (e & 3) * 16] : 0.0;
}
// E of cluster row jr = j S + sigma at that column: bias' + sum_e W'[e][jr] u_e in e
// order (the GEMM's sums, blocked differently: equal to rounding), before the VHEM
// division by esmooth (the caller applies it behind a uniform branch: written as a
// select, the fp64 division ran for every entry on the VBHEM path too)
__device__ __forceinline__ double k1_entry(const SplitArgs &p, int jr,
                                           const double (&u)[kK1InKernelMaxKdp]) {
  double acc = p.ebias[jr];
#pragma unroll
  for (int e = 0; e < kK1InKernelMaxKdp; ++e)
    if (e < p.ekdp) acc = fma(p.eW[(size_t)e * p.eksp + jr], u[e], acc);
  return acc;
}
bool split_supported(int S, int SB, int d);
int split_lpc(int S);      // lanes per column
int split_lpc_bwd(int S);  // lanes per column, alternative for kFbBackward (BwdLPC)
hipError_t launch_split(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st);
int split_resident_blocks(const SplitArgs &a, size_t lds);  // per CU, for a.mode

// fb_bwd2_kernel (vbhem_fb_bwd.hip): the backward-only pass (kFbBackward) for
// S <= kBwd2MaxS, two base-state columns per lane (S <= 8) or one; SplitArgs fields
// used: SB, K, S, T, nwb, i_begin/i_end/i_buf0, prior, A, logA, logPi, E, e_ld,
// Atg, LL, flags.
constexpr int kBwd2MaxS = 16;
int bwd2_waves(int S);            // waves per block (one block per CU)
size_t bwd2_lds(int S, int nwb);  // dynamic LDS bytes (0: S unsupported)
int bwd2_ppb(int S, int nwb);     // pairs per block
int bwd2_resident_blocks(int S, int nwb, size_t lds);
// t0 / t1 (optional): timing events recorded by the dispatch itself at the kernel's
// start and end (hipExtLaunchKernelGGL): no marker packets, no idle GPU around it
hipError_t launch_bwd2(const SplitArgs &a, unsigned grid, size_t lds, hipStream_t st,
                       hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);

// kernel timing hooks for code outside vbhem_capi.hip (null when timing is off)
void *timing_begin(hipStream_t st);
void timing_end_em_math(void *ev0, hipStream_t st);

// fb_bwd4_kernel (vbhem_fb_bwd4.hip): the backward-only pass for S = 8, SB <= 8 with
// both contractions on v_mfma_f64_4x4x4f64; SplitArgs fields as fb_bwd2_kernel
bool bwd4_supported(int S, int SB);
int bwd4_waves();            // waves per block
int bwd4_ppb();              // pairs per block (one tile per wavefront)
int bwd4_resident_blocks();  // per CU
bool bwd4_o32(const SplitArgs &a);  // the 32-bit-offset version applies (kernel <true>)
bool bwd12_o32(const SplitArgs &a);  // fb_bwd12_kernel's likewise
bool list4_fast(const SplitArgs &a);  // fb_list4_kernel<T, true>: SB == 8 and 32-bit offsets
bool list12_fast(const SplitArgs &a);  // fb_list12_kernel<T, true>: SB == 12 and 32-bit offsets
hipError_t launch_bwd4(const SplitArgs &a, unsigned grid, hipStream_t st, hipEvent_t t0 = nullptr,
                       hipEvent_t t1 = nullptr);
// fb_bwd12_kernel (vbhem_fb_bwd12.hip): the same pass for S = 12, SB <= 12 (3 x 3 blocks)
bool bwd12_supported(int S, int SB);
int bwd12_ppb();              // pairs per block (one quad per wavefront)
int bwd12_resident_blocks();  // per CU
hipError_t launch_bwd12(const SplitArgs &a, unsigned grid, hipStream_t st, hipEvent_t t0 = nullptr,
                        hipEvent_t t1 = nullptr);

// fb_list4_kernel (vbhem_fb_list4.hip): the gate-list pass for S = 8, SB <= 8, T = 10
// with every contraction on v_mfma_f64_4x4x4f64; SplitArgs fields as fb_split_kernel's
// list mode (E, A, prior, Atg, logA, logPi, lists, nu1 / xi / tnu, flags)
constexpr int kList4MaxK = 1024;
bool list4_supported(int S, int SB, int T, int K);
int list4_resident_blocks();  // per CU
// the wavefronts of a grid of fb_list4_kernel when its per-wave queue of flagged pairs
// (xinline) cannot overflow -- every cluster's list full -- else a count no inline
// fallback accepts
long long list4_inline_waves(const SplitArgs &a, unsigned grid);
hipError_t launch_list4(const SplitArgs &a, unsigned grid, hipStream_t st);

// fb_list12_kernel (vbhem_fb_list12.hip): the gate-list pass for S = 12, SB <= 12, T = 10
// (3 x 3 blocks of v_mfma_f64_4x4x4f64, the lattice in registers); fields as fb_list4_kernel
bool list12_supported(int S, int SB, int T, int K);
int list12_resident_blocks();  // per CU
hipError_t launch_list12(const SplitArgs &a, unsigned grid, hipStream_t st);

hipError_t launch_fb(const FbArgs &a, dim3 grid, dim3 block, size_t lds, hipStream_t st);
// Fallback bookkeeping in the workspace's int array `flags`:
//   [0] pairs flagged by the current pass (consumed and reset by fb_exact_kernel)
//   [1] pairs flagged over the whole call (vbhem_last_fallback_count)
//   [2] fb_exact_kernel blocks finished (the last one resets [0] and [2])
//   [kFlagHead ...] the flagged pair indices
// A pair is flagged only when its factorised normaliser underflowed with finite
// inputs; pairs whose cluster constants or emissions are not finite (a diverged
// EM trial) are not flagged: their L_elbo is written as NaN, as the reference's
// arithmetic would produce, and they cost the fallback nothing.
//   [3] the first entry of the gate-list pass (written by resp_kernel when the fallback
//       is folded: resp_kernel takes [0, [3]), the fb_exact_kernel launch before the
//       statistics the rest)
constexpr int kFlagHead = 4;
// Before the counters (flags - kFlagPre): [0..1] a 64-bit clean tag, [2] the last
// fused call's total ([1] copied there by stats_final_kernel, which then zeroes
// [0..3] and writes the tag: the counters are clean between calls), [3] kFlagLost:
// sticky, kFlagLostMark set by an fb_bwd2_kernel block that gave up waiting for block 0's tag (its
// flagged pairs may have been zeroed away); stats_final_kernel then writes NaN
// statistics, every call, until a path that zeroes the head runs.
// fb_bwd2_kernel's in-kernel preparation (SplitArgs::prep) zeroes the counters only
// when the tag is not this process's flag_tag(); every other path zeroes the
// kFlagPre + kFlagHead ints before its first pass (emission_prep_kernel, or a memset).
// Reuse of the memory by another tensor overwrites the tag first (it leads the buffer).
constexpr int kFlagPre = 4;
constexpr int kFlagLost = 3;
// the value that marks it (not just non-zero: a head of garbage -- memory reused from
// another tensor, which the in-kernel preparation must accept -- is not a lost handshake)
constexpr int kFlagLostMark = 0x4C4F5354;
unsigned long long flag_tag();
constexpr int kFlagBad = 1, kFlagNonFinite = 2;  // per-pair LDS flag bits
#ifndef VBHEM_EXACT_BLOCK
#define VBHEM_EXACT_BLOCK 512
#endif
// fb_exact_kernel: threads per block (8 wavefronts: half the workgroups of 4-wave blocks
// to dispatch for the same slots -- the launch is paid every E-step, flags or not)
constexpr int kExactBlock = VBHEM_EXACT_BLOCK;
constexpr int kExactBlocks = 131072 / kExactBlock;  // blocks (wavefronts grid-stride over the list)
constexpr int kExactSlots = kExactBlocks * kExactBlock / 64;  // scratch slots: one per wavefront
// from_fold: start at flag_count[3] (the entries before it were folded into resp_kernel)
hipError_t launch_fb_exact(const FbArgs &a, double *scratch, size_t stride, int nslots,
                           hipStream_t st, bool from_fold = false);
hipError_t launch_emit(const EmitArgs &a, hipStream_t st);
bool plan_stats(StatsArgs &a, size_t &lds, int &ngroups);
hipError_t launch_resp(const StatsArgs &a, int nchunk, hipStream_t st);
hipError_t launch_stats(const StatsArgs &a, int nchunk, int ngroups, size_t lds, hipStream_t st);
bool plan_stats_list(StatsArgs &a, size_t &lds);
hipError_t launch_gate_list(const StatsArgs &a, int nchunk, hipStream_t st);
size_t gate_list_lds(int K);  // dynamic LDS of gate_list_kernel for K clusters
size_t resp_lds(int K, int KT);  // dynamic LDS of resp_kernel / resp_trials_kernel
// *stats_slabs (optional): the slabs [0, n) holding this launch's N1 / M / U entries
hipError_t launch_stats_list(const StatsArgs &a, int nchunk, size_t lds, hipStream_t st,
                             int *stats_slabs = nullptr);
// sums slabs [0, nslab) of the Nj / Lt1 / Lt7 columns (resp_kernel's per-chunk partials)
// and slabs [0, nslab_stats) of the N1 / M / U columns (KT clusters x S states per
// section of SL doubles)
// fpre (optional): the flag head (flags - kFlagPre) to close: last total, counters
// zeroed, tag written (kFlagPre)
// done (optional, needs fpre): after every block's statistics are stored at system
// scope, the last block to finish stores done_val there (vbhem_arm_done_word)
hipError_t launch_stats_final(const double *slabs, int nslab, int nslab_stats, int slab_len, int KT,
                              int S, int SL, double *out, hipStream_t st, int *fpre = nullptr,
                              unsigned long long *done = nullptr, unsigned long long done_val = 0);

}  // namespace vbhem

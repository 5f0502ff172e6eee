// vbhem_capi.hip -- C ABI of libvbhem_estep.so (declared in include/vbhem_estep.h).
//
// Validates arguments, plans the launch geometry (pairs per block, LDS
// carve-up), carves the caller's workspace and enqueues the kernels of
// vbhem_kernels.hip on the caller's stream.  No allocation, no host
// synchronisation on the device-pointer entry points (graph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <string>
#include <utility>
#include <vector>

#include "vbhem_estep.h"
#include "vbhem_internal.h"
#include "vbhem_exact.h"
#include "vbhem_math.h"

// the fault-injection hook of vbhem_debug_extra_lds (tests only; 0 in production)
static std::atomic<size_t> g_debug_extra_lds{0};

namespace {

thread_local std::string g_err;

// Optional kernel timing (bench/profiling): hipEvents recorded on the launch
// stream around each kernel launch; read back (and synchronised) only by
// vbhem_timing_read*.  Off by default.  Per host thread (thread_local), like the
// schedule below: the library keeps no state shared between threads, so several
// host threads may drive it at once (the reference MEX is re-entrant).  Never
// recorded into a stream that is being captured into a graph: a captured event
// would be destroyed by the next vbhem_timing_read while the graph still
// records into it on every replay.
// Levels: 1 every timed launch (fb, emission, statistics, gated forward), 2 the fb
// launches only -- two events per E-step, so the instrumentation costs the timed
// region next to nothing (each recorded event is a marker packet the queue
// processes between kernels; a dozen per step was ~40 us at N = 12,500).  Events
// are recycled through a per-thread pool (no create/destroy per launch).
struct TimingState {
  int level = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> fb, stats, em, gf, emd;  // emd: EM-loop math kernel
  std::vector<long long> fb_pairs;
  std::vector<hipEvent_t> pool;
  ~TimingState() {
    for (hipEvent_t e : pool) (void)hipEventDestroy(e);
  }
};
thread_local TimingState g_timing;

// the kernels the last call of this host thread ran for its recursion passes
// (vbhem_last_kernel: what a benchmark line names, taken from the launch itself)
thread_local std::string g_last_kernel[2];
std::string split_name(const vbhem::SplitArgs &a) {
  return "vbhem::fb_split_kernel<" + std::to_string(a.S) + ", " + std::to_string(a.lpc) + ", " +
         std::to_string(a.mode) + ">";
}

// fused schedule of this host thread (vbhem_set_fused_mode; VBHEM_FUSED_DENSE=1
// in the environment sets every thread's default)
int default_fused_mode() {
  const char *ev = std::getenv("VBHEM_FUSED_DENSE");
  return (ev && std::atoi(ev) != 0) ? VBHEM_FUSED_DENSE : VBHEM_FUSED_GATED;
}
thread_local int g_fused_mode = default_fused_mode();

// timing is recorded for this launch: enabled on this thread and the stream
// is not capturing
bool timing_on(hipStream_t st, bool fb_launch = false) {
  if (g_timing.level == 0 || (g_timing.level == 2 && !fb_launch)) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return false;
  return cs == hipStreamCaptureStatusNone;
}

// a timing event from the pool, not recorded (st == nullptr), or recorded on st
hipEvent_t timing_event(hipStream_t st, bool record = true) {
  hipEvent_t ev = nullptr;
  if (!g_timing.pool.empty()) {
    ev = g_timing.pool.back();
    g_timing.pool.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) {
    // timing-only events: no system-scope release (an L2 writeback + invalidate
    // per record, ~6 us of idle GPU around each timed kernel at N = 12,500)
    return nullptr;
  }
  if (record) (void)hipEventRecord(ev, st);
  return ev;
}
void timing_recycle(hipEvent_t ev) {
  if (ev) g_timing.pool.push_back(ev);
}

}  // namespace

// EM-loop math kernel timing (vbhem_em.hip), same events and levels as the E-step's
namespace vbhem {
void *timing_begin(hipStream_t st) { return timing_on(st) ? timing_event(st) : nullptr; }
void timing_end_em_math(void *ev0, hipStream_t st) {
  if (ev0) g_timing.emd.emplace_back(static_cast<hipEvent_t>(ev0), timing_event(st));
}
// this process's clean tag of the flag head (kFlagPre): random, never 0 (a zeroed head)
unsigned long long flag_tag() {
  static const unsigned long long t = [] {
    std::random_device rd;
    unsigned long long v = ((unsigned long long)rd() << 32) ^ rd();
    v ^= (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
    return v | 1ull;
  }();
  return t;
}
}  // namespace vbhem

namespace {

int fail(int code, const std::string &msg) {
  g_err = msg;
  // a refused launch (too much LDS, a bad grid) also leaves HIP's per-thread last
  // error set; left pending it would surface in the caller's next, unrelated HIP
  // call (torch checks hipGetLastError after each of its launches).  The error is
  // reported here, through the status and vbhem_last_error(), so it is consumed.
  if (code == VBHEM_ERR_HIP) (void)hipGetLastError();
  return code;
}

int hip_fail(hipError_t e, const char *where) {
  return fail(VBHEM_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

}  // namespace

// shared with the other C-ABI translation units (vbhmm_fb.hip): vbhem_last_error()
int vbhem::set_error(int code, const std::string &msg) { return fail(code, msg); }

namespace {

constexpr size_t kLdsLimit = 160 * 1024;          // gfx950 LDS per workgroup
constexpr int kFbMaxThreads = 512;                // fb_pairs_kernel launch bound
constexpr int kExactThreads = vbhem::kExactSlots;  // fallback scratch slots (one per wavefront)
constexpr int kChunkMinBases = 64;                 // fused epilogue: bases per chunk, at least
constexpr size_t kGroupBudget = (size_t)8 << 30;  // per-pair buffers per group (fused)
constexpr int kMaxSlabs = 512;    // statistics chunks (= resp/stats blocks per group)

inline int odd_up(int x) { return (x % 2 == 0) ? x + 1 : x; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct FbPlan {
  vbhem::FbArgs a;
  dim3 block;
  size_t lds;
  int PPB;
};

bool plan_fb(int SB, int d, int covmode, int K, int S, int T, FbPlan &out) {
  const int NE = S * SB;
  if (NE > kFbMaxThreads) return false;
  const int RS = odd_up(SB), AS = odd_up(S), ABS = odd_up(SB);
  const int np = covmode == VBHEM_COV_FULL ? d * (d + 1) / 2 : d;
  const int MS = odd_up(d), PS = odd_up(np);
  double best = -1.0;
  bool found = false;
  for (int ppb = 1; ppb <= 32; ++ppb) {
    const int BJ = std::min(ppb, K);
    const int BI = ppb / BJ;
    const int P = BI * BJ;
    if (P != ppb) continue;
    const int threads = (P * NE + 63) / 64 * 64;
    if (threads > kFbMaxThreads) break;
    size_t off = 0;
    vbhem::FbArgs a{};
    a.off_At = (int)off; off += (size_t)BJ * S * AS;
    a.off_amax = (int)off; off += (size_t)BJ * S;
    a.off_lpi = (int)off; off += (size_t)BJ * S;
    a.off_Ab = (int)off; off += (size_t)BI * SB * ABS;
    a.off_pib = (int)off; off += (size_t)BI * SB;
    a.off_flag = (int)off; off += (size_t)(P + 1) / 2;
    a.off_reg = (int)off;
    size_t k1 = 0;
    a.off_k1m = (int)k1; k1 += (size_t)BJ * S * MS;
    a.off_k1P = (int)k1; k1 += (size_t)BJ * S * PS;
    a.off_k1c = (int)k1; k1 += (size_t)BJ * S;
    a.off_k1mu = (int)k1; k1 += (size_t)BI * SB * MS;
    a.off_k1C = (int)k1; k1 += (size_t)BI * SB * PS;
    const size_t pstride = (size_t)(T - 1) * S * RS + (size_t)(T - 1) * NE + 3 * (size_t)S * RS +
                           (size_t)S * S + SB;
    const size_t reg = std::max(k1, (size_t)P * pstride);
    const size_t lds = (off + reg) * sizeof(double);
    if (lds > kLdsLimit) continue;
    const double util = double(P * NE) / threads;
    const int blocks_per_cu = std::max<int>(1, (int)(kLdsLimit / lds));
    const int waves = std::min(32, blocks_per_cu * threads / 64);
    const double score = util * std::min(waves, 16) + 1e-3 * std::min(threads, 256);
    if (score > best) {
      best = score;
      found = true;
      a.SB = SB; a.d = d; a.covmode = covmode; a.K = K; a.S = S; a.T = T;
      a.BI = BI; a.BJ = BJ; a.NE = NE; a.RS = RS; a.AS = AS; a.ABS = ABS;
      a.njb = (K + BJ - 1) / BJ;
      a.np = np; a.MS = MS; a.PS = PS;
      a.pair_stride = (int)pstride;
      out.a = a;
      out.block = dim3(threads);
      out.lds = lds;
      out.PPB = P;
    }
  }
  return found;
}

struct SplitPlan {
  bool ok = false;
  vbhem::SplitArgs a{};
  size_t lds = 0;       // kFbDense
  size_t lds_bwd = 0;   // kFbBackward (no lattice)
  size_t lds_list = 0;  // kFbList (lattice + work-item prefix)
  int ppb = 0;
  // kFbList: its own geometry (up to 8 waves per block, compact tables in LDS)
  vbhem::SplitArgs al{};
  size_t lds_l = 0;
};

// Geometry of fb_split_kernel; must match SplitLayout<S, LPC> (vbhem_internal.h).
SplitPlan plan_split(int SB, int d, int covmode, int K, int S, int T, int LPC) {
  SplitPlan sp;
  if (!vbhem::split_supported(S, SB, d)) return sp;
  const int SH = (S + LPC - 1) / LPC;
  const int LPP = S * LPC;
  const int XCS = (LPC * SH + 1) / 2 * 2 + 2;
  const int XP = S * XCS + 2;
  const int OFF_X = (2 * S * S + 2 * S + 1) / 2 * 2;
  double best = -1.0;
  for (int nwb = 1; nwb <= 4; ++nwb) {
    const int NT = nwb * 64;
    const int ppb = NT / LPP;
    if (ppb < 1) continue;
    const int off_Y = OFF_X + ppb * XP;
    const int off_F = (off_Y + ppb * S + 1) / 2 * 2;
    const int off_R = (off_F + (ppb + 1) / 2 + 1) / 2 * 2;
    const size_t lattice = (size_t)std::max(0, T - 2) * SH * NT;
    const size_t xi_park = S > 8 ? (size_t)ppb * S * S * LPC * SH : 0;  // parked H blocks (sum_xi)
    const size_t region = std::max<size_t>(std::max(lattice, xi_park), 2);
    const size_t lds = ((size_t)off_R + region) * sizeof(double);
    const int off_L = (int)(off_R + region);
    const size_t lds_list = ((size_t)off_L + ((size_t)K + 2) / 2) * sizeof(double);
    if (lds_list > kLdsLimit) continue;
    const double util = double(ppb * LPP) / NT;
    if (util > best + 0.02 || (LPC != vbhem::split_lpc(S) && util >= best)) {
      best = util;
      vbhem::SplitArgs &x = sp.a;
      x.SB = SB; x.d = d; x.covmode = covmode; x.K = K; x.S = S; x.T = T; x.nwb = nwb;
      x.lpc = LPC;
      x.off_Y = off_Y; x.off_F = off_F; x.off_R = off_R; x.off_L = off_L;
      x.mode = vbhem::kFbDense;
      sp.lds = lds;
      x.off_T = off_R + 2;
      sp.lds_bwd = ((size_t)x.off_T + vbhem::kLogTabDoubles + vbhem::kExpTabDoubles) * sizeof(double);
      sp.lds_list = lds_list;
      sp.ppb = ppb;
      sp.ok = true;
    }
  }
  // list mode: the lattice dominates LDS and the kernel runs 2 waves per SIMD, so the
  // most waves per CU come from one 8-wave block (C4: 156 KB) rather than 4-wave
  // blocks that no longer pair up once the 4 KB of tables are added
  int best_w = 0;
  for (int nwb : {8, 4, 2, 1}) {
    if (!sp.ok) break;
    const int NT = nwb * 64;
    const int ppb = NT / LPP;
    if (ppb < 1) continue;
    const int off_Y = OFF_X + ppb * XP;
    const int off_F = (off_Y + ppb * S + 1) / 2 * 2;
    const int off_R = (off_F + (ppb + 1) / 2 + 1) / 2 * 2;
    const size_t lattice = (size_t)std::max(0, T - 2) * SH * NT;
    const size_t xi_park = S > 8 ? (size_t)ppb * S * S * LPC * SH : 0;
    const size_t region = std::max<size_t>(std::max(lattice, xi_park), 2);
    const int off_L = (int)(off_R + region);
    const int off_T = (off_L + (K + 2) / 2 + 1) / 2 * 2;
    const size_t lds = ((size_t)off_T + vbhem::kExpTabEntries + 2 * vbhem::kLogTabEntries) * sizeof(double);
    if (lds > kLdsLimit) continue;
    const int waves = std::min(8, nwb * (int)(kLdsLimit / lds));
    if (waves > best_w) {
      best_w = waves;
      vbhem::SplitArgs x = sp.a;
      x.nwb = nwb;
      x.off_Y = off_Y; x.off_F = off_F; x.off_R = off_R; x.off_L = off_L; x.off_T = off_T;
      x.mode = vbhem::kFbList;
      sp.al = x;
      sp.lds_l = lds;
    }
  }
  return sp;
}

size_t exact_stride(int S, int SB, int T) {  // Theta [T][S][S][SB], then the small arrays
  return (size_t)S * S * SB * T + (size_t)vbhem::exact_wave_lds(S, SB);
}

int check_inputs(const vbhem_base_t *b, const vbhem_cluster_t *c, int T, bool need_ptrs = true) {
  if (!b || !c) return fail(VBHEM_ERR_ARG, "null base or cluster descriptor");
  if (b->N < 0 || b->SB < 1 || b->d < 1 || c->K < 1 || c->S < 1 || T < 1)
    return fail(VBHEM_ERR_ARG, "invalid sizes (need N>=0, SB>=1, d>=1, K>=1, S>=1, T>=1)");
  if (b->covmode != VBHEM_COV_DIAG && b->covmode != VBHEM_COV_FULL)
    return fail(VBHEM_ERR_ARG, "covmode must be VBHEM_COV_DIAG or VBHEM_COV_FULL");
  if (need_ptrs && b->N > 0 &&
      (!b->prior || !b->A || !b->centres || !b->covars || !c->logA || !c->logPi || !c->m ||
       !c->P || !c->c))
    return fail(VBHEM_ERR_ARG, "null input array");
  if ((long long)b->N * c->K > 0x7fffffffLL)
    return fail(VBHEM_ERR_UNSUPPORTED, "N*K exceeds 2^31-1 pairs per call; shard the bases");
  return VBHEM_OK;
}

void fill_inputs(vbhem::FbArgs &a, const vbhem_base_t *b, const vbhem_cluster_t *c) {
  a.prior = b->prior; a.A = b->A; a.centres = b->centres; a.covars = b->covars;
  a.logA = c->logA; a.logPi = c->logPi; a.m = c->m; a.P = c->P; a.c = c->c;
}

// ---- workspace carving -------------------------------------------------------
struct Carver {
  char *base;
  size_t off = 0;
  explicit Carver(void *p) : base(static_cast<char *>(p)) {}
  template <class T>
  T *take(size_t n) {
    off = align_up(off, 256);
    T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

// emission_u_kernel applies (k-steps <= kUMaxKq): the per-call operand U is needed
// unless the caller prepared one (base->U)
bool u_gemm_ok(const vbhem_base_t *b) {
  return vbhem::emission_kdp(b->d, b->covmode) / 4 <= vbhem::kUMaxKq && !std::getenv("VBHEM_NO_UGEMM");
}
bool need_u_ws(const vbhem_base_t *b) { return !b->U && u_gemm_ok(b); }

struct PairsWs {
  int *fpre;   // the flag head (vbhem_internal.h kFlagPre), then
  int *flags;  // [0]=count [1]=total [2..] list
  double *scratch;
  double *tnu;
  double *E, *W, *bias, *shift;  // emission GEMM (split path)
  double *U;                     // the GEMM's base-set operand, built per call (null: prepared)
};

inline size_t emission_w_doubles(int d, int covmode, int K, int S) {
  return (size_t)vbhem::emission_kdp(d, covmode) * vbhem::emission_ksp(K * S);
}

size_t carve_pairs(void *ws, const vbhem_base_t *b, const vbhem_cluster_t *c, int T, bool need_tnu,
                   PairsWs &w) {
  Carver cv(ws);
  const size_t np = (size_t)b->N * c->K;
  w.fpre = cv.take<int>(vbhem::kFlagPre + vbhem::kFlagHead + np);  // first: see kFlagPre
  w.flags = w.fpre + vbhem::kFlagPre;
  w.tnu = need_tnu ? cv.take<double>(np * c->S * b->SB) : nullptr;
  w.E = cv.take<double>(np * c->S * b->SB);
  w.W = cv.take<double>(emission_w_doubles(b->d, b->covmode, c->K, c->S));
  w.bias = cv.take<double>((size_t)vbhem::emission_ksp(c->K * c->S));
  w.shift = cv.take<double>((size_t)b->d);
  w.U = need_u_ws(b) ? cv.take<double>(vbhem::u_doubles((long long)b->N * b->SB + 16, b->d,
                                                         b->covmode))
                     : nullptr;
  // the exact fallback's scratch last: its size does not move the hot buffers
  w.scratch = cv.take<double>(exact_stride(c->S, b->SB, T) * kExactThreads);
  return cv.off + 256;
}

struct FusedWs {
  int group;  // bases per group
  int nslab;
  int slab_len;
  int *fpre, *flags;                // the flag head (kFlagPre), the counters and list after it
  int *gate_cnt, *list, *list_tot;  // gated schedule: [nslab][K], [K][group], [K]
  double *Atg;                      // gated schedule: [K][S][S] A' for the backward pass
  double *scratch, *nu1, *xi, *tnu, *Z, *slabs;
  double *E, *W, *bias, *shift;
  double *U;                        // per-call operand of the emission GEMM (null: prepared)
};

size_t carve_fused(void *ws, const vbhem_base_t *b, const vbhem_cluster_t *c, int T, FusedWs &w,
                   int R = 1) {
  Carver cv(ws);
  const int K = c->K, S = c->S, SB = b->SB;
  const size_t per_base = (size_t)K * (S + (size_t)S * S + 2 * (size_t)S * SB) * sizeof(double);
  size_t g = std::max<size_t>(1, kGroupBudget / std::max<size_t>(1, per_base));
  g = std::min<size_t>(g, (size_t)std::max(1, b->N));
  if (const char *ev = std::getenv("VBHEM_GROUP_BASES"))  // tests: force several groups
    g = std::max<size_t>(1, std::min<size_t>(g, (size_t)std::atoll(ev)));
  w.group = (int)g;
  int maxslab = kMaxSlabs;
  if (const char *ev = std::getenv("VBHEM_NSLAB")) maxslab = std::max(1, std::min(8192, std::atoi(ev)));
  w.nslab = std::min<int>(w.group, maxslab);
  w.slab_len = R * (int)vbhem_stats_len(K / R, S, b->d, b->covmode);
  // flagged-pair list: with the fallback folded into the consumers the backward pass's
  // entries stay while the gate-list pass appends its own (at most g K + g K)
  w.fpre = cv.take<int>(vbhem::kFlagPre + vbhem::kFlagHead + 2 * g * K);  // first: see kFlagPre
  w.flags = w.fpre + vbhem::kFlagPre;
  w.nu1 = cv.take<double>(g * K * S);
  w.xi = cv.take<double>(g * K * S * S);
  w.tnu = cv.take<double>(g * K * S * SB);
  w.Z = cv.take<double>(g * K);
  w.slabs = cv.take<double>((size_t)w.nslab * w.slab_len);
  w.E = cv.take<double>(g * K * S * SB);
  w.W = cv.take<double>(emission_w_doubles(b->d, b->covmode, K, S));
  w.bias = cv.take<double>((size_t)vbhem::emission_ksp(K * S));
  w.shift = cv.take<double>((size_t)b->d);
  w.U = need_u_ws(b) ? cv.take<double>(vbhem::u_doubles((long long)g * SB + 16, b->d, b->covmode))
                     : nullptr;
  w.gate_cnt = cv.take<int>((size_t)w.nslab * K);
  w.list = cv.take<int>(g * K);
  w.list_tot = cv.take<int>((size_t)K);
  // A' [K][S][S] (read-only for every recursion kernel)
  w.Atg = cv.take<double>((size_t)K * S * S);
  // the exact fallback's scratch last: its size does not move the hot buffers
  w.scratch = cv.take<double>(exact_stride(S, SB, T) * kExactThreads);
  return cv.off + 256;
}

struct FbCtx {
  FbPlan plan;      // generic element-per-lane kernel
  SplitPlan split;  // column-per-LPC-lanes kernel (preferred when it applies)
  SplitPlan bwd;    // its backward-only mode (gated schedule), possibly another LPC
  // the backward-only pass on fb_bwd2_kernel (S <= 8): LDS bytes, pairs per block
  size_t bwd2_lds = 0;
  int bwd2_ppb = 0, bwd2_nwb = 0;
  bool bwd12 = false;  // S = 12, SB <= 12: fb_bwd12_kernel (MFMA contractions) instead
  bool bwd4 = false;  // S = 8, SB <= 8: fb_bwd4_kernel (MFMA contractions) instead
  bool list4 = false;  // S = 8, SB <= 8, T = 10: fb_list4_kernel for the gate-list pass
  bool list12 = false;  // S = 12, SB <= 12, T = 10: fb_list12_kernel for the gate-list pass
  // gated schedule on fb_bwd2_kernel + fb_split_kernel's list mode with a short K1
  // (kdp <= 8: C2, C3): both evaluate E from the prepared operand (SplitArgs::eU);
  // no emission GEMM launch, no E traffic
  bool k1_in_kernel = false;
  // ... and emission_prep_kernel's work inside fb_bwd2_kernel (SplitArgs::prep): set by
  // the fused call for a prepared operand; fpre = the workspace's flag head
  bool bwd2_prep = false;
  int *fpre = nullptr;
  vbhem::EmissionArgs em{};  // K1 GEMM feeding the split kernel
  size_t em_lds = 0;
  // emission_u_kernel: on the prepared operand (base->U) or one built per call in u_ws
  bool use_u = false;
  size_t em_lds_u = 0;
  const vbhem_base_t *base = nullptr;
  double *u_ws = nullptr;
};

int prepare_fb(FbCtx &c, const vbhem_base_t *b, const vbhem_cluster_t *cl, int T,
               double smooth = 1.0) {
  c.split = plan_split(b->SB, b->d, b->covmode, cl->K, cl->S, T, vbhem::split_lpc(cl->S));
  // backward-only pass: half the lanes per column (no forward-sweep registers to
  // hold), more rows per lane: no DPP for S <= 8, more independent exp/log chains
  c.bwd = plan_split(b->SB, b->d, b->covmode, cl->K, cl->S, T, vbhem::split_lpc_bwd(cl->S));
  if (c.split.ok) {
    vbhem::EmissionArgs &e = c.em;
    e.SB = b->SB; e.d = b->d; e.covmode = b->covmode; e.K = cl->K; e.S = cl->S;
    e.smooth = smooth;
    e.centres = b->centres; e.covars = b->covars; e.m = cl->m; e.P = cl->P; e.c = cl->c;
    if (!vbhem::plan_emission(e, c.em_lds)) c.split.ok = false;
    if (c.split.ok && u_gemm_ok(b) && vbhem::plan_emission_u(e, c.em_lds_u)) {
      c.use_u = true;
      e.zfix = b->U;  // a prepared operand carries its shift in its head
    }
  }
  c.base = b;
  const bool have_elems = plan_fb(b->SB, b->d, b->covmode, cl->K, cl->S, T, c.plan);
  if (!c.split.ok && !have_elems)
    return fail(VBHEM_ERR_UNSUPPORTED,
                "no launch geometry fits (S*SB must be <= 512 and the per-pair lattice "
                "(2*(T-1)+3)*S*SB doubles must fit in 160 KiB of LDS)");
  if (!have_elems) c.plan = FbPlan{};
  fill_inputs(c.plan.a, b, cl);
  // fields the exact fallback kernel needs even when the generic plan is unused
  c.plan.a.SB = b->SB; c.plan.a.d = b->d; c.plan.a.covmode = b->covmode;
  c.plan.a.K = cl->K; c.plan.a.S = cl->S; c.plan.a.T = T;
  c.plan.a.smooth = smooth;
  if (c.split.ok) {
    vbhem::SplitArgs &a = c.split.a;
    a.prior = b->prior; a.A = b->A; a.logA = cl->logA; a.logPi = cl->logPi;
    vbhem::SplitArgs &al = c.split.al;
    al.prior = b->prior; al.A = b->A; al.logA = cl->logA; al.logPi = cl->logPi;
    vbhem::SplitArgs &ab = c.bwd.a;
    ab.prior = b->prior; ab.A = b->A; ab.logA = cl->logA; ab.logPi = cl->logPi;
    if (c.bwd.ok && cl->S <= vbhem::kBwd2MaxS && !std::getenv("VBHEM_NO_BWD2")) {
      c.bwd2_nwb = vbhem::bwd2_waves(cl->S);
      c.bwd2_lds = vbhem::bwd2_lds(cl->S, c.bwd2_nwb);
      c.bwd2_ppb = vbhem::bwd2_ppb(cl->S, c.bwd2_nwb);
      c.bwd4 = vbhem::bwd4_supported(cl->S, b->SB) && !std::getenv("VBHEM_NO_BWD4");
      c.bwd12 = vbhem::bwd12_supported(cl->S, b->SB) && !std::getenv("VBHEM_NO_BWD12");
      c.list4 = vbhem::list4_supported(cl->S, b->SB, T, cl->K) && !std::getenv("VBHEM_NO_LIST4");
      c.list12 = vbhem::list12_supported(cl->S, b->SB, T, cl->K) && !std::getenv("VBHEM_NO_LIST12");
    }
    c.k1_in_kernel = c.use_u && c.bwd2_lds && !c.bwd4 && !c.bwd12 && !c.list4 && !c.list12 &&
                     c.em.kdp <= vbhem::kK1InKernelMaxKdp && !std::getenv("VBHEM_NO_K1_IN_KERNEL");
  }
  return VBHEM_OK;
}

// the in-kernel K1's operands (FbCtx::k1_in_kernel): the prepared operand, or this
// call's (run_fb builds it for bases from i_begin: tile 0 at column i_begin SB rounded
// down to 16)
void set_k1_operands(const FbCtx &c, int i_begin, vbhem::SplitArgs &ca) {
  if (c.base->U) {
    ca.eU = c.base->U;
    ca.e_col0 = 0;
  } else {
    ca.eU = c.u_ws;
    ca.e_col0 = (long long)i_begin * c.base->SB / 16 * 16;
  }
  ca.eW = c.em.W;
  ca.ebias = c.em.bias;
  ca.ekdp = c.em.kdp;
  ca.eksp = c.em.ksp;
  ca.esmooth = c.em.smooth;
}

// W, bias, shift of the emission GEMM: once per call (depends on the clusters only)
int run_emission_prep(FbCtx &c, double *W, double *bias, double *shift, hipStream_t st,
                      int *zero_ints = nullptr, int n_zero = 0, double *Atg = nullptr,
                      const double *logA = nullptr) {
  if (!c.split.ok) return VBHEM_OK;
  c.em.W = W; c.em.bias = bias; c.em.shift = shift;
  c.em.zero_ints = zero_ints; c.em.n_zero = zero_ints ? n_zero : 0;
  c.em.Atg = Atg; c.em.logA = logA;
  hipError_t e = vbhem::launch_emission_prep(c.em, st);
  if (e != hipSuccess) return hip_fail(e, "emission_prep_kernel");
  return VBHEM_OK;
}

// Persistent grid of the list-mode pass: every resident block of the device.
unsigned list_grid(const vbhem::SplitArgs &a, size_t lds) {
  const int cus = vbhem::device_cus();
  const int per_cu = std::max(1, vbhem::split_resident_blocks(a, lds));
  return (unsigned)(cus * per_cu);
}

// Gated schedule, second pass: both sweeps for the pairs of the gate lists.
int run_fb_list(const FbCtx &c, int i_begin, int i_end, int i_buf0, double *nu1, double *xi,
                double *tnu, const double *Ebuf, long long e_ld, const int *list,
                const int *list_tot, int list_cap, int *flags, double *scratch, double *LL,
                hipStream_t st, bool fold = false, bool *inlined = nullptr) {
  if (i_end <= i_begin) return VBHEM_OK;
  // flags[0] is zero here: the backward pass's fb_exact_kernel reset it
  if (!c.split.lds_l) return fail(VBHEM_ERR_UNSUPPORTED, "gate-list pass does not fit LDS");
  vbhem::SplitArgs ca = c.split.al;
  ca.mode = vbhem::kFbList;
  ca.E = Ebuf; ca.e_ld = e_ld;
  ca.i_begin = i_begin; ca.i_end = i_end; ca.i_buf0 = i_buf0;
  ca.LL = nullptr; ca.nu1 = nu1; ca.xi = xi; ca.tnu = tnu;
  ca.flag_count = flags; ca.flag_list = flags + vbhem::kFlagHead;
  ca.list = list; ca.list_tot = list_tot; ca.list_cap = list_cap;
  // folded fallback: the list kernel recomputes its own flagged pairs when its
  // persistent grid has a scratch slot per wavefront (then no launch after the pass)
  ca.xinline = 0;
  auto set_inline = [&](long long waves) {
    if (!fold || waves > kExactThreads || std::getenv("VBHEM_NO_LIST_INLINE")) return;
    ca.xinline = 1;
    ca.xscr = scratch;
    ca.xstride = (long long)exact_stride(c.plan.a.S, c.plan.a.SB, c.plan.a.T);
    vbhem::FbArgs &x = ca.xf;
    x = c.plan.a;
    x.i_begin = i_begin; x.i_end = i_end; x.i_buf0 = i_buf0;
    x.LL = LL; x.nu1 = nu1; x.xi = xi; x.tnu = tnu;
    x.flag_count = flags; x.flag_list = flags + vbhem::kFlagHead;
  };
  hipEvent_t ev0 = timing_on(st) ? timing_event(st) : nullptr;
  hipError_t e;
  if (c.list4) {  // S = 8, SB <= 8, T = 10: fb_list4_kernel (MFMA), one wave per quad item
    ca.Atg = c.bwd.a.Atg;
    const unsigned grid = (unsigned)(vbhem::device_cus() * std::max(1, vbhem::list4_resident_blocks()));
    set_inline(vbhem::list4_inline_waves(ca, grid));
    e = vbhem::launch_list4(ca, grid, st);
    if (e != hipSuccess) return hip_fail(e, "fb_list4_kernel");
    g_last_kernel[1] = "vbhem::fb_list4_kernel<" + std::to_string(ca.T) +
                       (vbhem::list4_fast(ca) ? ", true>" : ", false>");
  } else if (c.list12) {  // S = 12, SB <= 12, T = 10: fb_list12_kernel (MFMA), one wave per quad
    ca.Atg = c.bwd.a.Atg;
    const unsigned grid = (unsigned)(vbhem::device_cus() * std::max(1, vbhem::list12_resident_blocks()));
    e = vbhem::launch_list12(ca, grid, st);
    if (e != hipSuccess) return hip_fail(e, "fb_list12_kernel");
    g_last_kernel[1] = "vbhem::fb_list12_kernel<" + std::to_string(ca.T) +
                       (vbhem::list12_fast(ca) ? ", true>" : ", false>");
  } else {
    if (c.k1_in_kernel) set_k1_operands(c, i_begin, ca);
    const unsigned grid = list_grid(ca, c.split.lds_l);
    if (ca.S >= vbhem::kSplitInlineMinS && ca.S <= vbhem::kSplitInlineMaxS)
      set_inline((long long)grid * ca.nwb);
    e = vbhem::launch_split(ca, grid, c.split.lds_l, st);
    if (e != hipSuccess) return hip_fail(e, "fb_split_kernel(list)");
    g_last_kernel[1] = split_name(ca);
  }
  if (ev0) g_timing.gf.emplace_back(ev0, timing_event(st));
  if (inlined) *inlined = ca.xinline != 0;
  if (fold) return VBHEM_OK;  // inline, or launch_stats_list runs fb_exact_kernel from flag_count[3]
  vbhem::FbArgs a = c.plan.a;
  a.i_begin = i_begin; a.i_end = i_end; a.i_buf0 = i_buf0;
  a.LL = LL; a.nu1 = nu1; a.xi = xi; a.tnu = tnu;
  a.flag_count = flags; a.flag_list = flags + vbhem::kFlagHead;
  e = vbhem::launch_fb_exact(a, scratch, exact_stride(a.S, a.SB, a.T), kExactThreads, st);
  if (e != hipSuccess) return hip_fail(e, "fb_exact_kernel");
  return VBHEM_OK;
}

// K1 + K2-K4 over bases [i_begin, i_end) x all clusters.  mode kFbBackward
// (split kernel only) computes K2 + K3 (LL) alone; flagged pairs still get every
// output from the exact kernel.
int run_fb(const FbCtx &c, int i_begin, int i_end, int i_buf0, double *LL, double *nu1,
           double *xi, double *tnu, double *Ebuf, long long e_ld, int *flags, double *scratch,
           hipStream_t st, int mode = vbhem::kFbDense, vbhem::FbArgs *fold = nullptr) {
  if (i_end <= i_begin) return VBHEM_OK;
  vbhem::FbArgs a = c.plan.a;
  a.i_begin = i_begin;
  a.i_end = i_end;
  a.i_buf0 = i_buf0;
  a.LL = LL; a.nu1 = nu1; a.xi = xi; a.tnu = tnu;
  a.flag_count = flags;
  a.flag_list = flags + vbhem::kFlagHead;
  hipError_t e = hipSuccess;
  // K1 inside fb_bwd2_kernel (and the list pass after it): no emission GEMM
  const bool k1 = c.k1_in_kernel && mode == vbhem::kFbBackward;
  if (!c.split.ok) {  // split path: zeroed by emission_prep_kernel, reset by fb_exact_kernel
    e = hipMemsetAsync(flags, 0, sizeof(int), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(flags)");
  }
  if (c.split.ok) {
    vbhem::EmissionArgs ea = c.em;
    ea.i_begin = i_begin; ea.i_end = i_end; ea.i_buf0 = i_buf0; ea.E = Ebuf; ea.e_ld = e_ld;
    size_t em_lds = c.em_lds;
    hipEvent_t em0 = !k1 && timing_on(st) ? timing_event(st) : nullptr;
    if (c.use_u) {
      em_lds = c.em_lds_u;
      if (c.base->U) {
        ea.U = c.base->U;
        ea.u_col0 = 0;
      } else {  // this call's operand for bases [i_begin, i_end), shifted like W' / bias'
        if (!c.u_ws) return fail(VBHEM_ERR_WORKSPACE, "no operand buffer for the emission GEMM");
        const vbhem_base_t *b = c.base;
        vbhem::UPrepArgs ua{};
        ua.N = b->N; ua.SB = b->SB; ua.d = b->d; ua.covmode = b->covmode;
        ua.kdp = c.em.kdp; ua.i_begin = i_begin; ua.i_end = i_end;
        ua.u_col0 = (long long)i_begin * b->SB / 16 * 16;
        ua.nstates = b->nstates; ua.centres = b->centres; ua.covars = b->covars;
        ua.U = c.u_ws; ua.z = c.em.shift;
        e = vbhem::launch_u_prep(ua, st);
        if (e != hipSuccess) return hip_fail(e, "u_prep_kernel");
        ea.U = c.u_ws;
        ea.u_col0 = ua.u_col0;
      }
    }
    if (!k1) {
      e = vbhem::launch_emission(ea, em_lds, st);
      if (e != hipSuccess) return hip_fail(e, "emission_kernel");
      if (em0) g_timing.em.emplace_back(em0, timing_event(st));
    }
  }
  // the backward-only kernels take their timing events into the dispatch itself
  // (hipExtLaunchKernelGGL: start / end of the kernel, no marker packets around it);
  // the others are bracketed by two event records
  const bool ext_timed = c.split.ok && mode == vbhem::kFbBackward && (c.bwd4 || c.bwd12 || c.bwd2_lds);
  const bool timed = timing_on(st, true);
  hipEvent_t ev0 = timed ? timing_event(st, !ext_timed) : nullptr;
  hipEvent_t ev1 = timed && ext_timed ? timing_event(st, false) : nullptr;
  if (c.split.ok) {
    const SplitPlan &sp = mode == vbhem::kFbBackward ? c.bwd : c.split;
    vbhem::SplitArgs ca = sp.a;
    ca.mode = mode;
    ca.E = Ebuf; ca.e_ld = e_ld;
    ca.i_begin = i_begin; ca.i_end = i_end; ca.i_buf0 = i_buf0;
    ca.LL = LL; ca.nu1 = nu1; ca.xi = xi; ca.tnu = tnu;
    ca.flag_count = flags; ca.flag_list = flags + vbhem::kFlagHead;
    const unsigned ntile = (unsigned)((i_end - i_begin + sp.ppb - 1) / sp.ppb);
    unsigned grid = ntile * (unsigned)ca.K;
    if (mode == vbhem::kFbBackward && c.bwd4) {
      // fb_bwd4_kernel, persistent: NB blocks per cluster (x8 when possible)
      const int ppb = vbhem::bwd4_ppb();
      const unsigned nt4 = (unsigned)((i_end - i_begin + ppb - 1) / ppb);
      const unsigned all = (unsigned)(vbhem::device_cus() * std::max(1, vbhem::bwd4_resident_blocks()));
      unsigned nb = std::max(1u, std::min(nt4, all / (unsigned)ca.K));
      if (nb >= 8) nb = nb / 8 * 8;
      e = vbhem::launch_bwd4(ca, (unsigned)ca.K * nb, st, ev1 ? ev0 : nullptr, ev1);
      if (e != hipSuccess) return hip_fail(e, "fb_bwd4_kernel");
      g_last_kernel[0] = vbhem::bwd4_o32(ca) ? "vbhem::fb_bwd4_kernel<true>" : "vbhem::fb_bwd4_kernel<false>";
    } else if (mode == vbhem::kFbBackward && c.bwd12) {
      // fb_bwd12_kernel, persistent: NB blocks per cluster (x8 when possible)
      const int ppb = vbhem::bwd12_ppb();
      const unsigned nt12 = (unsigned)((i_end - i_begin + ppb - 1) / ppb);
      const unsigned all = (unsigned)(vbhem::device_cus() * std::max(1, vbhem::bwd12_resident_blocks()));
      unsigned nb = std::max(1u, std::min(nt12, all / (unsigned)ca.K));
      if (nb >= 8) nb = nb / 8 * 8;
      e = vbhem::launch_bwd12(ca, (unsigned)ca.K * nb, st, ev1 ? ev0 : nullptr, ev1);
      if (e != hipSuccess) return hip_fail(e, "fb_bwd12_kernel");
      g_last_kernel[0] = vbhem::bwd12_o32(ca) ? "vbhem::fb_bwd12_kernel<true>" : "vbhem::fb_bwd12_kernel<false>";
    } else if (mode == vbhem::kFbBackward && c.bwd2_lds) {
      // fb_bwd2_kernel, persistent: NB blocks per cluster (x8 when possible)
      ca.nwb = c.bwd2_nwb;
      if (k1) set_k1_operands(c, i_begin, ca);
      if (k1 && c.bwd2_prep) {
        ca.prep = 1;
        ca.pm = c.em.m; ca.pP = c.em.P; ca.pc = c.em.c; ca.pz = c.em.zfix; ca.pshift = c.em.shift;
        ca.ftag = reinterpret_cast<unsigned long long *>(c.fpre);
        ca.ftag_val = vbhem::flag_tag();
      }
      const unsigned nt2 = (unsigned)((i_end - i_begin + c.bwd2_ppb - 1) / c.bwd2_ppb);
      const unsigned all = (unsigned)(vbhem::device_cus() *
                                      std::max(1, vbhem::bwd2_resident_blocks(ca.S, ca.nwb, c.bwd2_lds)));
      unsigned nb = std::max(1u, std::min(nt2, all / (unsigned)ca.K));
      if (nb >= 8) nb = nb / 8 * 8;
      // vbhem_debug_extra_lds(n): n more bytes of dynamic LDS -- fault injection for the
      // tests of a refused launch (tests/test_robustness.py), never set in production
      const size_t lds2 = c.bwd2_lds + g_debug_extra_lds.load(std::memory_order_relaxed);
      e = vbhem::launch_bwd2(ca, (unsigned)ca.K * nb, lds2, st, ev1 ? ev0 : nullptr, ev1);
      if (e != hipSuccess) return hip_fail(e, "fb_bwd2_kernel");
      g_last_kernel[0] = "vbhem::fb_bwd2_kernel<" + std::to_string(ca.S) + ">";
    } else {
      if (mode == vbhem::kFbBackward) {  // persistent: NB blocks per cluster (x8 when possible)
        unsigned nb = std::max(1u, std::min(ntile, list_grid(ca, sp.lds_bwd) / (unsigned)ca.K));
        if (nb >= 8) nb = nb / 8 * 8;
        grid = (unsigned)ca.K * nb;
      }
      e = vbhem::launch_split(ca, grid, mode == vbhem::kFbBackward ? sp.lds_bwd : sp.lds, st);
      if (e != hipSuccess) return hip_fail(e, "fb_split_kernel");
      g_last_kernel[0] = split_name(ca);
    }
  } else {
    const int nib = (i_end - i_begin + a.BI - 1) / a.BI;
    const dim3 grid((unsigned)nib * (unsigned)a.njb);
    e = vbhem::launch_fb(a, grid, c.plan.block, c.plan.lds, st);
    if (e != hipSuccess) return hip_fail(e, "fb_pairs_kernel");
    g_last_kernel[0] = "vbhem::fb_pairs_kernel";
  }
  if (ev0) {
    g_timing.fb.emplace_back(ev0, ev1 ? ev1 : timing_event(st));
    g_timing.fb_pairs.push_back((long long)(i_end - i_begin) * a.K);
  }
  if (fold) {  // resp_kernel takes the flagged pairs (StatsArgs::fold): no exact launch
    *fold = a;
    return VBHEM_OK;
  }
  e = vbhem::launch_fb_exact(a, scratch, exact_stride(a.S, a.SB, a.T), kExactThreads, st);
  if (e != hipSuccess) return hip_fail(e, "fb_exact_kernel");
  return VBHEM_OK;
}

}  // namespace

extern "C" {

const char *vbhem_last_error(void) { return g_err.c_str(); }

size_t vbhem_debug_extra_lds(size_t bytes) { return g_debug_extra_lds.exchange(bytes); }

const char *vbhem_last_kernel(int pass) {
  return (pass == 0 || pass == 1) ? g_last_kernel[pass].c_str() : "";
}

const char *vbhem_version(void) { return "vbhem-mi355x 0.1.0 (gfx950)"; }

size_t vbhem_stats_nu(int d, int covmode) {
  return covmode == VBHEM_COV_FULL ? (size_t)1 + d + (size_t)d * (d + 1) / 2 : (size_t)1 + 2 * d;
}

size_t vbhem_stats_len(int K, int S, int d, int covmode) {
  return (size_t)K + (size_t)K * S + (size_t)K * S * S + 2 + (size_t)K * S * vbhem_stats_nu(d, covmode);
}

size_t vbhem_prepare_base_bytes(const vbhem_base_t *base) {
  if (!base || base->N < 0 || base->SB < 1 || base->d < 1 || base->d > vbhem::kUHead ||
      (base->covmode != VBHEM_COV_DIAG && base->covmode != VBHEM_COV_FULL))
    return 0;
  if (vbhem::emission_kdp(base->d, base->covmode) / 4 > vbhem::kUMaxKq) return 0;
  // the emission GEMM's operand U, then its statistics copy Us (vbhem_internal.h)
  return (vbhem::u_doubles((long long)base->N * base->SB, base->d, base->covmode) +
          vbhem::us_doubles(base->N, base->SB, base->d, base->covmode)) * sizeof(double);
}

int vbhem_prepare_base(const vbhem_base_t *base, double *U_dev, size_t bytes, void *stream) {
  const size_t need = vbhem_prepare_base_bytes(base);
  if (need == 0)
    return fail(VBHEM_ERR_UNSUPPORTED, "vbhem_prepare_base: invalid descriptor or d too large");
  if (!U_dev || bytes < need)
    return fail(VBHEM_ERR_WORKSPACE, "vbhem_prepare_base: need " + std::to_string(need) + " bytes");
  if (base->N > 0 && (!base->centres || !base->covars))
    return fail(VBHEM_ERR_ARG, "vbhem_prepare_base: null base array");
  vbhem::UPrepArgs ua{};
  ua.N = base->N; ua.SB = base->SB; ua.d = base->d; ua.covmode = base->covmode;
  ua.kdp = vbhem::emission_kdp(base->d, base->covmode);
  ua.i_begin = 0; ua.i_end = base->N; ua.u_col0 = 0;
  ua.nstates = base->nstates; ua.centres = base->centres; ua.covars = base->covars;
  ua.U = U_dev; ua.z = nullptr;  // shift = mean of the valid base means
  hipError_t e = vbhem::launch_u_prep(ua, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "u_prep_kernel");
  e = vbhem::launch_us_build(ua, U_dev + vbhem::u_doubles((long long)base->N * base->SB, base->d,
                                                         base->covmode),
                             static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "us_build_kernel");
  return VBHEM_OK;
}

size_t vbhem_pairs_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T) {
  if (check_inputs(base, clus, T, false) != VBHEM_OK) return 0;
  PairsWs w;
  return carve_pairs(nullptr, base, clus, T, true, w);
}

}  // extern "C"

namespace {

int estep_pairs_impl(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T, double smooth,
                     double *LL_elbo_dev, double *sum_nu_1_dev, double *emit_pr_dev,
                     double *emit_mu_dev, double *emit_Mu_dev, double *sum_xi_dev,
                     double *sum_t_nu_dev, void *workspace_dev, size_t workspace_bytes,
                     void *stream) {
  if (!(smooth > 0.0) || !std::isfinite(smooth))
    return fail(VBHEM_ERR_ARG, "smooth must be a positive finite number");
  int rc = check_inputs(base, clus, T);
  if (rc != VBHEM_OK) return rc;
  if (base->N == 0) return VBHEM_OK;
  if (!LL_elbo_dev || !sum_nu_1_dev || !emit_pr_dev || !emit_mu_dev || !emit_Mu_dev || !sum_xi_dev)
    return fail(VBHEM_ERR_ARG, "null output array");
  PairsWs w;
  const size_t need = carve_pairs(nullptr, base, clus, T, sum_t_nu_dev == nullptr, w);
  if (!workspace_dev || workspace_bytes < need)
    return fail(VBHEM_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  carve_pairs(workspace_dev, base, clus, T, sum_t_nu_dev == nullptr, w);
  double *tnu = sum_t_nu_dev ? sum_t_nu_dev : w.tnu;
  hipStream_t st = static_cast<hipStream_t>(stream);
  FbCtx ctx;
  rc = prepare_fb(ctx, base, clus, T, smooth);
  if (rc != VBHEM_OK) return rc;
  ctx.u_ws = w.U;
  if (!ctx.split.ok) {
    hipError_t e0 = hipMemsetAsync(w.fpre, 0, (vbhem::kFlagPre + vbhem::kFlagHead) * sizeof(int), st);
    if (e0 != hipSuccess) return hip_fail(e0, "hipMemsetAsync(flags)");
  }
  rc = run_emission_prep(ctx, w.W, w.bias, w.shift, st, w.fpre, vbhem::kFlagPre + vbhem::kFlagHead);
  if (rc != VBHEM_OK) return rc;
  rc = run_fb(ctx, 0, base->N, 0, LL_elbo_dev, sum_nu_1_dev, sum_xi_dev, tnu, w.E,
              (long long)base->N * base->SB, w.flags,
              w.scratch, st);
  if (rc != VBHEM_OK) return rc;
  vbhem::EmitArgs ea{};
  ea.SB = base->SB; ea.d = base->d; ea.covmode = base->covmode; ea.K = clus->K; ea.S = clus->S;
  ea.i_begin = 0; ea.i_end = base->N;
  ea.centres = base->centres; ea.covars = base->covars; ea.tnu = tnu;
  ea.emit_pr = emit_pr_dev; ea.emit_mu = emit_mu_dev; ea.emit_Mu = emit_Mu_dev;
  hipError_t e = vbhem::launch_emit(ea, st);
  if (e != hipSuccess) return hip_fail(e, "pair_emit_kernel");
  return VBHEM_OK;
}

}  // namespace

extern "C" {

int vbhem_estep_pairs(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      double *LL_elbo_dev, double *sum_nu_1_dev, double *emit_pr_dev,
                      double *emit_mu_dev, double *emit_Mu_dev, double *sum_xi_dev,
                      double *sum_t_nu_dev, void *workspace_dev, size_t workspace_bytes,
                      void *stream) {
  return estep_pairs_impl(base, clus, T, 1.0, LL_elbo_dev, sum_nu_1_dev, emit_pr_dev, emit_mu_dev,
                          emit_Mu_dev, sum_xi_dev, sum_t_nu_dev, workspace_dev, workspace_bytes,
                          stream);
}

int vhem_estep_pairs(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T, double smooth,
                     double *LL_elbo_dev, double *sum_nu_1_dev, double *emit_pr_dev,
                     double *emit_mu_dev, double *emit_Mu_dev, double *sum_xi_dev,
                     double *sum_t_nu_dev, void *workspace_dev, size_t workspace_bytes,
                     void *stream) {
  return estep_pairs_impl(base, clus, T, smooth, LL_elbo_dev, sum_nu_1_dev, emit_pr_dev,
                          emit_mu_dev, emit_Mu_dev, sum_xi_dev, sum_t_nu_dev, workspace_dev,
                          workspace_bytes, stream);
}

size_t vbhem_fused_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T) {
  return vbhem_fused_trials_workspace_bytes(base, clus, 1, T);
}

size_t vbhem_fused_trials_workspace_bytes(const vbhem_base_t *base, const vbhem_cluster_t *clus,
                                          int R, int T) {
  if (check_inputs(base, clus, T, false) != VBHEM_OK || R < 1 || clus->K % R != 0) return 0;
  FusedWs w;
  return carve_fused(nullptr, base, clus, T, w, R);
}

int vbhem_estep_fused(const vbhem_base_t *base, const vbhem_cluster_t *clus, int T,
                      const double *tildeN_dev, const double *logOmega_dev, double *stats_dev,
                      double *hatZ_dev, double *LL_elbo_dev, void *workspace_dev,
                      size_t workspace_bytes, void *stream) {
  return vbhem_estep_fused_trials(base, clus, 1, T, tildeN_dev, logOmega_dev, stats_dev, hatZ_dev,
                                  LL_elbo_dev, workspace_dev, workspace_bytes, stream);
}

// vbhem_arm_done_word: the completion word of the next fused call (taken by that call)
static std::atomic<unsigned long long *> g_done_word{nullptr};
static std::atomic<unsigned long long> g_done_val{0};

int vbhem_arm_done_word(void *word, unsigned long long value) {
  if (word && reinterpret_cast<uintptr_t>(word) % 8 != 0) return fail(VBHEM_ERR_ARG, "done word not 8-byte aligned");
  g_done_val.store(value);
  g_done_word.store(static_cast<unsigned long long *>(word));
  return VBHEM_OK;
}

int vbhem_done_word_alloc(void **host_ptr, void **dev_ptr) {
  if (!host_ptr || !dev_ptr) return fail(VBHEM_ERR_ARG, "null pointer");
  void *h = nullptr;
  hipError_t e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(done word)");
  std::memset(h, 0, 64);
  void *d = nullptr;
  e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return hip_fail(e, "hipHostGetDevicePointer(done word)");
  }
  *host_ptr = h;
  *dev_ptr = d;
  return VBHEM_OK;
}

int vbhem_done_word_free(void *host_ptr) {
  if (!host_ptr) return VBHEM_OK;
  const hipError_t e = hipHostFree(host_ptr);
  return e == hipSuccess ? VBHEM_OK : hip_fail(e, "hipHostFree(done word)");
}

int vbhem_estep_fused_trials(const vbhem_base_t *base, const vbhem_cluster_t *clus, int R, int T,
                             const double *tildeN_dev, const double *logOmega_dev,
                             double *stats_dev, double *hatZ_dev, double *LL_elbo_dev,
                             void *workspace_dev, size_t workspace_bytes, void *stream) {
  // (taken first: a call that fails leaves nothing armed for the next one)
  unsigned long long *const done_word = g_done_word.exchange(nullptr);
  const unsigned long long done_val = g_done_val.load();
  int rc = check_inputs(base, clus, T);
  if (rc != VBHEM_OK) return rc;
  if (R < 1 || clus->K % R != 0)
    return fail(VBHEM_ERR_ARG, "trials: K must be a positive multiple of R");
  if (R > 1 && clus->K > 256)
    return fail(VBHEM_ERR_UNSUPPORTED, "trials: at most 256 clusters in total (R * K_trial)");
  if (!logOmega_dev || !stats_dev ||
      (base->N > 0 && (!tildeN_dev || !hatZ_dev || !LL_elbo_dev)))
    return fail(VBHEM_ERR_ARG, "null fused argument");
  if (vbhem::resp_lds(clus->K, clus->K / R) > kLdsLimit)
    return fail(VBHEM_ERR_UNSUPPORTED, "fused: too many clusters for the responsibilities "
                                       "kernel (K <= ~2,400)");
  FusedWs w;
  const size_t need = carve_fused(nullptr, base, clus, T, w, R);
  if (!workspace_dev || workspace_bytes < need)
    return fail(VBHEM_ERR_WORKSPACE, "workspace too small: need " + std::to_string(need) + " bytes");
  carve_fused(workspace_dev, base, clus, T, w, R);
  hipStream_t st = static_cast<hipStream_t>(stream);

  // statistics kernels' geometry
  const int K = clus->K, S = clus->S, SB = base->SB, d = base->d;
  vbhem::StatsArgs sa{};
  sa.K = K; sa.S = S; sa.SB = SB; sa.d = d; sa.covmode = base->covmode;
  sa.NU = (int)vbhem_stats_nu(d, base->covmode);
  sa.slab_len = w.slab_len;
  sa.KT = K / R;
  sa.SL = w.slab_len / R;
  sa.centres = base->centres; sa.covars = base->covars; sa.LL = LL_elbo_dev;
  sa.nu1 = w.nu1; sa.xi = w.xi; sa.tnu = w.tnu; sa.tildeN = tildeN_dev; sa.logOmega = logOmega_dev;
  sa.Z = w.Z; sa.hatZ = hatZ_dev; sa.slabs = w.slabs;
  size_t slds = 0;
  int ngroups = 1;
  const bool dense_ok = vbhem::plan_stats(sa, slds, ngroups);  // dense-schedule statistics

  FbCtx ctx;
  rc = prepare_fb(ctx, base, clus, T);
  if (rc != VBHEM_OK) return rc;
  ctx.u_ws = w.U;
  // gated schedule: split kernel + list statistics tile must apply
  size_t sl_lds = 0;
  // (gate lists: per-wave ballot masks of all K clusters in LDS, K up to ~2,400)
  const bool gated = g_fused_mode == VBHEM_FUSED_GATED && ctx.split.ok && ctx.split.lds_l &&
                     vbhem::plan_stats_list(sa, sl_lds) &&
                     vbhem::gate_list_lds(K) <= kLdsLimit;
  if (R > 1 && !gated)
    return fail(VBHEM_ERR_UNSUPPORTED,
                "trials need the gated schedule (split-kernel shapes: S <= 16, Sb <= S)");
  if (!gated && !dense_ok)
    return fail(VBHEM_ERR_UNSUPPORTED, "statistics tile does not fit (S or d too large)");
  sa.gate_cnt = gated ? w.gate_cnt : nullptr;
  sa.list = w.list; sa.list_tot = w.list_tot; sa.list_cap = w.group;
  // chunks of >= kChunkMinBases bases; the first group has the most, and in the
  // gated schedule its kernels write (not add to) every entry of slabs [0, nslab_used)
  auto chunks = [&w](int nb) { return std::min(w.nslab, (nb + kChunkMinBases - 1) / kChunkMinBases); };
  const int nslab_used = std::max(1, chunks(std::min(base->N, w.group)));
  // the MFMA statistics kernel: at most 128 parts per cluster (stats_final_kernel then
  // sums 128 slabs of the N1 / M / U columns instead of every chunk's: C4 28 -> 7 MB)
  sa.nzero_m = std::min(nslab_used, 128);
  int stats_slabs = nslab_used;
  hipError_t e = hipSuccess;
  if (!gated || base->N == 0) {
    e = hipMemsetAsync(w.slabs, 0, sizeof(double) * (size_t)nslab_used * w.slab_len, st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(slabs)");
  }
  // a call that returns early leaves the flag head zeroed (tag included): the next
  // call's in-kernel preparation then zeroes the counters itself
  struct HeadGuard {
    int *fpre;
    hipStream_t st;
    ~HeadGuard() {
      if (fpre) (void)hipMemsetAsync(fpre, 0, (vbhem::kFlagPre + vbhem::kFlagHead) * sizeof(int), st);
    }
  } guard{w.fpre, st};
  if (!ctx.split.ok) {
    e = hipMemsetAsync(w.fpre, 0, (vbhem::kFlagPre + vbhem::kFlagHead) * sizeof(int), st);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(flags)");
  }
  if (gated) ctx.bwd.a.Atg = w.Atg;
  // K1 inside fb_bwd2_kernel on a prepared operand: W' / bias' / A' and the counters'
  // reset inside that kernel too (no emission_prep_kernel launch)
  // (thread 448 of the block runs the flag-head handshake: blocks of >= 8 waves only;
  // smaller ones, e.g. a VBHEM_BWD2_WAVES build, take the emission_prep_kernel path)
  if (gated && ctx.k1_in_kernel && ctx.em.zfix && ctx.bwd2_nwb * 64 >= 512 &&
      !std::getenv("VBHEM_NO_BWD2_PREP")) {
    ctx.em.W = w.W; ctx.em.bias = w.bias; ctx.em.shift = w.shift;
    ctx.bwd2_prep = true;
    ctx.fpre = w.fpre;
  } else {
    rc = run_emission_prep(ctx, w.W, w.bias, w.shift, st, w.fpre, vbhem::kFlagPre + vbhem::kFlagHead,
                           gated ? w.Atg : nullptr, clus->logA);
    if (rc != VBHEM_OK) return rc;
  }
  // the backward pass's exact fallback folded into resp_kernel (one base group, one
  // trial: one fb_exact_kernel launch less per E-step; the gate-list pass's flags get
  // their launch in launch_stats_list, from flag_count[3]); resp_kernel needs a
  // scratch slot per chunk block: at most kExactThreads chunks
  const bool fold = gated && R == 1 && base->N <= w.group && ctx.split.ok && K < kExactThreads &&
                    w.nslab <= kExactThreads && !std::getenv("VBHEM_NO_FOLD_EXACT");
  sa.fold = 0;
  for (int g0 = 0; g0 < base->N; g0 += w.group) {
    const int g1 = std::min(base->N, g0 + w.group);
    const long long e_ld = (long long)w.group * SB;
    rc = run_fb(ctx, g0, g1, g0, LL_elbo_dev, w.nu1, w.xi, w.tnu, w.E, e_ld, w.flags, w.scratch,
                st, gated ? vbhem::kFbBackward : vbhem::kFbDense, fold ? &sa.fx : nullptr);
    if (rc != VBHEM_OK) return rc;
    if (fold) {
      sa.fold = 1;
      sa.xscratch = w.scratch;
      sa.xstride = (long long)exact_stride(S, SB, T);
      sa.xslots = kExactThreads;
    }
    sa.i_begin = g0; sa.i_end = g1; sa.i_buf0 = g0;
    sa.assign = gated && g0 == 0;
    // the emission GEMM's operand for this group (prepared, or built by run_fb)
    sa.U = nullptr;
    sa.Us = nullptr;
    if (ctx.split.ok && ctx.use_u) {
      sa.ukdp = ctx.em.kdp;
      if (base->U) {
        sa.U = base->U; sa.uz = base->U; sa.u_col0 = 0;
        sa.Us = base->U + vbhem::u_doubles((long long)base->N * SB, base->d, base->covmode);
      } else if (ctx.u_ws) {
        sa.U = ctx.u_ws; sa.uz = ctx.em.shift; sa.u_col0 = (long long)g0 * SB / 16 * 16;
      }
    }
    const int nchunk = std::max(1, chunks(g1 - g0));
    hipEvent_t ev0 = timing_on(st) ? timing_event(st) : nullptr;
    e = vbhem::launch_resp(sa, nchunk, st);
    if (e != hipSuccess) return hip_fail(e, "resp_kernel");
    if (gated) {
      e = vbhem::launch_gate_list(sa, nchunk, st);
      if (e != hipSuccess) return hip_fail(e, "gate_list_kernel");
      if (ev0) g_timing.stats.emplace_back(ev0, timing_event(st));
      bool inl = false;
      rc = run_fb_list(ctx, g0, g1, g0, w.nu1, w.xi, w.tnu, w.E, e_ld, w.list, w.list_tot,
                       w.group, w.flags, w.scratch, LL_elbo_dev, st, fold, &inl);
      if (rc != VBHEM_OK) return rc;
      if (fold) sa.fold = inl ? 2 : 1;  // 2: no fb_exact_kernel launch before the statistics
      ev0 = timing_on(st) ? timing_event(st) : nullptr;
      int ss = nchunk;
      e = vbhem::launch_stats_list(sa, nchunk, sl_lds, st, &ss);
      if (e != hipSuccess) return hip_fail(e, "stats_list_kernel");
      if (g0 == 0) stats_slabs = ss;  // later groups add into [0, ss) with ss <= this
    } else {
      e = vbhem::launch_stats(sa, nchunk, ngroups, slds, st);
      if (e != hipSuccess) return hip_fail(e, "stats_kernel");
    }
    if (ev0) g_timing.stats.emplace_back(ev0, timing_event(st));
  }
  e = vbhem::launch_stats_final(w.slabs, nslab_used, stats_slabs, w.slab_len, sa.KT, S, sa.SL,
                                stats_dev, st, w.fpre, done_word, done_val);
  if (e != hipSuccess) return hip_fail(e, "stats_final_kernel");
  guard.fpre = nullptr;
  return VBHEM_OK;
}

int vbhem_set_fused_mode(int mode) {
  const int prev = g_fused_mode;
  if (mode == VBHEM_FUSED_GATED || mode == VBHEM_FUSED_DENSE) g_fused_mode = mode;
  return prev;
}

int vbhem_timing_enable(int on) {
  g_timing.level = (on == 1 || on == 2) ? on : 0;
  return VBHEM_OK;
}

int vbhem_timing_read(double *fb_ms, long long *fb_launches, long long *fb_pairs, double *stats_ms,
                      long long *stats_launches) {
  double f = 0.0, s = 0.0;
  long long np = 0;
  int rc = VBHEM_OK;
  auto drain = [&rc](std::vector<std::pair<hipEvent_t, hipEvent_t>> &v, double &acc) {
    for (auto &pr : v) {
      float ms = 0.f;
      if (pr.first && pr.second) {
        hipError_t e = hipEventSynchronize(pr.second);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, pr.first, pr.second);
        if (e != hipSuccess) rc = hip_fail(e, "vbhem_timing_read");
        acc += ms;
      }
      timing_recycle(pr.first);
      timing_recycle(pr.second);
    }
  };
  const long long nf = (long long)g_timing.fb.size(), ns = (long long)g_timing.stats.size();
  drain(g_timing.fb, f);
  drain(g_timing.stats, s);
  for (long long x : g_timing.fb_pairs) np += x;
  g_timing.fb.clear();
  g_timing.stats.clear();
  g_timing.fb_pairs.clear();
  if (fb_ms) *fb_ms = f;
  if (fb_launches) *fb_launches = nf;
  if (fb_pairs) *fb_pairs = np;
  if (stats_ms) *stats_ms = s;
  if (stats_launches) *stats_launches = ns;
  return rc;
}

static int drain_events(std::vector<std::pair<hipEvent_t, hipEvent_t>> &v, double *ms_out,
                        long long *n_out, const char *where) {
  double t = 0.0;
  int rc = VBHEM_OK;
  const long long n = (long long)v.size();
  for (auto &pr : v) {
    float ms = 0.f;
    if (pr.first && pr.second) {
      hipError_t e = hipEventSynchronize(pr.second);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, pr.first, pr.second);
      if (e != hipSuccess) rc = hip_fail(e, where);
      t += ms;
    }
    timing_recycle(pr.first);
    timing_recycle(pr.second);
  }
  v.clear();
  if (ms_out) *ms_out = t;
  if (n_out) *n_out = n;
  return rc;
}

int vbhem_timing_read_em_math(double *ms, long long *launches) {
  return drain_events(g_timing.emd, ms, launches, "vbhem_timing_read_em_math");
}

int vbhem_timing_read_gated(double *fwd_ms, long long *fwd_launches) {
  return drain_events(g_timing.gf, fwd_ms, fwd_launches, "vbhem_timing_read_gated");
}

int vbhem_timing_read_emission(double *em_ms, long long *em_launches) {
  double t = 0.0;
  int rc = VBHEM_OK;
  const long long n = (long long)g_timing.em.size();
  for (auto &pr : g_timing.em) {
    float ms = 0.f;
    if (pr.first && pr.second) {
      hipError_t e = hipEventSynchronize(pr.second);
      if (e == hipSuccess) e = hipEventElapsedTime(&ms, pr.first, pr.second);
      if (e != hipSuccess) rc = hip_fail(e, "vbhem_timing_read_emission");
      t += ms;
    }
    timing_recycle(pr.first);
    timing_recycle(pr.second);
  }
  g_timing.em.clear();
  if (em_ms) *em_ms = t;
  if (em_launches) *em_launches = n;
  return rc;
}

int vbhem_last_fallback_count(void *stream, const void *workspace_dev) {
  // the flag head leads the workspace (vbhem_internal.h kFlagPre): a fused call
  // leaves its total in [2] and the counters zeroed; the pairs path zeroes [2] and
  // leaves its count in the counters ([1] the total, [0] the last pass's)
  int v[vbhem::kFlagPre + 2] = {0};
  if (!workspace_dev) return fail(VBHEM_ERR_ARG, "null workspace");
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipError_t e = hipMemcpyAsync(v, workspace_dev, sizeof(v), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "vbhem_last_fallback_count");
  if (v[vbhem::kFlagLost] == vbhem::kFlagLostMark)
    return fail(VBHEM_ERR_WORKSPACE, "fb_bwd2_kernel lost the flag-head handshake: the fused "
                                     "call's statistics are NaN (results untrusted)");
  return std::max(v[2], std::max(v[vbhem::kFlagPre], v[vbhem::kFlagPre + 1]));
}

int vbhem_host_device_pointer(void *host_ptr, void **dev_ptr) {
  if (!host_ptr || !dev_ptr) return fail(VBHEM_ERR_ARG, "null pointer");
  *dev_ptr = nullptr;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, host_ptr) != hipSuccess || at.type != hipMemoryTypeHost) {
    (void)hipGetLastError();
    return fail(VBHEM_ERR_ARG, "not pinned host memory");
  }
  void *d = nullptr;
  hipError_t e = hipHostGetDevicePointer(&d, host_ptr, 0);
  if (e != hipSuccess || !d) {
    (void)hipGetLastError();
    return fail(VBHEM_ERR_ARG, "pinned host memory is not mapped for the device");
  }
  *dev_ptr = d;
  return VBHEM_OK;
}

}  // extern "C"

namespace {

int estep_pairs_host_impl(int device, const vbhem_base_t *bh, const vbhem_cluster_t *ch, int T,
                          double smooth, double *LL_elbo, double *sum_nu_1, double *emit_pr,
                          double *emit_mu, double *emit_Mu, double *sum_xi) {
  int rc = check_inputs(bh, ch, T);
  if (rc != VBHEM_OK) return rc;
  if (bh->N == 0) return VBHEM_OK;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  const size_t N = bh->N, SB = bh->SB, d = bh->d, K = ch->K, S = ch->S;
  const size_t dC = bh->covmode == VBHEM_COV_FULL ? d * d : d;
  const size_t n_in[] = {N * SB, N * SB * SB, N * SB * d, N * SB * dC,
                         K * S * S, K * S, K * S * d, K * S * dC, K * S};
  const double *h_in[] = {bh->prior, bh->A, bh->centres, bh->covars,
                          ch->logA, ch->logPi, ch->m, ch->P, ch->c};
  const size_t n_out[] = {N * K, N * K * S, N * K * S, N * K * S * d, N * K * S * dC, N * K * S * S};
  double *h_out[] = {LL_elbo, sum_nu_1, emit_pr, emit_mu, emit_Mu, sum_xi};
  double *d_in[9] = {nullptr};
  double *d_out[6] = {nullptr};
  void *ws = nullptr;
  rc = VBHEM_OK;
  for (int k = 0; k < 9 && rc == VBHEM_OK; ++k) {
    e = hipMalloc(&d_in[k], std::max<size_t>(1, n_in[k]) * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(d_in[k], h_in[k], n_in[k] * sizeof(double), hipMemcpyHostToDevice);
    if (e != hipSuccess) rc = hip_fail(e, "upload");
  }
  for (int k = 0; k < 6 && rc == VBHEM_OK; ++k) {
    e = hipMalloc(&d_out[k], std::max<size_t>(1, n_out[k]) * sizeof(double));
    if (e != hipSuccess) rc = hip_fail(e, "hipMalloc(out)");
  }
  vbhem_base_t bd = *bh;
  vbhem_cluster_t cd = *ch;
  bd.nstates = nullptr;
  bd.U = nullptr;  // host entry point: the call builds its own operand
  bd.prior = d_in[0]; bd.A = d_in[1]; bd.centres = d_in[2]; bd.covars = d_in[3];
  cd.logA = d_in[4]; cd.logPi = d_in[5]; cd.m = d_in[6]; cd.P = d_in[7]; cd.c = d_in[8];
  size_t wsb = 0;
  if (rc == VBHEM_OK) {
    wsb = vbhem_pairs_workspace_bytes(&bd, &cd, T);
    e = hipMalloc(&ws, wsb);
    if (e != hipSuccess) rc = hip_fail(e, "hipMalloc(workspace)");
  }
  if (rc == VBHEM_OK)
    rc = estep_pairs_impl(&bd, &cd, T, smooth, d_out[0], d_out[1], d_out[2], d_out[3], d_out[4],
                          d_out[5], nullptr, ws, wsb, nullptr);
  if (rc == VBHEM_OK) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = hip_fail(e, "kernel execution");
  }
  for (int k = 0; k < 6 && rc == VBHEM_OK; ++k) {
    e = hipMemcpy(h_out[k], d_out[k], n_out[k] * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) rc = hip_fail(e, "download");
  }
  for (int k = 0; k < 9; ++k) if (d_in[k]) (void)hipFree(d_in[k]);
  for (int k = 0; k < 6; ++k) if (d_out[k]) (void)hipFree(d_out[k]);
  if (ws) (void)hipFree(ws);
  return rc;
}

}  // namespace

extern "C" {

int vbhem_estep_pairs_host(int device, const vbhem_base_t *bh, const vbhem_cluster_t *ch, int T,
                           double *LL_elbo, double *sum_nu_1, double *emit_pr, double *emit_mu,
                           double *emit_Mu, double *sum_xi) {
  return estep_pairs_host_impl(device, bh, ch, T, 1.0, LL_elbo, sum_nu_1, emit_pr, emit_mu,
                               emit_Mu, sum_xi);
}

int vhem_estep_pairs_host(int device, const vbhem_base_t *bh, const vbhem_cluster_t *ch, int T,
                          double smooth, double *LL_elbo, double *sum_nu_1, double *emit_pr,
                          double *emit_mu, double *emit_Mu, double *sum_xi) {
  return estep_pairs_host_impl(device, bh, ch, T, smooth, LL_elbo, sum_nu_1, emit_pr, emit_mu,
                               emit_Mu, sum_xi);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Host-array fused E-step: a context with the base set resident on a device.
// ---------------------------------------------------------------------------
struct vbhem_ctx {
  int device = 0, N = 0, SB = 0, d = 0, covmode = 0, K = 0, S = 0, R = 1, T = 1;
  size_t stats_len = 0, ws_bytes = 0;
  hipStream_t stream = nullptr;
  int *nstates = nullptr;
  double *prior = nullptr, *A = nullptr, *centres = nullptr, *covars = nullptr;
  double *logA = nullptr, *logPi = nullptr, *m = nullptr, *P = nullptr, *c = nullptr;
  double *tildeN = nullptr, *logOmega = nullptr, *stats = nullptr, *hatZ = nullptr, *LL = nullptr;
  double *U = nullptr;  // the prepared operand of the emission GEMM (vbhem_prepare_base), or null
  void *ws = nullptr;
};

namespace {

void ctx_free(vbhem_ctx *x) {
  if (!x) return;
  int prev = 0;
  const bool dev_ok = hipGetDevice(&prev) == hipSuccess && hipSetDevice(x->device) == hipSuccess;
  void *ptrs[] = {x->nstates, x->prior, x->A, x->centres, x->covars, x->logA, x->logPi, x->m,
                  x->P, x->c, x->tildeN, x->logOmega, x->stats, x->hatZ, x->LL, x->U, x->ws};
  for (void *q : ptrs)
    if (q) (void)hipFree(q);
  if (x->stream) (void)hipStreamDestroy(x->stream);
  if (dev_ok) (void)hipSetDevice(prev);
  delete x;
}

template <class T>
hipError_t dev_alloc(T **p, size_t n) {
  return hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(1, n) * sizeof(T));
}

}  // namespace

extern "C" {

int vbhem_ctx_create(int device, const vbhem_base_t *bh, int K, int S, int R, int T,
                     vbhem_ctx_t **ctx_out) {
  if (!ctx_out) return fail(VBHEM_ERR_ARG, "null context pointer");
  *ctx_out = nullptr;
  vbhem_cluster_t probe{K, S, nullptr, nullptr, nullptr, nullptr, nullptr};
  int rc = check_inputs(bh, &probe, T, false);
  if (rc != VBHEM_OK) return rc;
  if (bh->N > 0 && (!bh->prior || !bh->A || !bh->centres || !bh->covars))
    return fail(VBHEM_ERR_ARG, "null base array");
  if (R < 1 || K % R != 0) return fail(VBHEM_ERR_ARG, "trials: K must be a positive multiple of R");
  vbhem_ctx *x = new vbhem_ctx;
  x->device = device; x->N = bh->N; x->SB = bh->SB; x->d = bh->d; x->covmode = bh->covmode;
  x->K = K; x->S = S; x->R = R; x->T = T;
  x->stats_len = (size_t)R * vbhem_stats_len(K / R, S, bh->d, bh->covmode);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { ctx_free(x); return hip_fail(e, "hipSetDevice"); }
  e = hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking);
  const size_t N = bh->N, SB = bh->SB, d = bh->d;
  const size_t dC = bh->covmode == VBHEM_COV_FULL ? d * d : d;
  if (e == hipSuccess) e = dev_alloc(&x->nstates, N);
  if (e == hipSuccess) e = dev_alloc(&x->prior, N * SB);
  if (e == hipSuccess) e = dev_alloc(&x->A, N * SB * SB);
  if (e == hipSuccess) e = dev_alloc(&x->centres, N * SB * d);
  if (e == hipSuccess) e = dev_alloc(&x->covars, N * SB * dC);
  if (e == hipSuccess) e = dev_alloc(&x->logA, (size_t)K * S * S);
  if (e == hipSuccess) e = dev_alloc(&x->logPi, (size_t)K * S);
  if (e == hipSuccess) e = dev_alloc(&x->m, (size_t)K * S * d);
  if (e == hipSuccess) e = dev_alloc(&x->P, (size_t)K * S * dC);
  if (e == hipSuccess) e = dev_alloc(&x->c, (size_t)K * S);
  if (e == hipSuccess) e = dev_alloc(&x->tildeN, N);
  if (e == hipSuccess) e = dev_alloc(&x->logOmega, (size_t)K);
  if (e == hipSuccess) e = dev_alloc(&x->stats, x->stats_len);
  if (e == hipSuccess) e = dev_alloc(&x->hatZ, N * K);
  if (e == hipSuccess) e = dev_alloc(&x->LL, N * K);
  if (e != hipSuccess) { ctx_free(x); return hip_fail(e, "vbhem_ctx_create(alloc)"); }
  if (N > 0) {
    if (bh->nstates) {
      e = hipMemcpy(x->nstates, bh->nstates, N * sizeof(int), hipMemcpyHostToDevice);
    } else {
      std::vector<int> ns(N, (int)SB);
      e = hipMemcpy(x->nstates, ns.data(), N * sizeof(int), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMemcpy(x->prior, bh->prior, N * SB * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(x->A, bh->A, N * SB * SB * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(x->centres, bh->centres, N * SB * d * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(x->covars, bh->covars, N * SB * dC * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) { ctx_free(x); return hip_fail(e, "vbhem_ctx_create(upload)"); }
  }
  vbhem_base_t bd{bh->N, bh->SB, bh->d, bh->covmode, x->nstates, x->prior, x->A, x->centres,
                  x->covars, nullptr};
  // the base set stays resident: its emission-GEMM operand is built once, here
  if (const size_t ub = vbhem_prepare_base_bytes(&bd)) {
    e = hipMalloc(&x->U, ub);
    if (e != hipSuccess) { ctx_free(x); return hip_fail(e, "vbhem_ctx_create(U)"); }
    rc = vbhem_prepare_base(&bd, x->U, ub, x->stream);
    if (rc != VBHEM_OK) { ctx_free(x); return rc; }
    bd.U = x->U;
  }
  vbhem_cluster_t cd{K, S, x->logA, x->logPi, x->m, x->P, x->c};
  x->ws_bytes = vbhem_fused_trials_workspace_bytes(&bd, &cd, R, T);
  if (x->ws_bytes == 0) { ctx_free(x); return fail(VBHEM_ERR_ARG, "vbhem_ctx_create: bad sizes"); }
  e = hipMalloc(&x->ws, x->ws_bytes);
  if (e != hipSuccess) { ctx_free(x); return hip_fail(e, "vbhem_ctx_create(workspace)"); }
  *ctx_out = x;
  return VBHEM_OK;
}

int vbhem_ctx_fused(vbhem_ctx_t *x, const vbhem_cluster_t *ch, const double *tildeN_host,
                    const double *logOmega_host, double *stats_host, double *hatZ_host,
                    double *LL_host) {
  if (!x || !ch) return fail(VBHEM_ERR_ARG, "null context or cluster descriptor");
  if (ch->K != x->K || ch->S != x->S)
    return fail(VBHEM_ERR_ARG, "cluster descriptor K/S differ from the context's");
  if (!ch->logA || !ch->logPi || !ch->m || !ch->P || !ch->c || !logOmega_host || !stats_host ||
      (x->N > 0 && !tildeN_host))
    return fail(VBHEM_ERR_ARG, "null host array");
  hipError_t e = hipSetDevice(x->device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  const size_t K = x->K, S = x->S, d = x->d, N = x->N;
  const size_t dC = x->covmode == VBHEM_COV_FULL ? d * d : d;
  hipStream_t st = x->stream;
  e = hipMemcpyAsync(x->logA, ch->logA, K * S * S * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(x->logPi, ch->logPi, K * S * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(x->m, ch->m, K * S * d * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(x->P, ch->P, K * S * dC * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(x->c, ch->c, K * S * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(x->logOmega, logOmega_host, K * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && N > 0)
    e = hipMemcpyAsync(x->tildeN, tildeN_host, N * 8, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "vbhem_ctx_fused(upload)");
  vbhem_base_t bd{x->N, x->SB, x->d, x->covmode, x->nstates, x->prior, x->A, x->centres,
                  x->covars, x->U};
  vbhem_cluster_t cd{x->K, x->S, x->logA, x->logPi, x->m, x->P, x->c};
  int rc = vbhem_estep_fused_trials(&bd, &cd, x->R, x->T, x->tildeN, x->logOmega, x->stats,
                                    x->hatZ, x->LL, x->ws, x->ws_bytes, st);
  if (rc != VBHEM_OK) return rc;
  e = hipMemcpyAsync(stats_host, x->stats, x->stats_len * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && hatZ_host && N > 0)
    e = hipMemcpyAsync(hatZ_host, x->hatZ, N * K * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && LL_host && N > 0)
    e = hipMemcpyAsync(LL_host, x->LL, N * K * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "vbhem_ctx_fused(download)");
  return VBHEM_OK;
}

void vbhem_ctx_destroy(vbhem_ctx_t *x) { ctx_free(x); }

int vbhem_estep_fused_host(int device, const vbhem_base_t *bh, const vbhem_cluster_t *ch, int T,
                           const double *tildeN_host, const double *logOmega_host,
                           double *stats_host, double *hatZ_host, double *LL_host) {
  if (!ch) return fail(VBHEM_ERR_ARG, "null cluster descriptor");
  vbhem_ctx_t *x = nullptr;
  int rc = vbhem_ctx_create(device, bh, ch->K, ch->S, 1, T, &x);
  if (rc != VBHEM_OK) return rc;
  rc = vbhem_ctx_fused(x, ch, tildeN_host, logOmega_host, stats_host, hatZ_host, LL_host);
  vbhem_ctx_destroy(x);
  return rc;
}

}  // extern "C"

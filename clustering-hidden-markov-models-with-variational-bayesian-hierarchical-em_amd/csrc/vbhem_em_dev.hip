// vbhem_em_dev.hip -- the per-iteration host math of the EM loop, on the device.
//
// vbhem_h3m_c_step_fc.m runs, between two E-steps, the lower bound (vbhemh3m_lb.m:
// 64-186), the M-step (vbhem_compute_Statistics.m:57-82, vbhem_mstep_component.m:
// 42-70, :396) and the next iteration's psi prelude (:118-165, 180-191, 271-273).
// vbhem_em.hip has them in C++ on the host; here the same arithmetic is ONE kernel on
// the E-step's stream, so an EM iteration never leaves the GPU: the packed
// statistics are read where the statistics kernel (and the all-reduce) left them,
// the prelude writes the next E-step's cluster constants in place, and only the
// bound (one double) goes to the host, for the convergence test.
//
// em_iter_kernel: one WAVEFRONT per cluster state (k, s).  Each does, with its
// lanes working in parallel:
//   1. the (k, s) terms of the bound for the current posterior (lgammas over the
//      lanes, the quadratic forms over lanes = matrix entries), written as partial
//      sums; the last wave to finish (a ticket counter) reduces all of them in a
//      fixed order and writes L (deterministic);
//   2. the M-step of (k, s) into the other posterior buffer: the d x d inverse of
//      W0^-1 + Nr SC + mult1 dd' by Gauss-Jordan elimination without row exchanges
//      (the operand is symmetric positive definite; see gauss_jordan) in
//      wave-private LDS, lanes = entries of [A | I];
//   3. the prelude of the new (k, s): logLambdaTilde (psi over the lanes, det W by
//      the same elimination), c, P = v W, m, its logATilde row, logPiTilde and (one
//      wave per cluster) logOmega -- the sums over a cluster's states or over all
//      clusters are recomputed by every wave that needs them, in one fixed order.
// A prelude-only launch (no bound, no M-step) starts the loop.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vbhem_em_dev.h"

namespace vbhem {

namespace {

constexpr double kPiD = 3.14159265358979323846;
constexpr double kLn2D = 0.69314718055994530942;
constexpr int kWaves = 4;  // waves (cluster states) per block

// digamma for x > 0 (the host routine's series): psi(x) = psi(x + n) -
// sum_{i<n} 1/(x + i) with x + n >= 8, the sum as ONE division of a running
// numerator / denominator (fp64 division is a long dependent sequence on the GPU),
// then ln z - 1/(2z) - sum B_2k / (2k z^2k)
__device__ double psi_dev(double x) {
  if (!(x > 0.0 && x < INFINITY)) return x == INFINITY ? x : __builtin_nan("");
  double num = 0.0, den = 1.0;
  while (x < 8.0) {  // num / den = sum 1/(x_i) so far
    num = fma(num, x, den);
    den *= x;
    x += 1.0;
  }
  const double r = 1.0 / x, r2 = r * r;
  const double series =
      r2 * (1.0 / 12 - r2 * (1.0 / 120 - r2 * (1.0 / 252 - r2 * (1.0 / 240 - r2 * (1.0 / 132 -
      r2 * (691.0 / 32760 - r2 * (1.0 / 12)))))));
  return log(x) - 0.5 * r - series - num / den;
}

// log Gamma for x > 0: lgamma(x) = lgamma(x + n) - log(prod_{i<n} (x + i)) with
// z = x + n >= 10, then Stirling's series (z - 1/2) ln z - z + ln(2 pi)/2 +
// sum B_2k / (2k (2k - 1) z^(2k-1)) through z^-15 (next term < 3e-18 at z = 10)
__device__ double lgamma_dev(double x) {
  if (!(x > 0.0 && x < INFINITY)) return x == INFINITY ? x : __builtin_nan("");
  double prod = 1.0;
  while (x < 10.0) {
    prod *= x;
    x += 1.0;
  }
  const double r = 1.0 / x, r2 = r * r;
  const double series =
      r * (1.0 / 12 - r2 * (1.0 / 360 - r2 * (1.0 / 1260 - r2 * (1.0 / 1680 - r2 * (1.0 / 1188 -
      r2 * (691.0 / 360360 - r2 * (1.0 / 156 - r2 * (3617.0 / 122400))))))));
  return (x - 0.5) * log(x) - x + 0.91893853320467274178 + series - log(prod);
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xf, true);
  return __hiloint2double(hi, lo);
}

// fixed-order wavefront sum by DPP (row_shr 1, 2, 4, 8, row_bcast15, row_bcast31:
// the total lands in lane 63), broadcast to every lane; every wave summing the same
// 64 values gets the same result
__device__ __forceinline__ double wsum(double v) {
  v += dpp_d<0x111, 0xf>(v);
  v += dpp_d<0x112, 0xf>(v);
  v += dpp_d<0x114, 0xf>(v);
  v += dpp_d<0x118, 0xf>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
  return __hiloint2double(hi, lo);
}

// Gauss-Jordan elimination of the d x d matrix in g[0 .. d) x [0 .. cols) (row
// stride 2d, wave-private LDS).  cols = 2d with I in the right half on entry: on exit
// the right half holds the inverse; cols = d: the left half only (for the
// determinant).  Returns det (every lane).  Both matrices it is used on are
// symmetric positive definite (Mt = W0^-1 + Nr SC + mult1 dd', and W), so the
// diagonal pivots are positive and need no row exchanges (the host path's LU
// pivots as MATLAB does; the results agree to rounding).  Lanes own the entries
// x = lane + 64 j of the d x cols array (row / column computed once); per step every
// lane reads the pivot, its row's multiplier and the pivot row's entry of its column
// (three independent LDS reads), one reciprocal, one fma per entry.
__device__ __forceinline__ double gauss_jordan(double *g, int d, int cols, int lane) {
  const int w2 = 2 * d, n = d * cols;
  int er[8], ec[8];  // n / 64 <= 8 entries per lane (d <= 16); er < 0: no entry
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int x = lane + 64 * j;
    er[j] = x < n ? x / cols : -1;
    ec[j] = x < n ? x - er[j] * cols : 0;
  }
  double det = 1.0;
  for (int k = 0; k < d; ++k) {
    const double piv = g[k * w2 + k], rp = 1.0 / piv;
    double nv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (er[j] >= 0) {
        const int r = er[j], c = ec[j];
        const double rk = g[k * w2 + c] * rp;  // new pivot row
        nv[j] = r == k ? rk : fma(-g[r * w2 + k], rk, g[r * w2 + c]);
      }
    }
    det *= piv;
    wsync();
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (er[j] >= 0) g[er[j] * w2 + ec[j]] = nv[j];
    wsync();
  }
  return det;
}

// packed statistics (include/vbhem_estep.h): Nj | N1 | M | Lt1 Lt7 | U
struct StatsView {
  const double *Nj, *N1, *M, *U;
  double Lt1, Lt7;
  __device__ StatsView(const double *v, int K, int S) {
    Nj = N1 = M = U = nullptr;
    Lt1 = Lt7 = 0.0;
    if (!v) return;
    size_t o = 0;
    Nj = v + o; o += K;
    N1 = v + o; o += (size_t)K * S;
    M = v + o; o += (size_t)K * S * S;
    Lt1 = v[o];
    Lt7 = v[o + 1];
    o += 2;
    U = v + o;
  }
};

// bound partial sums per (k, s), stored quantity-major [13][K S]: 0 Lt51, 1 lLT, 2 v trW, 3 lt10a, 4 H, 5 Lt9, 6 logPi,
// 7 sum logA row, 8 Lt2, 9 logOmega, 10 Lt8b, 11 lgamma(alpha), 12 alpha
constexpr int kNQ = 13;

#ifdef EMDEV_TIMING
__device__ long long emdev_t[8][1024];  // [phase][wave]: s_memrealtime (100 MHz)
#define EMDEV_MARK(ph)                                                  \
  if (lane == 0 && ks < 1024) emdev_t[ph][ks] = __builtin_amdgcn_s_memrealtime()
#else
#define EMDEV_MARK(ph)
#endif

__global__ __launch_bounds__(64 * kWaves) void em_iter_kernel(const EmDevArgs a, int mode,
                                                              double *L_out) {
  __shared__ double glds[kWaves][2 * kEmDevMaxD * kEmDevMaxD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K = a.K, S = a.S, d = a.d;
  const int ks = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wave);  // wave-uniform
  if (ks >= K * S) return;
  const int k = ks / S, s = ks - k * S;
  const bool full = a.covmode == 1;
  const int dd = full ? d * d : d;
  double *g = glds[wave];
  const bool iterate = mode == kEmIterate;
  // (the view is built in both modes: a.stats is always a valid buffer, so a load
  // the compiler hoists out of an `iterate ? stats : posterior` select cannot fault)
  const StatsView st(a.stats, K, S);
  EMDEV_MARK(0);

  // ---- 1. bound terms of the current posterior (vbhemh3m_lb.m:64-186) ----
  if (iterate) {
    const double v = a.v[ks], lam = a.lam[ks], lLT = a.lLT[ks], l0 = a.lambda0;
    const double *W = a.W + (size_t)ks * dd, *mk = a.m + (size_t)ks * d;
    // the epsilon row on lanes 32 + s2 (and its sum), eta, the cluster's eta sum and
    // alpha_k first, so that every lgamma of the (k, s) terms is one parallel round:
    // lanes q < d lgamma((v + 1 - q) / 2), lanes 32 + s2 lgamma(eps), lanes 16..19
    // lgamma of sum(eps row), eta, sum(eta) and alpha_k (the last two for state 0)
    double t_eps = 0.0, t_ept = 0.0, t_la = 0.0;
    if (lane >= 32 && lane - 32 < S) {
      const int s2 = lane - 32;
      const double la = a.logA[(size_t)ks * S + s2];
      t_eps = a.eps[(size_t)ks * S + s2];
      t_ept = (t_eps - 1) * la;
      t_la = la;
    }
    const double e = a.eta[ks];
    double es = 0.0, lo = 0.0, al = 0.0;
    if (s == 0) {
      es = wsum(lane < S ? a.eta[(size_t)k * S + lane] : 0.0);
      lo = a.logOmega[k];
      al = a.alpha[k];
    }
    const double ps = wsum(t_eps);
    double xg = 0.0;
    bool lg_on = false;
    if (lane < d) {
      xg = 0.5 * (v - lane);
      lg_on = true;
    } else if (lane >= 32 && lane - 32 < S) {
      xg = t_eps;
      lg_on = true;
    } else if (lane >= 16 && lane < 20) {
      xg = lane == 16 ? ps : lane == 17 ? e : lane == 18 ? es : al;
      lg_on = lane < 18 || s == 0;
    }
    const double lgx = lg_on ? lgamma_dev(xg) : 0.0;
    // quadratic forms over the lanes = entries (x, z)
    double t_mwm = 0.0, t_tr = 0.0;
    for (int x = lane; x < d * d; x += 64) {
      const int r = x / d, c = x - r * d;
      const double wrc = full ? W[x] : (r == c ? W[r] : 0.0);
      const double wcr = full ? W[c * d + r] : wrc;
      t_mwm += (mk[r] - a.m0[r]) * wrc * (mk[c] - a.m0[c]);
      t_tr += a.W0inv[x] * wcr;
    }
    const double sg = wsum(lane < d ? lgx : 0.0), lgp = wsum(lane >= 32 ? lgx : 0.0);
    const double pt = wsum(t_ept), sla = wsum(t_la), mWm = wsum(t_mwm), trW = wsum(t_tr);
    const double lg_ps = __shfl(lgx, 16, 64), lg_e = __shfl(lgx, 17, 64);
    const double lg_es = __shfl(lgx, 18, 64), lg_al = __shfl(lgx, 19, 64);
    if (lane < kNQ) {
      const double logBk = -(v / 2) * a.logdetW[ks] - (v * d / 2) * kLn2D -
                           (d * (d - 1) / 4.0) * log(kPiD) - sg;
      double q = 0.0;
      switch (lane) {
        case 0: q = d * log(l0 / (2 * kPiD)) + lLT - d * l0 / lam - l0 * v * mWm; break;
        case 1: q = lLT; break;
        case 2: q = v * trW; break;
        case 3: q = lLT + d * log(lam / (2 * kPiD)); break;
        case 4: q = -logBk - 0.5 * (v - d - 1) * lLT + 0.5 * v * d; break;
        case 5: q = lg_ps - lgp + pt - lg_e + (e - 1) * a.logPi[ks] + (s == 0 ? lg_es : 0.0); break;
        case 6: q = a.logPi[ks]; break;
        case 7: q = sla; break;
        case 8: q = s == 0 ? (st.Nj[k] + 1e-50) * lo : 0.0; break;
        case 9: q = s == 0 ? lo : 0.0; break;
        case 10: q = s == 0 ? (al - 1) * lo : 0.0; break;
        case 11: q = s == 0 ? lg_al : 0.0; break;
        default: q = s == 0 ? al : 0.0; break;
      }
      a.part[(size_t)lane * K * S + ks] = q;  // quantity-major: one lane sums each below
    }
  }

  EMDEV_MARK(1);
  // ---- 2. M-step of (k, s) (vbhem_compute_Statistics.m:57-82, mstep_component.m:42-70) ----
  // Every lane keeps what it needs of the new posterior in registers or in its own
  // LDS entries (no lane reads another lane's global stores): v, lam in all lanes,
  // m_a in lane a, the epsilon row entry s2 in lanes s2 and 32 + s2, W in the left
  // half of g (then [W | I] for its determinant).
  const int w2 = 2 * d;
  double v, lam, m_l = 0.0, e_l = 0.0, eta_ks, sum_eta = 0.0, alpha_k, det_mt = 1.0;
  if (iterate) {
    const double *u = st.U + (size_t)ks * a.NU;
    const double Nr = u[0] + 1e-50, l0 = a.lambda0;
    lam = l0 + Nr;
    v = a.v0 + Nr + 1.0;
    const double mult1 = l0 * Nr / (l0 + Nr);
    // [Mt | I]: Mt = W0^-1 + Nr SC + mult1 (y - m0)(y - m0)', SC = S_plus_C / Nr - y y'
    for (int x = lane; x < d * w2; x += 64) {
      const int r = x / w2, c = x - r * w2;
      double val;
      if (c < d) {
        const double yr = u[1 + r] / Nr, yc = u[1 + c] / Nr;
        double sc;
        if (full) {
          const int lo = r < c ? r : c, hi = r < c ? c : r;
          sc = u[1 + d + lo * d - lo * (lo - 1) / 2 + (hi - lo)] / Nr - yr * yc;
        } else {
          sc = r == c ? u[1 + d + r] / Nr - yr * yr : 0.0;
        }
        val = a.W0inv[r * d + c] + Nr * sc + mult1 * (yr - a.m0[r]) * (yc - a.m0[c]);
      } else {
        val = (c - d == r) ? 1.0 : 0.0;
      }
      g[x] = val;
    }
    if (lane < d) {
      m_l = (l0 * a.m0[lane] + Nr * (u[1 + lane] / Nr)) / (l0 + Nr);
      a.m_o[(size_t)ks * d + lane] = m_l;
    }
    if (lane == 0) {
      a.lam_o[ks] = lam;
      a.v_o[ks] = v;
    }
    wsync();
    EMDEV_MARK(2);
    det_mt = gauss_jordan(g, d, 2 * d, lane);
    EMDEV_MARK(3);
    // W = (tW + tW') / 2, left half of g; right half back to I
    double nw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = lane + 64 * j;
      if (x < d * d) {
        const int r = x / d, c = x - r * d;
        nw[j] = (g[r * w2 + d + c] + g[c * w2 + d + r]) / 2;
      }
    }
    wsync();
    double *Wo = a.W_o + (size_t)ks * dd;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int x = lane + 64 * j;
      if (x < d * d) {
        const int r = x / d, c = x - r * d;
        g[r * w2 + c] = full ? nw[j] : (r == c ? nw[j] : 0.0);
        g[r * w2 + d + c] = r == c ? 1.0 : 0.0;
        if (full) Wo[x] = nw[j];
        else if (r == c) Wo[r] = nw[j];
      }
    }
    eta_ks = a.eta0 + st.N1[ks];
    if (lane < S) sum_eta = a.eta0 + st.N1[(size_t)k * S + lane];
    const int s2 = lane & 31;
    if (s2 < S) {
      e_l = a.epsilon0 + (S > 1 ? st.M[(size_t)ks * S + s2] : 1e-12);
      if (lane < 32) a.eps_o[(size_t)ks * S + s2] = e_l;
    }
    if (lane == 0) a.eta_o[ks] = eta_ks;
    alpha_k = a.alpha0 + (st.Nj[k] + 1e-50);
    if (s == 0 && lane == 0) a.alpha_o[k] = alpha_k;
  } else {
    v = a.v[ks];
    lam = a.lam[ks];
    eta_ks = a.eta[ks];
    if (lane < S) sum_eta = a.eta[(size_t)k * S + lane];
    if (lane < d) m_l = a.m[(size_t)ks * d + lane];
    if ((lane & 31) < S) e_l = a.eps[(size_t)ks * S + (lane & 31)];
    alpha_k = a.alpha[k];
    const double *W = a.W + (size_t)ks * dd;
    for (int x = lane; x < d * w2; x += 64) {
      const int r = x / w2, c = x - r * w2;
      g[x] = c < d ? (full ? W[r * d + c] : (r == c ? W[r] : 0.0)) : ((c - d == r) ? 1.0 : 0.0);
    }
  }
  wsync();
  EMDEV_MARK(4);
  sum_eta = wsum(lane < S ? sum_eta : 0.0);  // the cluster's eta (lanes < S hold them)

  // ---- 3. prelude of (k, s) (step_fc.m:118-165, 180-191, 271-273) ----
  const double es = wsum(lane >= 32 && lane - 32 < S ? e_l : 0.0);
  double sa = 0.0;  // sum_k alpha (state 0's wave): lane-strided partials, one DPP sum
  if (s == 0) {
    double t = 0.0;
    for (int j = lane; j < K; j += 64)
      t += iterate ? a.alpha0 + (st.Nj[j] + 1e-50) : a.alpha[j];
    sa = wsum(t);
  }
  // every psi of (k, s) in one parallel round: lanes q < d psi((v + 1 - q) / 2),
  // lanes 32 + s2 the epsilon row, lanes 16..20 psi of sum(eps row), eta, sum(eta),
  // alpha_k and sum(alpha) (the last two for state 0)
  double xp = 0.0;
  bool p_on = false;
  if (lane < d) {
    xp = 0.5 * (v - lane);
    p_on = true;
  } else if (lane >= 32 && lane - 32 < S) {
    xp = e_l;
    p_on = true;
  } else if (lane >= 16 && lane < 21) {
    xp = lane == 16 ? es : lane == 17 ? eta_ks : lane == 18 ? sum_eta : lane == 19 ? alpha_k : sa;
    p_on = lane < 19 || s == 0;
  }
  const double pl = p_on ? psi_dev(xp) : 0.0;
  const double t1 = wsum(lane < d ? pl : 0.0);
  const double pes = __shfl(pl, 16, 64), pet = __shfl(pl, 17, 64), pst = __shfl(pl, 18, 64);
  const double pal = __shfl(pl, 19, 64), psa = __shfl(pl, 20, 64);
  // P = v W and the diagonal's logs from g's left half, before the elimination
  for (int x = lane; x < dd; x += 64) {
    const int r = full ? x / d : x, c = full ? x - r * d : x;
    a.P[(size_t)ks * dd + x] = v * g[r * w2 + c];
  }
  double logdet;
  if (full && iterate) {
    // W = (inv(Mt) + inv(Mt)') / 2: log det W = -log det Mt (the M-step's
    // elimination; the symmetrisation moves it by rounding only)
    logdet = -log(det_mt);
  } else if (full) {
    wsync();
    logdet = log(gauss_jordan(g, d, d, lane));
  } else {
    logdet = wsum(lane < d ? log(g[lane * w2 + lane]) : 0.0);
  }
  EMDEV_MARK(5);
  const double lLT = t1 + d * kLn2D + logdet;
  if (lane < d) a.cm[(size_t)ks * d + lane] = m_l;
  if (lane >= 32 && lane - 32 < S) a.logA[(size_t)ks * S + (lane - 32)] = pl - pes;
  if (lane == 0) {
    a.lLT[ks] = lLT;
    a.logdetW[ks] = logdet;
    a.c[ks] = -lLT + d / lam;
    a.logPi[ks] = pet - pst;
    if (s == 0) a.logOmega[k] = pal - psa;
  }

  EMDEV_MARK(6);
  // ---- the bound: the last wave reduces every (k, s)'s partial sums ----
  if (iterate) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    int last = 0;
    if (lane == 0) last = atomicAdd(a.ticket, 1) == K * S - 1;
    last = __shfl(last, 0, 64);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      // every lane sums its strided share of each quantity (independent loads),
      // then one fixed-order DPP sum per quantity
      double q[kNQ];
#pragma unroll
      for (int x = 0; x < kNQ; ++x) q[x] = 0.0;
      for (int j = lane; j < K * S; j += 64) {  // the 13 loads of a round in flight together
#pragma unroll
        for (int x = 0; x < kNQ; ++x) q[x] += a.part[(size_t)x * K * S + j];
      }
#pragma unroll
      for (int x = 0; x < kNQ; ++x) q[x] = wsum(q[x]);
      if (lane == 0) {
        const double a0 = a.alpha0, e0 = a.eta0, ep0 = a.epsilon0, v0 = a.v0;
        const double Lt3 = K * a.logCeta0 + (e0 - 1) * q[6];
        const double Lt4 = (double)K * S * a.logCepsilon0 + (ep0 - 1) * q[7];
        const double Lt5 =
            0.5 * q[0] + (double)K * S * a.logB0 + 0.5 * (v0 - d - 1) * q[1] - 0.5 * q[2];
        const double Lt6 = a.logCalpha0 + (a0 - 1) * q[9];
        const double Lt8 = (lgamma_dev(q[12]) - q[11]) + q[10];
        const double Lt10 = 0.5 * q[3] - 0.5 * d * S * K - q[4];
        *L_out = st.Lt1 + q[8] + Lt3 + Lt4 + Lt5 + Lt6 - st.Lt7 - Lt8 - q[5] - Lt10;
        *a.ticket = 0;  // ready for the next launch
        EMDEV_MARK(7);
        if (a.flag) {   // the host polls this word (mapped memory) instead of syncing
          __threadfence_system();
          __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

}  // namespace

bool em_dev_supported(int d, int S) { return d >= 1 && d <= kEmDevMaxD && S >= 1 && S <= 32; }

hipError_t launch_em_dev(const EmDevArgs &a, int mode, double *L_out, hipStream_t st) {
  if (!em_dev_supported(a.d, a.S) || (mode == kEmIterate && (!L_out || !a.ticket || !a.part)))
    return hipErrorInvalidValue;
  const int nw = a.K * a.S;
  hipLaunchKernelGGL(em_iter_kernel, dim3((nw + kWaves - 1) / kWaves), dim3(64 * kWaves), 0, st, a,
                     mode, L_out);
  return hipGetLastError();
}

}  // namespace vbhem

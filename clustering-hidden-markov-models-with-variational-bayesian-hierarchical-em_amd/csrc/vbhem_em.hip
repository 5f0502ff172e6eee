// vbhem_em.hip -- the VBHEM-H3M EM host loop (include/vbhem_em.h), host C++.
//
// Mirrors, per EM iteration, src/vbhem/vbhem_h3m_c_step_fc.m:
//   psi prelude            :118-165, 180-191, 271-273      vbhem_em_prelude
//   E-step (device)        :168-198, 270-296               vbhem_estep_fused
//   lower bound            vbhemh3m_lb.m:64-186            vbhem_em_lower_bound
//   convergence / NaN      :311-374                        vbhem_em_run
//   statistics + M-step    vbhem_compute_Statistics.m:57-82,
//                          vbhem_mstep_component.m:42-70, :396   vbhem_em_mstep
// The arithmetic follows vbhem_amd/host.py (the Python host path, itself checked
// against the oracle's restatement of the MATLAB code); psi is evaluated by
// recurrence to x >= 8 plus the asymptotic series, lgamma is libm's, and the
// d x d inverse / determinant use LU with partial pivoting (as MATLAB's inv/det).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "vbhem_em.h"
#include "vbhem_em_dev.h"
#include "vbhem_internal.h"

namespace {

constexpr double kPi = 3.14159265358979323846;

// digamma for x > 0: psi(x) = psi(x + n) - sum_{k<n} 1/(x + k), then the
// asymptotic expansion ln x - 1/(2x) - sum B_2k / (2k x^2k) at x >= 8.
double psi(double x) {
  if (!(x > 0.0 && x < INFINITY)) return x == INFINITY ? x : std::nan("");
  double acc = 0.0;
  while (x < 8.0) {
    acc -= 1.0 / x;
    x += 1.0;
  }
  const double r = 1.0 / x, r2 = r * r;
  const double series =
      r2 * (1.0 / 12 - r2 * (1.0 / 120 - r2 * (1.0 / 252 - r2 * (1.0 / 240 - r2 * (1.0 / 132 -
      r2 * (691.0 / 32760 - r2 * (1.0 / 12)))))));
  return acc + std::log(x) - 0.5 * r - series;
}

// sum_{q=1..d} psi((v + 1 - q) / 2) (step_fc.m:136): the arguments are two chains
// v/2, v/2 - 1, ... and (v-1)/2, (v-1)/2 - 1, ...; one psi per chain, the rest by
// psi(x - 1) = psi(x) - 1/(x - 1)
double psi_sum_half(double v, int d) {
  double acc = 0.0;
  for (int c = 0; c < 2 && c < d; ++c) {
    double x = 0.5 * (v - c), p = psi(x);
    for (int q = c; q < d; q += 2) {
      acc += p;
      x -= 1.0;
      p -= 1.0 / x;
    }
  }
  return acc;
}

// sum_{q=1..d} lgamma((v + 1 - q) / 2) (vbhemh3m_lb.m:81-83), the same two chains
// with lgamma(x - 1) = lgamma(x) - log(x - 1)
double lgamma_sum_half(double v, int d) {
  double acc = 0.0;
  for (int c = 0; c < 2 && c < d; ++c) {
    double x = 0.5 * (v - c), g = std::lgamma(x);
    for (int q = c; q < d; q += 2) {
      acc += g;
      x -= 1.0;
      if (q + 2 < d) g -= std::log(x);
    }
  }
  return acc;
}

// per-thread scratch of the d x d factorisations (no allocation per matrix)
struct LuScratch {
  std::vector<double> a, x;
  std::vector<int> piv;
  void size(int d) {
    if ((int)piv.size() < d) {
      a.resize((size_t)d * d);
      x.resize((size_t)d);
      piv.resize((size_t)d);
    }
  }
};
thread_local LuScratch tl_lu;

// LU with partial pivoting of a d x d row-major matrix (in place); returns det.
double lu_det(double *a, int d, int *piv) {
  double det = 1.0;
  for (int k = 0; k < d; ++k) {
    int p = k;
    for (int r = k + 1; r < d; ++r)
      if (std::fabs(a[(size_t)r * d + k]) > std::fabs(a[(size_t)p * d + k])) p = r;
    piv[k] = p;
    if (p != k) {
      for (int c = 0; c < d; ++c) std::swap(a[(size_t)k * d + c], a[(size_t)p * d + c]);
      det = -det;
    }
    const double pk = a[(size_t)k * d + k];
    det *= pk;
    if (pk == 0.0) continue;
    for (int r = k + 1; r < d; ++r) {
      const double f = a[(size_t)r * d + k] / pk;
      a[(size_t)r * d + k] = f;
      for (int c = k + 1; c < d; ++c) a[(size_t)r * d + c] -= f * a[(size_t)k * d + c];
    }
  }
  return det;
}

double det_of(const double *m, int d) {
  LuScratch &s = tl_lu;
  s.size(d);
  std::copy(m, m + (size_t)d * d, s.a.begin());
  return lu_det(s.a.data(), d, s.piv.data());
}

// inverse through the LU factors (solve for the identity columns)
void inv_of(const double *m, int d, double *out) {
  LuScratch &s = tl_lu;
  s.size(d);
  double *a = s.a.data(), *x = s.x.data();
  int *piv = s.piv.data();
  std::copy(m, m + (size_t)d * d, a);
  lu_det(a, d, piv);
  for (int col = 0; col < d; ++col) {
    for (int r = 0; r < d; ++r) x[r] = r == col ? 1.0 : 0.0;
    for (int k = 0; k < d; ++k) std::swap(x[k], x[piv[k]]);
    for (int r = 0; r < d; ++r)
      for (int c = 0; c < r; ++c) x[r] -= a[(size_t)r * d + c] * x[c];
    for (int r = d - 1; r >= 0; --r) {
      for (int c = r + 1; c < d; ++c) x[r] -= a[(size_t)r * d + c] * x[c];
      x[r] /= a[(size_t)r * d + r];
    }
    for (int r = 0; r < d; ++r) out[(size_t)r * d + col] = x[r];
  }
}

bool post_ok(const vbhem_post_t *p) {
  return p && p->K >= 1 && p->S >= 1 && p->d >= 1 &&
         (p->covmode == VBHEM_COV_DIAG || p->covmode == VBHEM_COV_FULL) && p->alpha && p->eta &&
         p->epsilon && p->lam && p->v && p->m && p->W;
}

bool opt_ok(const vbhem_em_opt_t *o, int d) {
  return o && o->m0 && o->W0 && (o->W0_len == 1 || o->W0_len == d) && o->max_iter >= 0;
}

// W0 as a full matrix and its inverse (host.py::_W0)
void w0_inv(const vbhem_em_opt_t *o, int d, std::vector<double> &W0inv) {
  std::vector<double> W0((size_t)d * d, 0.0);
  for (int a = 0; a < d; ++a) W0[(size_t)a * d + a] = o->W0_len == 1 ? o->W0[0] : o->W0[a];
  W0inv.assign((size_t)d * d, 0.0);
  inv_of(W0.data(), d, W0inv.data());
}

// packed statistics accessors (include/vbhem_estep.h: Nj | N1 | M | Lt1 Lt7 | U)
struct Stats {
  const double *Nj, *N1, *M, *U;
  double Lt1, Lt7;
  int NU;
  Stats(const double *v, int K, int S, int d, int covmode) {
    NU = (int)vbhem_stats_nu(d, covmode);
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

}  // namespace

extern "C" {

int vbhem_em_prelude(const vbhem_post_t *post, double *logA, double *logPi, double *m, double *P,
                     double *c, double *logLambdaTilde, double *logOmega) {
  if (!post_ok(post) || !logA || !logPi || !m || !P || !c || !logLambdaTilde || !logOmega)
    return VBHEM_ERR_ARG;
  const int K = post->K, S = post->S, d = post->d;
  const bool full = post->covmode == VBHEM_COV_FULL;
  const size_t dd = full ? (size_t)d * d : (size_t)d;
  for (int k = 0; k < K; ++k) {
    for (int s = 0; s < S; ++s) {
      const size_t ks = (size_t)k * S + s;
      const double v = post->v[ks];
      const double t1 = psi_sum_half(v, d);
      const double *W = post->W + ks * dd;
      double logdet;
      if (full) {
        logdet = std::log(det_of(W, d));
      } else {
        logdet = 0.0;
        for (int a = 0; a < d; ++a) logdet += std::log(W[a]);
      }
      const double lLT = t1 + d * std::log(2.0) + logdet;
      logLambdaTilde[ks] = lLT;
      c[ks] = -lLT + d / post->lam[ks];
      for (size_t x = 0; x < dd; ++x) P[ks * dd + x] = v * W[x];
      for (int a = 0; a < d; ++a) m[ks * d + a] = post->m[ks * d + a];
      // logATilde row (step_fc.m:156-157)
      const double *eps = post->epsilon + ks * S;
      double es = 0.0;
      for (int s2 = 0; s2 < S; ++s2) es += eps[s2];
      const double pes = psi(es);
      for (int s2 = 0; s2 < S; ++s2) logA[ks * S + s2] = psi(eps[s2]) - pes;
    }
    double ets = 0.0;
    for (int s = 0; s < S; ++s) ets += post->eta[(size_t)k * S + s];
    const double pet = psi(ets);
    for (int s = 0; s < S; ++s)
      logPi[(size_t)k * S + s] = psi(post->eta[(size_t)k * S + s]) - pet;
  }
  double as = 0.0;
  for (int k = 0; k < K; ++k) as += post->alpha[k];
  const double pas = psi(as);
  for (int k = 0; k < K; ++k) logOmega[k] = psi(post->alpha[k]) - pas;
  return VBHEM_OK;
}

int vbhem_em_lower_bound(const vbhem_post_t *post, const vbhem_em_opt_t *opt,
                         const double *stats, const double *logLambdaTilde, const double *logA,
                         const double *logPi, const double *logOmega, double *L) {
  if (!post_ok(post) || !opt_ok(opt, post->d) || !stats || !logLambdaTilde || !logA || !logPi ||
      !logOmega || !L)
    return VBHEM_ERR_ARG;
  const int K = post->K, S = post->S, d = post->d;
  const bool full = post->covmode == VBHEM_COV_FULL;
  const size_t dd = full ? (size_t)d * d : (size_t)d;
  const Stats st(stats, K, S, d, post->covmode);
  const double a0 = opt->alpha0, e0 = opt->eta0, ep0 = opt->epsilon0, l0 = opt->lambda0,
               v0 = opt->v0;
  std::vector<double> W0inv;
  w0_inv(opt, d, W0inv);
  double logdetW0inv = 0.0;
  if (opt->W0_len == 1) logdetW0inv = d * std::log(W0inv[0]);
  else for (int a = 0; a < d; ++a) logdetW0inv += std::log(W0inv[(size_t)a * d + a]);
  const double sg0 = lgamma_sum_half(v0, d);
  const double logCalpha0 = std::lgamma(K * a0) - K * std::lgamma(a0);
  const double logCeta0 = std::lgamma(S * e0) - S * std::lgamma(e0);
  const double logCepsilon0 = std::lgamma(S * ep0) - S * std::lgamma(ep0);
  const double logB0 = (v0 / 2) * logdetW0inv - (v0 * d / 2) * std::log(2.0) -
                       (d * (d - 1) / 4.0) * std::log(kPi) - sg0;
  const double const2 = d * std::log(l0 / (2 * kPi));
  double asum = 0.0, lga = 0.0;
  for (int k = 0; k < K; ++k) {
    asum += post->alpha[k];
    lga += std::lgamma(post->alpha[k]);
  }
  const double logCalpha = std::lgamma(asum) - lga;
  double Lt2 = 0.0, sumLO = 0.0, Lt8b = 0.0;
  for (int k = 0; k < K; ++k) {
    Lt2 += (st.Nj[k] + 1e-50) * logOmega[k];
    sumLO += logOmega[k];
    Lt8b += (post->alpha[k] - 1) * logOmega[k];
  }
  double sumLPi = 0.0, sumLA = 0.0;
  for (size_t x = 0; x < (size_t)K * S; ++x) sumLPi += logPi[x];
  for (size_t x = 0; x < (size_t)K * S * S; ++x) sumLA += logA[x];
  const double Lt3 = K * logCeta0 + (e0 - 1) * sumLPi;
  const double Lt4 = K * S * logCepsilon0 + (ep0 - 1) * sumLA;
  const double Lt6 = logCalpha0 + (a0 - 1) * sumLO;
  const double Lt8 = logCalpha + Lt8b;
  double Lt5 = 0.0, Lt9 = 0.0, Lt10 = 0.0;
  std::vector<double> Wf((size_t)d * d);
  for (int k = 0; k < K; ++k) {
    double H = 0.0, Lt51 = 0.0, sumLLT = 0.0, sumVtr = 0.0, lt10a = 0.0;
    for (int s = 0; s < S; ++s) {
      const size_t ks = (size_t)k * S + s;
      const double v = post->v[ks], lam = post->lam[ks], lLT = logLambdaTilde[ks];
      const double *W = post->W + ks * dd;
      if (full) {
        for (size_t x = 0; x < dd; ++x) Wf[x] = W[x];
      } else {
        std::fill(Wf.begin(), Wf.end(), 0.0);
        for (int a = 0; a < d; ++a) Wf[(size_t)a * d + a] = W[a];
      }
      const double sg = lgamma_sum_half(v, d);
      const double logBk = -(v / 2) * std::log(det_of(Wf.data(), d)) - (v * d / 2) * std::log(2.0) -
                           (d * (d - 1) / 4.0) * std::log(kPi) - sg;
      H += -logBk - 0.5 * (v - d - 1) * lLT + 0.5 * v * d;
      double mWm = 0.0, trW = 0.0;
      const double *mk = post->m + ks * d;
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) {
          mWm += (mk[a] - opt->m0[a]) * Wf[(size_t)a * d + b] * (mk[b] - opt->m0[b]);
          trW += W0inv[(size_t)a * d + b] * Wf[(size_t)b * d + a];
        }
      Lt51 += const2 + lLT - d * l0 / lam - l0 * v * mWm;
      sumLLT += lLT;
      sumVtr += v * trW;
      lt10a += lLT + d * std::log(lam / (2 * kPi));
    }
    Lt5 += 0.5 * Lt51 + S * logB0 + 0.5 * (v0 - d - 1) * sumLLT - 0.5 * sumVtr;
    // Lt9: Dirichlet entropies of eta and epsilon rows
    double es = 0.0, lge = 0.0, ept = 0.0;
    for (int s = 0; s < S; ++s) {
      const double e = post->eta[(size_t)k * S + s];
      es += e;
      lge += std::lgamma(e);
      ept += (e - 1) * logPi[(size_t)k * S + s];
    }
    Lt9 += std::lgamma(es) - lge + ept;
    for (int r = 0; r < S; ++r) {
      double ps = 0.0, lgp = 0.0, pt = 0.0;
      for (int s = 0; s < S; ++s) {
        const size_t x = ((size_t)k * S + r) * S + s;
        ps += post->epsilon[x];
        lgp += std::lgamma(post->epsilon[x]);
        pt += (post->epsilon[x] - 1) * logA[x];
      }
      Lt9 += std::lgamma(ps) - lgp + pt;
    }
    Lt10 += 0.5 * lt10a - 0.5 * d * S - H;
  }
  *L = st.Lt1 + Lt2 + Lt3 + Lt4 + Lt5 + Lt6 - st.Lt7 - Lt8 - Lt9 - Lt10;
  return VBHEM_OK;
}

int vbhem_em_mstep(const vbhem_em_opt_t *opt, const double *stats, vbhem_post_t *post) {
  if (!post_ok(post) || !opt_ok(opt, post->d) || !stats) return VBHEM_ERR_ARG;
  const int K = post->K, S = post->S, d = post->d;
  const bool full = post->covmode == VBHEM_COV_FULL;
  const size_t dd = full ? (size_t)d * d : (size_t)d;
  const Stats st(stats, K, S, d, post->covmode);
  const double l0 = opt->lambda0;
  std::vector<double> W0inv;
  w0_inv(opt, d, W0inv);
  std::vector<double> y(d), SC((size_t)d * d), Mt((size_t)d * d), tW((size_t)d * d);
  for (int k = 0; k < K; ++k) {
    post->alpha[k] = opt->alpha0 + (st.Nj[k] + 1e-50);
    for (int s = 0; s < S; ++s) {
      const size_t ks = (size_t)k * S + s;
      const double *u = st.U + ks * st.NU;
      // vbhem_compute_Statistics.m:57-82
      const double Nr = u[0] + 1e-50;
      for (int a = 0; a < d; ++a) y[a] = u[1 + a] / Nr;
      std::fill(SC.begin(), SC.end(), 0.0);
      if (full) {
        int e = 1 + d;
        for (int a = 0; a < d; ++a)
          for (int b = a; b < d; ++b, ++e) {
            SC[(size_t)a * d + b] = u[e] / Nr - y[a] * y[b];
            SC[(size_t)b * d + a] = u[e] / Nr - y[b] * y[a];
          }
      } else {
        for (int a = 0; a < d; ++a) SC[(size_t)a * d + a] = u[1 + d + a] / Nr - y[a] * y[a];
      }
      // vbhem_mstep_component.m:42-70
      const double lam = l0 + Nr, v = opt->v0 + Nr + 1.0, mult1 = l0 * Nr / (l0 + Nr);
      post->lam[ks] = lam;
      post->v[ks] = v;
      for (int a = 0; a < d; ++a)
        post->m[ks * d + a] = (l0 * opt->m0[a] + Nr * y[a]) / (l0 + Nr);
      for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b)
          Mt[(size_t)a * d + b] = W0inv[(size_t)a * d + b] + Nr * SC[(size_t)a * d + b] +
                                  mult1 * (y[a] - opt->m0[a]) * (y[b] - opt->m0[b]);
      inv_of(Mt.data(), d, tW.data());
      double *W = post->W + ks * dd;
      if (full) {
        for (int a = 0; a < d; ++a)
          for (int b = 0; b < d; ++b)
            W[(size_t)a * d + b] = (tW[(size_t)a * d + b] + tW[(size_t)b * d + a]) / 2;
      } else {
        for (int a = 0; a < d; ++a) W[a] = (tW[(size_t)a * d + a] + tW[(size_t)a * d + a]) / 2;
      }
      post->eta[ks] = opt->eta0 + st.N1[ks];
      for (int s2 = 0; s2 < S; ++s2)
        post->epsilon[ks * S + s2] = opt->epsilon0 + (S > 1 ? st.M[ks * S + s2] : 1e-12);
    }
  }
  return VBHEM_OK;
}

int vbhem_em_lower_bound_derivs(const vbhem_post_t *post, const vbhem_em_opt_t *opt,
                                const double *logLambdaTilde, const double *logA,
                                const double *logPi, const double *logOmega, double *dLL) {
  if (!post_ok(post) || !opt_ok(opt, post->d) || !logLambdaTilde || !logA || !logPi || !logOmega ||
      !dLL)
    return VBHEM_ERR_ARG;
  // vbhemh3m_lb.m:202-345 (the same arithmetic as vbhem_amd/host.py::lower_bound_derivs)
  const int K = post->K, S = post->S, d = post->d;
  const bool full = post->covmode == VBHEM_COV_FULL;
  const size_t dd = full ? (size_t)d * d : (size_t)d;
  const double a0 = opt->alpha0, e0 = opt->eta0, ep0 = opt->epsilon0, l0 = opt->lambda0,
               v0 = opt->v0;
  std::vector<double> W0inv;
  w0_inv(opt, d, W0inv);
  const bool iid = opt->W0_len == 1;
  double logdetW0inv = 0.0;
  if (iid) logdetW0inv = d * std::log(W0inv[0]);
  else for (int a = 0; a < d; ++a) logdetW0inv += std::log(W0inv[(size_t)a * d + a]);
  double sO = 0.0, sPi = 0.0, sA = 0.0, sL = 0.0;
  for (int k = 0; k < K; ++k) sO += logOmega[k];
  for (size_t x = 0; x < (size_t)K * S; ++x) { sPi += logPi[x]; sL += logLambdaTilde[x]; }
  for (size_t x = 0; x < (size_t)K * S * S; ++x) sA += logA[x];
  double *g = dLL;
  g[0] = K * psi(K * a0) - K * psi(a0) + sO;                              // alpha0
  g[1] = K * (S * psi(S * e0) - S * psi(e0)) + sPi;                       // eta0
  g[2] = (double)K * S * (S * psi(S * ep0) - S * psi(ep0)) + sA;          // epsilon0
  double sp = 0.0;
  for (int q = 1; q <= d; ++q) sp += psi(0.5 * (v0 + 1 - q));
  g[3] = (double)K * S * (0.5 * logdetW0inv - (d / 2.0) * std::log(2.0) - 0.5 * sp) + 0.5 * sL;  // v0
  const int nW = opt->W0_len;
  double *gW = g + 5, *gm = g + 5 + nW;
  double lam0 = 0.0;
  for (int x = 0; x < nW; ++x) gW[x] = 0.0;
  for (int a = 0; a < d; ++a) gm[a] = 0.0;
  std::vector<double> Wf((size_t)d * d), Wd((size_t)d);
  for (size_t ks = 0; ks < (size_t)K * S; ++ks) {
    const double *W = post->W + ks * dd, *mk = post->m + ks * d;
    const double v = post->v[ks], lam = post->lam[ks];
    if (full) {
      for (size_t x = 0; x < dd; ++x) Wf[x] = W[x];
    } else {
      std::fill(Wf.begin(), Wf.end(), 0.0);
      for (int a = 0; a < d; ++a) Wf[(size_t)a * d + a] = W[a];
    }
    double mWm = 0.0, trW = 0.0;
    for (int a = 0; a < d; ++a) {
      double wd = 0.0;  // (W (m - m0))[a]
      for (int b = 0; b < d; ++b) wd += Wf[(size_t)a * d + b] * (mk[b] - opt->m0[b]);
      mWm += (mk[a] - opt->m0[a]) * wd;
      trW += Wf[(size_t)a * d + a];
      gm[a] += l0 * v * wd;
    }
    lam0 += 0.5 * (d / l0 - d / lam - v * mWm);
    if (iid) {
      gW[0] += -0.5 * (-v * W0inv[0] * W0inv[0] * trW);
    } else {
      for (int a = 0; a < d; ++a) {
        const double wi = W0inv[(size_t)a * d + a];
        gW[a] += -0.5 * (-v * wi * wi * Wf[(size_t)a * d + a]);
      }
    }
  }
  g[4] = lam0;                                                            // lambda0
  if (iid) gW[0] += (double)K * S * (-0.5 * v0 * d * W0inv[0]);
  else for (int a = 0; a < d; ++a) gW[a] += (double)K * S * (-0.5 * v0 * W0inv[(size_t)a * d + a]);
  return VBHEM_OK;
}

int vbhem_em_host_iteration(const vbhem_em_opt_t *opt, const double *stats, vbhem_post_t *post,
                             double *logA, double *logPi, double *m, double *P, double *c,
                             double *logLambdaTilde, double *logOmega, double *L) {
  if (!L) return VBHEM_ERR_ARG;
  int rc = vbhem_em_lower_bound(post, opt, stats, logLambdaTilde, logA, logPi, logOmega, L);
  if (rc != VBHEM_OK) return rc;
  if (std::isnan(*L)) return VBHEM_OK;  // step_fc.m:338-374: no M-step for an unstable model
  rc = vbhem_em_mstep(opt, stats, post);
  if (rc != VBHEM_OK) return rc;
  return vbhem_em_prelude(post, logA, logPi, m, P, c, logLambdaTilde, logOmega);
}

size_t vbhem_em_workspace_bytes(const vbhem_base_t *base, int K, int S, int T) {
  if (!base || K < 1 || S < 1) return 0;
  const int d = base->d;
  const size_t dd = base->covmode == VBHEM_COV_FULL ? (size_t)d * d : (size_t)d;
  vbhem_cluster_t c = {K, S, nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t fused = vbhem_fused_workspace_bytes(base, &c, T);
  if (fused == 0) return 0;
  const size_t consts = (size_t)K * S * S + (size_t)K * S + (size_t)K * S * d + (size_t)K * S * dd +
                        (size_t)K * S + (size_t)K;
  // device-side host math (vbhem_em_dev.hip): three posteriors (the loop runs one
  // iteration ahead), logLambdaTilde, log det W, m0, W0^-1, the bound's partial sums,
  // its ticket, and a second hat_Z / L_elbo pair
  const size_t postn = (size_t)K + 3 * (size_t)K * S + (size_t)K * S * S + (size_t)K * S * d +
                       (size_t)K * S * dd;
  const size_t dev = 3 * postn + 2 * (size_t)K * S + (size_t)d + (size_t)d * d +
                     (size_t)K * S * 13 + 1 + 2 * (size_t)base->N * K;
  return (fused + 255) / 256 * 256 + (consts + dev) * sizeof(double) + 256;
}

namespace {

// the bound's hyperparameter constants (vbhemh3m_lb.m:74-86), as vbhem_em_lower_bound
void bound_constants(const vbhem_em_opt_t *opt, int K, int S, int d, const std::vector<double> &W0inv,
                     double &logCalpha0, double &logCeta0, double &logCepsilon0, double &logB0) {
  double logdetW0inv = 0.0;
  if (opt->W0_len == 1) logdetW0inv = d * std::log(W0inv[0]);
  else for (int a = 0; a < d; ++a) logdetW0inv += std::log(W0inv[(size_t)a * d + a]);
  const double a0 = opt->alpha0, e0 = opt->eta0, ep0 = opt->epsilon0, v0 = opt->v0;
  logCalpha0 = std::lgamma(K * a0) - K * std::lgamma(a0);
  logCeta0 = std::lgamma(S * e0) - S * std::lgamma(e0);
  logCepsilon0 = std::lgamma(S * ep0) - S * std::lgamma(ep0);
  logB0 = (v0 / 2) * logdetW0inv - (v0 * d / 2) * std::log(2.0) - (d * (d - 1) / 4.0) * std::log(kPi) -
          lgamma_sum_half(v0, d);
}

// spin on the sequence word the bound kernel writes to mapped host memory; the
// stream is queried now and then so a failed launch ends the wait with its error
hipError_t wait_flag(const int *flag, int seq, hipStream_t st) {
  for (long n = 0;; ++n) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
    if ((n & 1023) == 1023) {
      const hipError_t q = hipStreamQuery(st);
      if (q != hipSuccess && q != hipErrorNotReady) return q;
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? hipSuccess
                                                                                 : hipErrorUnknown;
    }
  }
}

struct PostDev {
  double *alpha, *eta, *eps, *lam, *v, *m, *W;
};

PostDev carve_post(double *&p, int K, int S, int d, size_t dd) {
  PostDev q;
  q.alpha = p; p += K;
  q.eta = p; p += (size_t)K * S;
  q.eps = p; p += (size_t)K * S * S;
  q.lam = p; p += (size_t)K * S;
  q.v = p; p += (size_t)K * S;
  q.m = p; p += (size_t)K * S * d;
  q.W = p; p += (size_t)K * S * dd;
  return q;
}

hipError_t copy_post(const vbhem_post_t *h, const PostDev &q, size_t dd, hipMemcpyKind kind,
                     hipStream_t st) {
  const int K = h->K, S = h->S, d = h->d;
  double *hp[7] = {h->alpha, h->eta, h->epsilon, h->lam, h->v, h->m, h->W};
  double *dp[7] = {q.alpha, q.eta, q.eps, q.lam, q.v, q.m, q.W};
  const size_t n[7] = {(size_t)K, (size_t)K * S, (size_t)K * S * S, (size_t)K * S, (size_t)K * S,
                       (size_t)K * S * d, (size_t)K * S * dd};
  for (int x = 0; x < 7; ++x) {
    hipError_t e = kind == hipMemcpyHostToDevice
                       ? hipMemcpyAsync(dp[x], hp[x], n[x] * sizeof(double), kind, st)
                       : hipMemcpyAsync(hp[x], dp[x], n[x] * sizeof(double), kind, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The loop's bound slots + sequence words live in pinned, mapped host memory.  One
// 64-byte block per concurrent run, taken from a per-device pool and given back at
// the end of the run: allocated once per process, not per run (hipHostMalloc /
// hipHostFree of mapped memory cost a kernel-driver round trip each).
struct Mapped {
  double *h = nullptr, *d = nullptr;
};
std::mutex g_mapped_mu;
std::map<int, std::vector<Mapped>> g_mapped_free;

hipError_t acquire_mapped(Mapped &m) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    std::lock_guard<std::mutex> g(g_mapped_mu);
    auto &v = g_mapped_free[dev];
    if (!v.empty()) {
      m = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  e = hipHostMalloc(reinterpret_cast<void **>(&m.h), 64, hipHostMallocMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&m.d), m.h, 0);
  return e;
}

void release_mapped(const Mapped &m) {
  if (!m.h) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;  // keep it (never reused) rather than free mid-run
  std::lock_guard<std::mutex> g(g_mapped_mu);
  g_mapped_free[dev].push_back(m);
}

// the statistics' one collective per E-step run: in-stream RCCL, or the caller's hook
int reduce_stats(const vbhem_em_ext_t *ext, vbhem_allreduce_fn allreduce, void *ctx,
                 double *stats_dev, size_t slen, hipStream_t st) {
  if (ext && ext->rccl_comm) return vbhem_rccl_allreduce_sum(ext->rccl_comm, stats_dev, slen, st);
  if (allreduce && allreduce(stats_dev, slen, st, ctx) != 0) return VBHEM_ERR_HIP;
  return VBHEM_OK;
}

// a host copy of a posterior (the one before the last M-step, for the derivatives)
struct HostPost {
  std::vector<double> a[7];
  vbhem_post_t t{};
  void size_like(const vbhem_post_t *p) {
    const int K = p->K, S = p->S, d = p->d;
    const size_t dd = p->covmode == VBHEM_COV_FULL ? (size_t)d * d : (size_t)d;
    const size_t n[7] = {(size_t)K, (size_t)K * S, (size_t)K * S * S, (size_t)K * S, (size_t)K * S,
                         (size_t)K * S * d, (size_t)K * S * dd};
    for (int x = 0; x < 7; ++x) a[x].resize(n[x]);
    t = {K, S, d, p->covmode, a[0].data(), a[1].data(), a[2].data(), a[3].data(), a[4].data(),
         a[5].data(), a[6].data()};
  }
  void copy_from(const vbhem_post_t *p) {
    size_like(p);
    const double *src[7] = {p->alpha, p->eta, p->epsilon, p->lam, p->v, p->m, p->W};
    for (int x = 0; x < 7; ++x) std::copy(src[x], src[x] + a[x].size(), a[x].begin());
  }
};

// vbhemh3m_lb.m:202-345 at a posterior: its prelude, then the raw derivatives
int derivs_at(const vbhem_post_t *p, const vbhem_em_opt_t *opt, double *dLL) {
  const int K = p->K, S = p->S, d = p->d;
  const size_t dd = p->covmode == VBHEM_COV_FULL ? (size_t)d * d : (size_t)d;
  std::vector<double> lA((size_t)K * S * S), lPi((size_t)K * S), m((size_t)K * S * d),
      P((size_t)K * S * dd), c((size_t)K * S), lLT((size_t)K * S), lO((size_t)K);
  int rc = vbhem_em_prelude(p, lA.data(), lPi.data(), m.data(), P.data(), c.data(), lLT.data(),
                            lO.data());
  if (rc != VBHEM_OK) return rc;
  return vbhem_em_lower_bound_derivs(p, opt, lLT.data(), lA.data(), lPi.data(), lO.data(), dLL);
}

void nan_derivs(const vbhem_em_opt_t *opt, int d, double *dLL) {
  for (int x = 0; x < VBHEM_DLL_LEN(d, opt->W0_len); ++x) dLL[x] = std::nan("");
}

// The EM loop with the per-iteration host math in C++ on the host (shapes outside
// the device kernels: d > 16 or S > 32).
int em_run_host(const vbhem_base_t *base, const double *tildeN_dev, int T, const vbhem_em_opt_t *opt,
                vbhem_post_t *post, double *LogLs, int *iters, double *L_final, int *stable,
                double *stats_dev, double *hatZ_dev, double *LL_dev, void *workspace_dev,
                hipStream_t st, vbhem_allreduce_fn allreduce, void *allreduce_ctx,
                const vbhem_em_ext_t *ext) {
  const int K = post->K, S = post->S, d = post->d;
  const size_t dd = post->covmode == VBHEM_COV_FULL ? (size_t)d * d : (size_t)d;
  vbhem_cluster_t c0 = {K, S, nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t fused = (vbhem_fused_workspace_bytes(base, &c0, T) + 255) / 256 * 256;
  // device constants: logA | logPi | m | P | c | logOmega (one upload per iteration)
  const size_t nA = (size_t)K * S * S, nPi = (size_t)K * S, nm = (size_t)K * S * d,
               nP = (size_t)K * S * dd, nc = (size_t)K * S, nO = (size_t)K;
  std::vector<double> h(nA + nPi + nm + nP + nc + nO), lLT(nc);
  double *dc = reinterpret_cast<double *>(static_cast<char *>(workspace_dev) + fused);
  vbhem_cluster_t cl = {K, S, dc, dc + nA, dc + nA + nPi, dc + nA + nPi + nm,
                        dc + nA + nPi + nm + nP};
  const double *dlogOmega = dc + nA + nPi + nm + nP + nc;
  const size_t slen = vbhem_stats_len(K, S, d, post->covmode);
  std::vector<double> stats(slen);
  const bool deriv = ext && ext->calc_deriv && ext->dLL;
  HostPost pre;
  double lastL = -DBL_MAX, L = -INFINITY;
  int it = 0;
  *stable = 1;
  double *hA = h.data(), *hPi = hA + nA, *hm = hPi + nPi, *hP = hm + nm, *hc = hP + nP,
         *hO = hc + nc;
  int rc = vbhem_em_prelude(post, hA, hPi, hm, hP, hc, lLT.data(), hO);
  if (rc != VBHEM_OK) return rc;
  while (true) {
    hipError_t e = hipMemcpyAsync(dc, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return VBHEM_ERR_HIP;
    rc = vbhem_estep_fused(base, &cl, T, tildeN_dev, dlogOmega, stats_dev, hatZ_dev, LL_dev,
                           workspace_dev, fused, st);
    if (rc != VBHEM_OK) return rc;
    rc = reduce_stats(ext, allreduce, allreduce_ctx, stats_dev, slen, st);
    if (rc != VBHEM_OK) return rc;
    e = hipMemcpyAsync(stats.data(), stats_dev, slen * sizeof(double), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return VBHEM_ERR_HIP;
    if (deriv) pre.copy_from(post);
    // the bound of this iteration's E-step, then (stable) the M-step and the next
    // iteration's prelude: the whole per-iteration host math, one call
    rc = vbhem_em_host_iteration(opt, stats.data(), post, hA, hPi, hm, hP, hc, lLT.data(), hO, &L);
    if (rc != VBHEM_OK) return rc;
    if (ext && ext->iter_seconds) ext->iter_seconds[it] = now_s();
    if (std::isnan(L)) {  // step_fc.m:338-374: unstable model, stop before the M-step
      L = -INFINITY;
      *stable = 0;
      break;
    }
    bool do_break = false;
    if (it > 1 && std::fabs((L - lastL) / lastL) <= opt->minDiff) do_break = true;
    if (it == opt->max_iter) do_break = true;
    LogLs[it] = L;
    ++it;
    lastL = L;
    if (do_break) break;
  }
  *iters = it;
  *L_final = L;
  if (deriv) {
    if (*stable) return derivs_at(&pre.t, opt, ext->dLL);  // step_fc.m:356-360
    nan_derivs(opt, d, ext->dLL);                           // :362-368
  }
  return VBHEM_OK;
}

}  // namespace

int vbhem_em_run_ext(const vbhem_base_t *base, const double *tildeN_dev, int T,
                     const vbhem_em_opt_t *opt, vbhem_post_t *post, double *LogLs, int *iters,
                     double *L_final, int *stable, double *stats_dev, double *hatZ_dev,
                     double *LL_dev, void *workspace_dev, size_t workspace_bytes, void *stream,
                     vbhem_allreduce_fn allreduce, void *allreduce_ctx, const vbhem_em_ext_t *ext) {
  if (!base || !post_ok(post) || !opt_ok(opt, post->d) || !LogLs || !iters || !L_final ||
      !stable || !stats_dev || post->d != base->d || post->covmode != base->covmode)
    return VBHEM_ERR_ARG;
  if (ext && ext->rccl_comm && allreduce)
    return vbhem::set_error(VBHEM_ERR_ARG, "vbhem_em_run_ext: an RCCL communicator and an all-reduce callback");
  const int K = post->K, S = post->S, d = post->d;
  const size_t dd = post->covmode == VBHEM_COV_FULL ? (size_t)d * d : (size_t)d;
  const size_t need = vbhem_em_workspace_bytes(base, K, S, T);
  if (need == 0 || !workspace_dev || workspace_bytes < need) return VBHEM_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!vbhem::em_dev_supported(d, S) || std::getenv("VBHEM_EM_HOST_MATH"))
    return em_run_host(base, tildeN_dev, T, opt, post, LogLs, iters, L_final, stable, stats_dev,
                       hatZ_dev, LL_dev, workspace_dev, st, allreduce, allreduce_ctx, ext);
  vbhem_cluster_t c0 = {K, S, nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t fused = (vbhem_fused_workspace_bytes(base, &c0, T) + 255) / 256 * 256;
  const size_t nA = (size_t)K * S * S, nPi = (size_t)K * S, nm = (size_t)K * S * d,
               nP = (size_t)K * S * dd, nc = (size_t)K * S;
  double *dc = reinterpret_cast<double *>(static_cast<char *>(workspace_dev) + fused);
  vbhem_cluster_t cl = {K, S, dc, dc + nA, dc + nA + nPi, dc + nA + nPi + nm,
                        dc + nA + nPi + nm + nP};
  double *dlogOmega = dc + nA + nPi + nm + nP + nc;
  double *p = dlogOmega + K;
  PostDev pd[3];
  for (int x = 0; x < 3; ++x) pd[x] = carve_post(p, K, S, d, dd);
  double *dlLT = p; p += nc;
  double *dlogdetW = p; p += nc;
  double *dm0 = p; p += d;
  double *dW0inv = p; p += (size_t)d * d;
  double *dpart = p; p += (size_t)K * S * 13;
  int *dticket = reinterpret_cast<int *>(p); p += 1;
  // E-step j writes hat_Z / L_elbo into pair j % 2 (the caller's arrays are pair 0):
  // the speculative E-step of the next iteration keeps this one's
  double *hz[2] = {hatZ_dev, p}, *ll[2] = {LL_dev, p + (size_t)base->N * K};
  // hyperparameters: W0^-1 and the bound's constants once per run
  std::vector<double> W0inv;
  w0_inv(opt, d, W0inv);
  vbhem::EmDevArgs a{};
  a.K = K; a.S = S; a.d = d; a.covmode = post->covmode; a.NU = (int)vbhem_stats_nu(d, post->covmode);
  a.stats = stats_dev;
  a.alpha0 = opt->alpha0; a.eta0 = opt->eta0; a.epsilon0 = opt->epsilon0; a.lambda0 = opt->lambda0;
  a.v0 = opt->v0;
  bound_constants(opt, K, S, d, W0inv, a.logCalpha0, a.logCeta0, a.logCepsilon0, a.logB0);
  a.m0 = dm0; a.W0inv = dW0inv;
  a.logA = dc; a.logPi = dc + nA; a.cm = dc + nA + nPi; a.P = dc + nA + nPi + nm;
  a.c = dc + nA + nPi + nm + nP; a.lLT = dlLT; a.logOmega = dlogOmega; a.logdetW = dlogdetW;
  a.part = dpart; a.ticket = dticket;
  hipError_t e = hipMemcpyAsync(dm0, opt->m0, d * sizeof(double), hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(dW0inv, W0inv.data(), W0inv.size() * sizeof(double), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = copy_post(post, pd[0], dd, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(dticket, 0, sizeof(int), st);
  // the bound of iteration j goes straight to pinned, mapped host memory (slot j % 2),
  // followed by a sequence word the host polls: no stream synchronisation per
  // iteration, and the next E-step is already queued behind the bound
  Mapped mb;
  if (e == hipSuccess) e = acquire_mapped(mb);
  double *Lh = mb.h, *Ld = mb.d;
  int *flag_h = Lh ? reinterpret_cast<int *>(Lh + 2) : nullptr;  // two ints after L[2]
  if (flag_h) flag_h[0] = flag_h[1] = 0;
  auto set_post = [&a](const PostDev &in, const PostDev &out) {
    a.alpha = in.alpha; a.eta = in.eta; a.eps = in.eps; a.lam = in.lam; a.v = in.v; a.m = in.m;
    a.W = in.W;
    a.alpha_o = out.alpha; a.eta_o = out.eta; a.eps_o = out.eps; a.lam_o = out.lam; a.v_o = out.v;
    a.m_o = out.m; a.W_o = out.W;
  };
  set_post(pd[0], pd[1]);
  if (e == hipSuccess) e = vbhem::launch_em_dev(a, vbhem::kEmPrelude, nullptr, st);
  const size_t slen = vbhem_stats_len(K, S, d, post->covmode);
  int rc = VBHEM_OK;
  // iteration j: E-step (constants of posterior j % 3) -> all-reduce -> bound of
  // posterior j % 3 + M-step into (j + 1) % 3 + prelude (the constants of E-step j + 1)
  auto enqueue = [&](int j) -> bool {
    rc = vbhem_estep_fused(base, &cl, T, tildeN_dev, dlogOmega, stats_dev, hz[j % 2], ll[j % 2],
                           workspace_dev, fused, st);
    if (rc != VBHEM_OK) return false;
    rc = reduce_stats(ext, allreduce, allreduce_ctx, stats_dev, slen, st);
    if (rc != VBHEM_OK) return false;
    set_post(pd[j % 3], pd[(j + 1) % 3]);
    a.seq = j + 1;
    a.flag = reinterpret_cast<int *>(Ld + 2) + (j % 2);
    void *t0 = vbhem::timing_begin(st);
    e = vbhem::launch_em_dev(a, vbhem::kEmIterate, Ld + (j % 2), st);
    vbhem::timing_end_em_math(t0, st);
    return e == hipSuccess;
  };
  double lastL = -DBL_MAX, L = -INFINITY;
  int it = 0, fin_post = 0, fin_e = 0;
  *stable = 1;
  bool ok = e == hipSuccess && enqueue(0);
  while (ok) {
    // the next iteration is queued before this one's bound is read (it is discarded
    // when this one ends the loop; never past max_iter)
    if (it + 1 <= opt->max_iter && !enqueue(it + 1)) break;
    e = wait_flag(flag_h + (it % 2), it + 1, st);
    if (e != hipSuccess) break;
    if (ext && ext->iter_seconds) ext->iter_seconds[it] = now_s();
    L = Lh[it % 2];
    fin_e = it % 2;
    if (std::isnan(L)) {  // step_fc.m:338-374: unstable model, the posterior before the M-step
      L = -INFINITY;
      *stable = 0;
      fin_post = it % 3;
      break;
    }
    bool do_break = false;
    if (it > 1 && std::fabs((L - lastL) / lastL) <= opt->minDiff) do_break = true;
    if (it == opt->max_iter) do_break = true;
    LogLs[it] = L;
    ++it;
    lastL = L;
    fin_post = it % 3;  // the M-step's posterior
    if (do_break) break;
  }
  hipError_t e2 = hipStreamSynchronize(st);  // the discarded speculative iteration drains
  if (e == hipSuccess) e = e2;
  if (e == hipSuccess && rc == VBHEM_OK && fin_e == 1 && base->N > 0) {
    e = hipMemcpyAsync(hatZ_dev, hz[1], (size_t)base->N * K * sizeof(double),
                       hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(LL_dev, ll[1], (size_t)base->N * K * sizeof(double),
                         hipMemcpyDeviceToDevice, st);
  }
  // the derivatives (step_fc.m:356-368) are taken at the posterior before the last
  // M-step: pd[(it - 1) % 3], which neither the last M-step nor the discarded
  // speculative one ((it + 1) % 3) wrote
  const bool deriv = ext && ext->calc_deriv && ext->dLL;
  HostPost pre;
  if (deriv && *stable && it >= 1) pre.size_like(post);
  if (e == hipSuccess && rc == VBHEM_OK) e = copy_post(post, pd[fin_post], dd, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && rc == VBHEM_OK && deriv && *stable && it >= 1)
    e = copy_post(&pre.t, pd[(it - 1) % 3], dd, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && rc == VBHEM_OK) e = hipStreamSynchronize(st);
  if (e == hipSuccess) release_mapped(mb);  // a failed stream may still write it: not reused
  if (rc != VBHEM_OK) return rc;
  if (e != hipSuccess) return VBHEM_ERR_HIP;
  *iters = it;
  *L_final = L;
  if (deriv) {
    if (*stable && it >= 1) return derivs_at(&pre.t, opt, ext->dLL);
    nan_derivs(opt, d, ext->dLL);
  }
  return VBHEM_OK;
}

int vbhem_em_run(const vbhem_base_t *base, const double *tildeN_dev, int T,
                 const vbhem_em_opt_t *opt, vbhem_post_t *post, double *LogLs, int *iters,
                 double *L_final, int *stable, double *stats_dev, double *hatZ_dev,
                 double *LL_dev, void *workspace_dev, size_t workspace_bytes, void *stream,
                 vbhem_allreduce_fn allreduce, void *allreduce_ctx) {
  return vbhem_em_run_ext(base, tildeN_dev, T, opt, post, LogLs, iters, L_final, stable, stats_dev,
                          hatZ_dev, LL_dev, workspace_dev, workspace_bytes, stream, allreduce,
                          allreduce_ctx, nullptr);
}

}  // extern "C"

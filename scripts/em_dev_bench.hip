// scripts/em_dev_bench.hip -- time em_iter_kernel alone (C4 shape: K = 16, S = 8,
// d = 8 full) on synthetic statistics, with per-phase s_memrealtime marks.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -DEMDEV_TIMING -I<pkg>/csrc -o scripts/em_dev_bench.bin scripts/em_dev_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "vbhem_em_dev.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 16, S = argc > 2 ? atoi(argv[2]) : 8, d = argc > 3 ? atoi(argv[3]) : 8;
  const int KS = K * S, dd = d * d, NU = 1 + d + d * (d + 1) / 2;
  std::vector<double> h;
  auto put = [&](size_t n, double v) { size_t o = h.size(); h.resize(o + n, v); return o; };
  // posterior
  size_t o_alpha = put(K, 3.0), o_eta = put(KS, 2.0), o_eps = put((size_t)KS * S, 1.5), o_lam = put(KS, 5.0),
         o_v = put(KS, 20.0), o_m = put((size_t)KS * d, 0.1), o_W = put((size_t)KS * dd, 0.0);
  for (int x = 0; x < KS; ++x) for (int r = 0; r < d; ++r) h[o_W + (size_t)x * dd + r * d + r] = 0.05 + 0.001 * r;
  size_t o_out = put(K + 3 * (size_t)KS + (size_t)KS * S + (size_t)KS * d + (size_t)KS * dd, 0.0);
  // stats: Nj | N1 | M | Lt1 Lt7 | U
  size_t o_st = put(K, 100.0); put(KS, 12.0); put((size_t)KS * S, 1.3); put(2, -5.0);
  size_t o_U = put((size_t)KS * NU, 0.0);
  for (int x = 0; x < KS; ++x) {
    double *u = &h[o_U + (size_t)x * NU];
    const double Nr = 10.0 + x % 7;
    u[0] = Nr;
    for (int a = 0; a < d; ++a) u[1 + a] = Nr * 0.2 * (a - 3);
    int q = 1 + d;
    for (int a = 0; a < d; ++a) for (int b = a; b < d; ++b) u[q++] = Nr * ((a == b ? 1.0 : 0.1) + 0.04 * (a - 3) * (b - 3));
  }
  size_t o_m0 = put(d, 0.0), o_W0 = put(dd, 0.0);
  for (int r = 0; r < d; ++r) h[o_W0 + r * d + r] = 1.0;
  size_t o_c = put((size_t)KS * S + KS + (size_t)KS * d + (size_t)KS * dd + KS + KS + K + KS, 0.0);
  for (int x = 0; x < KS; ++x) h[o_c + (size_t)KS * S + KS + (size_t)KS * d + (size_t)KS * dd + KS + x] = -10.0;  // lLT
  size_t o_part = put((size_t)KS * 13, 0.0), o_tick = put(1, 0.0), o_L = put(1, 0.0);
  double *D;
  CK(hipMalloc(&D, h.size() * sizeof(double)));
  CK(hipMemcpy(D, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  vbhem::EmDevArgs a{};
  a.K = K; a.S = S; a.d = d; a.covmode = 1; a.NU = NU;
  a.alpha = D + o_alpha; a.eta = D + o_eta; a.eps = D + o_eps; a.lam = D + o_lam; a.v = D + o_v; a.m = D + o_m; a.W = D + o_W;
  double *q = D + o_out;
  a.alpha_o = q; q += K; a.eta_o = q; q += KS; a.eps_o = q; q += (size_t)KS * S; a.lam_o = q; q += KS;
  a.v_o = q; q += KS; a.m_o = q; q += (size_t)KS * d; a.W_o = q;
  a.stats = D + o_st;
  a.alpha0 = 1; a.eta0 = 1; a.epsilon0 = 1; a.lambda0 = 1; a.v0 = 10;
  a.m0 = D + o_m0; a.W0inv = D + o_W0;
  double *c = D + o_c;
  a.logA = c; c += (size_t)KS * S; a.logPi = c; c += KS; a.cm = c; c += (size_t)KS * d; a.P = c; c += (size_t)KS * dd;
  a.c = c; c += KS; a.logdetW = c; c += KS; a.logOmega = c; c += K; a.lLT = c;
  a.part = D + o_part; a.ticket = reinterpret_cast<int *>(D + o_tick); a.flag = nullptr;
  double *L = D + o_L;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int mode = 0; mode < 2; ++mode) {
    for (int w = 0; w < 5; ++w) CK(vbhem::launch_em_dev(a, mode, L, 0));
    CK(hipDeviceSynchronize());
    const int n = 200;
    CK(hipEventRecord(e0, 0));
    for (int w = 0; w < n; ++w) CK(vbhem::launch_em_dev(a, mode, L, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // one more, then the phase marks of that launch
    CK(vbhem::launch_em_dev(a, mode, L, 0));
    CK(hipDeviceSynchronize());
    static long long t[8][1024];
    CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(vbhem::emdev_t), sizeof(t)));
    long long t0 = t[0][0];
    for (int x = 0; x < KS && x < 1024; ++x) if (t[0][x] < t0) t0 = t[0][x];
    printf("mode %d: %.2f us per launch (%d back to back); phase marks (us after the first wave's start), waves 0, KS/2, KS-1:\n",
           mode, 1e3 * ms / n, n);
    for (int ph = 0; ph < 8; ++ph) {
      printf("  mark %d:", ph);
      for (int x : {0, KS / 2, KS - 1}) printf(" %8.2f", (t[ph][x] - t0) / 100.0);
      long long mx = 0;
      for (int x = 0; x < KS && x < 1024; ++x) if (t[ph][x] - t0 > mx) mx = t[ph][x] - t0;
      printf("   max %8.2f\n", mx / 100.0);
    }
  }
  double Lh;
  CK(hipMemcpy(&Lh, L, sizeof(double), hipMemcpyDeviceToHost));
  printf("L = %.6f\n", Lh);
  return 0;
}

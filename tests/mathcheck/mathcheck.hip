// tests/mathcheck/mathcheck.hip -- TEST-ONLY exports of the restricted-domain
// fp64 exp/log/reciprocal in csrc/vbhem_math.h, evaluated on the host (the
// same source compiled for the CPU; rcp seed = 1/b) and on the device (the
// gfx950 code path: v_rcp_f64 seed), so tests can measure their ulp error
// against libm.
#include <hip/hip_runtime.h>

#include "vbhem_log_table.h"
#include "vbhem_math.h"
#include "vbhem_mfma4.h"

static const double kLogTabHost[vbhem::kLogTabDoubles] = VBHEM_LOG_TABLE_INIT;
__device__ const double kLogTabDev[vbhem::kLogTabDoubles] = VBHEM_LOG_TABLE_INIT;
static const double kExpTabHost[vbhem::kExpTabDoubles] = VBHEM_EXP_TABLE_INIT;
__device__ const double kExpTabDev[vbhem::kExpTabDoubles] = VBHEM_EXP_TABLE_INIT;

// compact tables of exp_tabc_n / log_tabc_n (as fb_bwd2_kernel stages them)
struct CompactTabs {
  double e[vbhem::kExpTabEntries];
  double l[2 * vbhem::kLogTabEntries];
};
static const double kLogEHost[2 * vbhem::kLogTabEEntries] = VBHEM_LOG1024_TABLE_INIT;
__device__ const double kLogEDev[2 * vbhem::kLogTabEEntries] = VBHEM_LOG1024_TABLE_INIT;
static const double kExpEHost[vbhem::kExpTabEEntries] = VBHEM_EXP2048_TABLE_INIT;
__device__ const double kExpEDev[vbhem::kExpTabEEntries] = VBHEM_EXP2048_TABLE_INIT;
static CompactTabs compact_host() {
  CompactTabs c;
  for (int j = 0; j < vbhem::kExpTabEntries; ++j) c.e[j] = kExpTabHost[2 * j];
  for (int j = 0; j < vbhem::kLogTabEntries; ++j) {
    c.l[2 * j] = kLogTabHost[4 * j];
    c.l[2 * j + 1] = kLogTabHost[4 * j + 1];
  }
  return c;
}

namespace {

__global__ void logtabc_kernel(int n, const double* __restrict__ x, double* __restrict__ l,
                               double* __restrict__ e) {
  __shared__ __attribute__((aligned(16))) double lt[2 * vbhem::kLogTabEntries];
  __shared__ __attribute__((aligned(16))) double et[vbhem::kExpTabEntries];
  for (int k = threadIdx.x; k < vbhem::kExpTabEntries; k += blockDim.x) et[k] = kExpTabDev[2 * k];
  for (int k = threadIdx.x; k < vbhem::kLogTabEntries; k += blockDim.x) {
    lt[2 * k] = kLogTabDev[4 * k];
    lt[2 * k + 1] = kLogTabDev[4 * k + 1];
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    double y[1], z[1] = {x[i]}, m[1] = {-x[i]};
    vbhem::log_tabc_n<1>(y, z, lt);
    l[i] = y[0];
    vbhem::exp_tabc_n<1>(y, m, et);
    e[i] = y[0];
  }
}

__global__ void logtabe_kernel(int n, const double* __restrict__ x, double* __restrict__ l,
                               double* __restrict__ e) {
  __shared__ __attribute__((aligned(16))) double lt[2 * vbhem::kLogTabEEntries];
  __shared__ __attribute__((aligned(16))) double et[vbhem::kExpTabEEntries];
  for (int k = threadIdx.x; k < vbhem::kExpTabEEntries; k += blockDim.x) et[k] = kExpEDev[k];
  for (int k = threadIdx.x; k < 2 * vbhem::kLogTabEEntries; k += blockDim.x) lt[k] = kLogEDev[k];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    double y[1], z[1] = {x[i]}, m[1] = {-x[i]};
    vbhem::log_tabe_n<1>(y, z, lt);
    l[i] = y[0];
    vbhem::exp_tabe_n<1>(y, m, et);
    e[i] = y[0];
  }
}

// exp_m_n / log_m_n of the MFMA kernels (vbhem_mfma4.h) with the column maximum m = 0:
// log at x, exp at -x (device only: integer builtins of gfx950)
__global__ void logtabm_kernel(int n, const double* __restrict__ x, double* __restrict__ l,
                               double* __restrict__ e) {
  __shared__ __attribute__((aligned(16))) double et[2048];
  __shared__ __attribute__((aligned(16))) double lt[2 * 1024];
  vbhem::m4::stage_tables(et, lt, threadIdx.x, blockDim.x);
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    double y[1];
    const double z[1] = {x[i]}, v[1] = {-x[i]}, s[1] = {vbhem::m4::red_s(-x[i])};
    const int wq[1] = {(int)(2147483648u + vbhem::m4::kWq0)};
    const unsigned wp[1] = {2147483648u - vbhem::m4::kBias};
    vbhem::m4::log_m_n<1>(y, z, wq, lt);
    l[i] = y[0];
    vbhem::m4::exp_m_n<1>(y, v, s, wp, et);
    e[i] = y[0];
  }
}

// round 6: the log on the 2^1023-scaled 1/c table (log_x_n, fb_bwd4_kernel /
// fb_bwd12_kernel) beside the form it replaces (log_q_n on the plain table), column
// maximum 0: log at x (both the decoupled and the 2048-unit maxima), exp at -x.  Tables in global memory
// (the helpers take any pointer)
__global__ void stagex_kernel(double* et, double* lx, double* lq) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
  for (int k = tid; k < 2048; k += nt) et[k] = vbhem::m4::kExpTab4[k] * 0x1p-1010;
  vbhem::m4::stage_log8k_x(lx, tid, nt);
  vbhem::m4::stage_log8k(lq, tid, nt);
}
__global__ void logtabx_kernel(int n, const double* __restrict__ x, double* __restrict__ out,
                               const double* et, const double* lx, const double* lq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using namespace vbhem::m4;
  double y[1];
  const double z[1] = {x[i]};
  const int wq[1] = {-1023}, wq0[1] = {-1023 * 2048};
  log_x_n<1, true>(y, z, wq, lx);
  out[6 * i + 0] = y[0];
  log_q_n<1, true>(y, z, wq, lq);
  out[6 * i + 1] = y[0];
  log_x_n<1, false>(y, z, wq0, lx);
  out[6 * i + 2] = y[0];
  log_q_n<1, false>(y, z, wq0, lq);
  out[6 * i + 3] = y[0];
  const double v[1] = {-x[i]}, s[1] = {red_s(-x[i])};
  const double t[1] = {etab_at(et, s[0])};
  const unsigned wph[1] = {(1u << 20) - 1010u};
  exp_d_n<1>(y, v, s, t, wph);
  out[6 * i + 4] = y[0];
  exp_d_n<1>(y, v, s, t, wph);
  out[6 * i + 5] = y[0];
}

__global__ void math_kernel(int n, const double* __restrict__ x, double* __restrict__ e,
                            double* __restrict__ l, double* __restrict__ r) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  e[i] = vbhem::exp_nonpos(-v);
  l[i] = vbhem::log_pos(v);
  r[i] = vbhem::rcp_pos(v);
}

__global__ void logtab_kernel(int n, const double* __restrict__ x, double* __restrict__ l,
                              double* __restrict__ e, int fast) {
  __shared__ __attribute__((aligned(16))) double tab[vbhem::kLogTabDoubles];
  __shared__ __attribute__((aligned(16))) double etab[vbhem::kExpTabDoubles];
  for (int k = threadIdx.x; k < vbhem::kLogTabDoubles; k += blockDim.x) tab[k] = kLogTabDev[k];
  for (int k = threadIdx.x; k < vbhem::kExpTabDoubles; k += blockDim.x) etab[k] = kExpTabDev[k];
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    if (fast) {
      l[i] = vbhem::log_tabf(x[i], tab);
      e[i] = vbhem::exp_tabf(-x[i], etab);
    } else {
      l[i] = vbhem::log_tab(x[i], tab);
      e[i] = vbhem::exp_tab(-x[i], etab);
    }
  }
}

}  // namespace

extern "C" {

// x > 0 for every element: exp is evaluated at -x, log and rcp at x.
void mathcheck_host(int n, const double* x, double* e, double* l, double* r) {
  for (int i = 0; i < n; i++) {
    e[i] = vbhem::exp_nonpos(-x[i]);
    l[i] = vbhem::log_pos(x[i]);
    r[i] = vbhem::rcp_pos(x[i]);
  }
}

// table-driven log / exp: log at x, exp at -x; host / device; the *f variants are
// the reduced-operation pair of the backward-only pass
void logtab_host(int n, const double* x, double* l, double* e) {
  for (int i = 0; i < n; i++) {
    l[i] = vbhem::log_tab(x[i], kLogTabHost);
    e[i] = vbhem::exp_tab(-x[i], kExpTabHost);
  }
}

void logtabf_host(int n, const double* x, double* l, double* e) {
  for (int i = 0; i < n; i++) {
    l[i] = vbhem::log_tabf(x[i], kLogTabHost);
    e[i] = vbhem::exp_tabf(-x[i], kExpTabHost);
  }
}

// compact-table pair of fb_bwd2_kernel: log at x, exp at -x
void logtabc_host(int n, const double* x, double* l, double* e) {
  static const CompactTabs c = compact_host();
  for (int i = 0; i < n; i++) {
    double y[1], z[1] = {x[i]}, m[1] = {-x[i]};
    vbhem::log_tabc_n<1>(y, z, c.l);
    l[i] = y[0];
    vbhem::exp_tabc_n<1>(y, m, c.e);
    e[i] = y[0];
  }
}

// short-series pair of fb_bwd2_kernel: log at x, exp at -x
void logtabe_host(int n, const double* x, double* l, double* e) {
  for (int i = 0; i < n; i++) {
    double y[1], z[1] = {x[i]}, m[1] = {-x[i]};
    vbhem::log_tabe_n<1>(y, z, kLogEHost);
    l[i] = y[0];
    vbhem::exp_tabe_n<1>(y, m, kExpEHost);
    e[i] = y[0];
  }
}

static int logtab_device_impl(int n, const double* x, double* l, double* e, int fast) {
  double *dx = nullptr, *dl = nullptr, *de = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(n > 0 ? n : 1);
  hipError_t st = hipMalloc(&dx, bytes);
  if (st == hipSuccess) st = hipMalloc(&dl, bytes);
  if (st == hipSuccess) st = hipMalloc(&de, bytes);
  if (st == hipSuccess) st = hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  if (st == hipSuccess && n > 0) {
    if (fast == 2) logtabc_kernel<<<(n + 255) / 256, 256>>>(n, dx, dl, de);
    else if (fast == 3) logtabe_kernel<<<(n + 255) / 256, 256>>>(n, dx, dl, de);
    else if (fast == 4) logtabm_kernel<<<(n + 255) / 256, 256>>>(n, dx, dl, de);
    else logtab_kernel<<<(n + 255) / 256, 256>>>(n, dx, dl, de, fast);
    st = hipGetLastError();
  }
  if (st == hipSuccess) st = hipMemcpy(l, dl, sizeof(double) * n, hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemcpy(e, de, sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dl);
  (void)hipFree(de);
  return (int)st;
}

int logtab_device(int n, const double* x, double* l, double* e) {
  return logtab_device_impl(n, x, l, e, 0);
}

int logtabf_device(int n, const double* x, double* l, double* e) {
  return logtab_device_impl(n, x, l, e, 1);
}

int logtabc_device(int n, const double* x, double* l, double* e) {
  return logtab_device_impl(n, x, l, e, 2);
}

int logtabe_device(int n, const double* x, double* l, double* e) {
  return logtab_device_impl(n, x, l, e, 3);
}

int logtabm_device(int n, const double* x, double* l, double* e) {
  return logtab_device_impl(n, x, l, e, 4);
}

// logtabx_kernel on device 0: out[6 i + (log new, log old, log2048 new, log2048 old,
// exp new, exp old)]
int logtabx_device(int n, const double* x, double* out) {
  double *dx = nullptr, *dout = nullptr, *tabs = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(n > 0 ? n : 1);
  hipError_t st = hipMalloc(&dx, bytes);
  if (st == hipSuccess) st = hipMalloc(&dout, 6 * bytes);
  if (st == hipSuccess) st = hipMalloc(&tabs, sizeof(double) * (2048 + 4 * 8192));
  if (st == hipSuccess) st = hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  if (st == hipSuccess && n > 0) {
    stagex_kernel<<<64, 256>>>(tabs, tabs + 2048, tabs + 2048 + 2 * 8192);
    logtabx_kernel<<<(n + 255) / 256, 256>>>(n, dx, dout, tabs, tabs + 2048, tabs + 2048 + 2 * 8192);
    st = hipGetLastError();
  }
  if (st == hipSuccess) st = hipMemcpy(out, dout, 6 * sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dout);
  (void)hipFree(tabs);
  return (int)st;
}

// Same on device 0 (host arrays in/out).  Returns 0 or a hipError_t.
int mathcheck_device(int n, const double* x, double* e, double* l, double* r) {
  double *dx = nullptr, *de = nullptr, *dl = nullptr, *dr = nullptr;
  const size_t bytes = sizeof(double) * (size_t)(n > 0 ? n : 1);
  hipError_t st = hipMalloc(&dx, bytes);
  if (st == hipSuccess) st = hipMalloc(&de, bytes);
  if (st == hipSuccess) st = hipMalloc(&dl, bytes);
  if (st == hipSuccess) st = hipMalloc(&dr, bytes);
  if (st == hipSuccess) st = hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
  if (st == hipSuccess && n > 0) {
    math_kernel<<<(n + 255) / 256, 256>>>(n, dx, de, dl, dr);
    st = hipGetLastError();
  }
  if (st == hipSuccess) st = hipMemcpy(e, de, sizeof(double) * n, hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemcpy(l, dl, sizeof(double) * n, hipMemcpyDeviceToHost);
  if (st == hipSuccess) st = hipMemcpy(r, dr, sizeof(double) * n, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(de);
  (void)hipFree(dl);
  (void)hipFree(dr);
  return (int)st;
}

}  // extern "C"

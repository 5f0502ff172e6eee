// tests/mathcheck/mathcheck.hip -- TEST-ONLY exports of the restricted-domain
// fp64 exp/log/reciprocal in csrc/vbhem_math.h, evaluated on the host (the
// same source compiled for the CPU; rcp seed = 1/b) and on the device (the
// gfx950 code path: v_rcp_f64 seed), so tests can measure their ulp error
// against libm.
#include <hip/hip_runtime.h>

#include "vbhem_math.h"

namespace {

__global__ void math_kernel(int n, const double* __restrict__ x, double* __restrict__ e,
                            double* __restrict__ l, double* __restrict__ r) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  e[i] = vbhem::exp_nonpos(-v);
  l[i] = vbhem::log_pos(v);
  r[i] = vbhem::rcp_pos(v);
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

// ubench_coexec.hip -- does the fp64 matrix pipe run beside fp64 (or int32) VALU work
// issued by OTHER waves of the same SIMD on gfx950?  (VERDICT r05 "next" item 3: the
// answer decides whether the emission GEMM -- MFMA-bound at C5 -- could hide under the
// VALU-bound backward pass by co-residence.)  Development tool, not part of the library.
//
// One 16-wave block per CU (a 96 KB dynamic LDS request keeps it alone there); waves are
// dealt to the CU's 4 SIMDs round-robin, so waves 0-7 put two on every SIMD and waves
// 8-15 two more.  Per mode:
//   mfma      waves 0-7 run independent v_mfma_f64_4x4x4 chains, waves 8-15 exit
//   mfma16    the same with v_mfma_f64_16x16x4
//   valu      waves 8-15 run independent v_fma_f64 chains, waves 0-7 exit
//   ivalu     waves 8-15 run independent v_add_u32 / v_xor_b32 chains (int32 VALU)
//   mfma+valu, mfma16+valu, mfma+ivalu   both halves at once
// If the matrix pipe co-executes with the other waves' VALU work, a "both" run takes
// ~max of its two halves; if the two share issue or a datapath, ~their sum.  Each mode is
// its own template instance, so a rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES,
// SQ_VALU_MFMA_COEXEC_CYCLES) reports it per kernel (scripts/ubench_coexec.sh).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_coexec scripts/ubench_coexec.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef double double4_t __attribute__((ext_vector_type(4)));

enum Half { NONE = 0, MFMA4 = 1, MFMA16 = 2, VALU64 = 3, VALU32 = 4 };

// ITM / ITV: loop trips of the matrix and VALU halves (set so each takes ~1 ms alone)
template <int LO, int HI>
__global__ __launch_bounds__(1024) void coexec_kernel(double *out, long long *cyc, int itm, int itv) {
  const int wave = threadIdx.x >> 6;
  const int what = wave < 8 ? LO : HI;
  double s = 0.0;
  const long long t0 = clock64();
  if (what == MFMA4) {
    double acc[8];
    for (int q = 0; q < 8; ++q) acc[q] = 1.0 + q * 1e-3 + threadIdx.x * 1e-6;
    const double a = 1.0000001, b = 0.9999999;
    for (int it = 0; it < itm; ++it) {
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[q], 0, 0, 0);
    }
    for (int q = 0; q < 8; ++q) s += acc[q];
  } else if (what == MFMA16) {
    double4_t acc[4];
    for (int q = 0; q < 4; ++q) acc[q] = double4_t{1.0 + q, 1.0, 1.0, 1.0};
    const double a = 1.0000001, b = 0.9999999;
    for (int it = 0; it < itm; ++it) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    }
    for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][3];
  } else if (what == VALU64) {
    double x[8];
    for (int q = 0; q < 8; ++q) x[q] = 1.0 + q * 1e-3 + threadIdx.x * 1e-6;
    const double b = 1.0000001, c = 1e-9;
    for (int it = 0; it < itv; ++it) {
#pragma unroll
      for (int q = 0; q < 8; ++q) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[q]) : "v"(b), "v"(c));
    }
    for (int q = 0; q < 8; ++q) s += x[q];
  } else if (what == VALU32) {
    unsigned x[8];
    for (int q = 0; q < 8; ++q) x[q] = threadIdx.x + q;
    for (int it = 0; it < itv; ++it) {
#pragma unroll
      for (int q = 0; q < 8; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[q]) : "v"(0x9e3779b9u));
    }
    for (int q = 0; q < 8; ++q) s += x[q];
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + wave] = what == NONE ? 0 : t1 - t0;
}

template <int LO, int HI>
static int run(const char *name, double *d_out, long long *d_cyc, int cus, int itm, int itv) {
  auto *fn = &coexec_kernel<LO, HI>;
  const size_t lds = 96 * 1024;  // one block per CU
  CK(hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(fn, dim3(cus), dim3(1024), lds, 0, d_out, d_cyc, itm, itv);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(fn, dim3(cus), dim3(1024), lds, 0, d_out, d_cyc, itm, itv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  long long *h = new long long[cus * 16];
  CK(hipMemcpy(h, d_cyc, sizeof(long long) * cus * 16, hipMemcpyDeviceToHost));
  double lo = 0, hi = 0;
  for (int b = 0; b < cus; ++b)
    for (int w = 0; w < 16; ++w) (w < 8 ? lo : hi) += (double)h[b * 16 + w];
  delete[] h;
  printf("%-14s %8.3f ms   mean clock64 cycles per wave: waves 0-7 %.3e, waves 8-15 %.3e\n", name,
         best, lo / (cus * 8), hi / (cus * 8));
  return 0;
}

int main(int argc, char **argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // trips: 8 MFMA4 per trip, 4 MFMA16 per trip, 8 fma / add per trip
  const int itm4 = 4000, itm16 = 2000, itv = 20000;
  double *d_out;
  long long *d_cyc;
  CK(hipMalloc(&d_out, (size_t)cus * 1024 * 8));
  CK(hipMalloc(&d_cyc, (size_t)cus * 16 * 8));
  printf("one 16-wave block per CU (%d CUs); waves 0-7: 2 per SIMD, waves 8-15: 2 more\n", cus);
  if (run<MFMA4, NONE>("mfma4", d_out, d_cyc, cus, itm4, itv) ||
      run<NONE, VALU64>("valu64", d_out, d_cyc, cus, itm4, itv) ||
      run<MFMA4, VALU64>("mfma4+valu64", d_out, d_cyc, cus, itm4, itv) ||
      run<NONE, VALU32>("valu32", d_out, d_cyc, cus, itm4, itv) ||
      run<MFMA4, VALU32>("mfma4+valu32", d_out, d_cyc, cus, itm4, itv) ||
      run<MFMA16, NONE>("mfma16", d_out, d_cyc, cus, itm16, itv) ||
      run<MFMA16, VALU64>("mfma16+valu64", d_out, d_cyc, cus, itm16, itv) ||
      run<MFMA16, VALU32>("mfma16+valu32", d_out, d_cyc, cus, itm16, itv))
    return 1;
  return 0;
}

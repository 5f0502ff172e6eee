// ubench_valu.hip -- gfx950 issue rates and operand layouts the backward kernel's
// design depends on (development tool, not part of the library):
//   * cycles per wave64 instruction (per SIMD, 4 waves per SIMD) of the fp64 /
//     int ops of the exp/log/recursion inner loop, and of v_mfma_f64_16x16x4 /
//     v_mfma_f64_4x4x4 (alone, and interleaved with independent fp64 FMAs);
//   * the lane maps of v_mfma_f64_4x4x4 (A, B, D) by one-hot probing;
//   * v_permlane16_swap / v_permlane32_swap semantics.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/ubench_valu scripts/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

typedef double double4_t __attribute__((ext_vector_type(4)));
#ifndef UB_ITERS
#define UB_ITERS 2048
#endif
constexpr int kIters = UB_ITERS;

enum Op { FMA64, ADD64, MUL64, MAX64, RNDNE64, CVT_PAIR, LDEXP64, AND32, ADDU32, FMA32,
          MFMA16, MFMA4, MFMA16_FMA, MFMA4_FMA, MADI24, BFI32, LSHLADD, SUBCLAMP, PERMLANE16,
          MOV32, CVTF64I32, FRMANT64, NOP_ };
static const char *kOpName[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_max_f64",
                                "v_rndne_f64", "cvt_i32_f64+cvt_f64_i32", "v_ldexp_f64",
                                "v_and_b32", "v_add_u32", "v_fma_f32", "mfma_f64_16x16x4",
                                "mfma_f64_4x4x4", "mfma16 + 16 fma_f64", "mfma4 + 4 fma_f64",
                                "v_mad_i32_i24", "v_bfi_b32", "v_lshl_add_u32", "v_sub_u32 clamp",
                                "v_permlane16_swap", "v_mov_b32", "v_cvt_f64_i32", "v_frexp_mant_f64"};

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(double *out, long long *cyc, double seed) {
  double a[8];
  int ia[8];
  float fa[8];
  double4_t acc[4];
  double macc[4];
  for (int q = 0; q < 8; ++q) {
    a[q] = seed + q + threadIdx.x * 1e-3;
    ia[q] = (int)threadIdx.x + q;
    fa[q] = (float)a[q];
  }
  for (int q = 0; q < 4; ++q) {
    acc[q] = double4_t{a[q], a[q], a[q], a[q]};
    macc[q] = a[q];
  }
  const double b = 1.0000001, c = 1e-9;
  const long long t0 = clock64();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if constexpr (OP == FMA64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[q]) : "v"(b), "v"(c));
      if constexpr (OP == ADD64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[q]) : "v"(c));
      if constexpr (OP == MUL64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[q]) : "v"(b));
      if constexpr (OP == MAX64) asm volatile("v_max_f64 %0, %0, %1" : "+v"(a[q]) : "v"(c));
      if constexpr (OP == RNDNE64) asm volatile("v_rndne_f64 %0, %0" : "+v"(a[q]));
      if constexpr (OP == CVT_PAIR) {
        int t;
        asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(t) : "v"(a[q]));
        asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(a[q]) : "v"(t));
      }
      if constexpr (OP == LDEXP64) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(a[q]) : "v"(0));
      if constexpr (OP == AND32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(ia[q]) : "v"(0x7fffffff));
      if constexpr (OP == ADDU32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ia[q]) : "v"(1));
      if constexpr (OP == FMA32) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(fa[q]) : "v"(1.0f), "v"(1e-9f));
      if constexpr (OP == MADI24) asm volatile("v_mad_i32_i24 %0, %0, %1, %2" : "+v"(ia[q]) : "v"(3), "v"(1));
      if constexpr (OP == BFI32) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(ia[q]) : "v"(0x000fffff), "v"(0x3ff00000));
      if constexpr (OP == LSHLADD) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(ia[q]) : "v"(7));
      if constexpr (OP == SUBCLAMP) asm volatile("v_sub_u32_e64 %0, %0, %1 clamp" : "+v"(ia[q]) : "v"(1));
      if constexpr (OP == PERMLANE16) {
        if (q % 2 == 0) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(ia[q]), "+v"(ia[q + 1]));
      }
      if constexpr (OP == MOV32) asm volatile("v_mov_b32 %0, %1" : "=v"(ia[q]) : "v"(ia[(q + 1) % 8]));
      if constexpr (OP == CVTF64I32) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(a[q]) : "v"(ia[q]));
      if constexpr (OP == FRMANT64) asm volatile("v_frexp_mant_f64 %0, %0" : "+v"(a[q]));
    }
    if constexpr (OP == MFMA16 || OP == MFMA16_FMA) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b, acc[q], 0, 0, 0);
      if constexpr (OP == MFMA16_FMA) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int q = 4; q < 8; ++q) asm volatile("v_fma_f64 %0, %0, %1, %2\n\tv_fma_f64 %0, %0, %1, %2" : "+v"(a[q]) : "v"(b), "v"(c));
      }
    }
    if constexpr (OP == MFMA4 || OP == MFMA4_FMA) {
#pragma unroll
      for (int q = 0; q < 4; ++q) macc[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[q], b, macc[q], 0, 0, 0);
      if constexpr (OP == MFMA4_FMA) {
#pragma unroll
        for (int q = 4; q < 8; ++q) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[q]) : "v"(b), "v"(c));
      }
    }
  }
  const long long t1 = clock64();
  double s = 0;
  for (int q = 0; q < 8; ++q) s += a[q] + ia[q] + fa[q];
  for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][3] + macc[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

// D of one v_mfma_f64_4x4x4 with A = one-hot at lane `hot` (value 1), B lane l = 1000 + l
__global__ void layout4_kernel(double *out) {
  const int l = threadIdx.x;
  for (int hot = 0; hot < 64; ++hot) {
    const double a = (l == hot) ? 1.0 : 0.0;
    const double b = 1000.0 + l;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[hot * 64 + l] = d;
  }
}
// the same with B one-hot (value 1), A lane l = 1000 + l
__global__ void layout4b_kernel(double *out) {
  const int l = threadIdx.x;
  for (int hot = 0; hot < 64; ++hot) {
    const double b = (l == hot) ? 1.0 : 0.0;
    const double a = 1000.0 + l;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[hot * 64 + l] = d;
  }
}

__global__ void permlane_kernel(int *out) {
  const int l = threadIdx.x;
  const unsigned x = 100 + l, y = 200 + l;
  auto r16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  auto r32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[0 * 64 + l] = r16[0];
  out[1 * 64 + l] = r16[1];
  out[2 * 64 + l] = r32[0];
  out[3 * 64 + l] = r32[1];
}

template <int OP>
static int run_rate(double *d_out, long long *d_cyc, int blocks) {
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 1.0);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(rate_kernel<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc, 1.0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> cyc(blocks * 4);
  CK(hipMemcpy(cyc.data(), d_cyc, cyc.size() * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for (auto c : cyc) avg += (double)c;
  avg /= cyc.size();
  // instructions per wave per iteration
  double ninst = 8;
  if (OP == CVT_PAIR) ninst = 16;
  if (OP == PERMLANE16) ninst = 4;
  if (OP == MFMA16 || OP == MFMA4) ninst = 4;
  if (OP == MFMA16_FMA) ninst = 4;   // cycles per MFMA with 16 fp64 FMAs alongside
  if (OP == MFMA4_FMA) ninst = 4;
  // waves per SIMD = blocks * 4 / (CUs * 4)
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double wps = (double)blocks * 4 / (cus * 4);
  const double cyc_per_inst = avg / (kIters * ninst) / wps;  // SIMD cycles per wave-instr
  const double clk_ghz = avg / (ms * 1e6);
  // wall-clock rate: wave-instructions per SIMD per ns (x 64 lanes x 2 flops for an FMA)
  const double winst = (double)blocks * 4 * kIters * ninst / (cus * 4);
  printf("%-28s %7.3f SIMD-cycles/wave-instr  (waves/SIMD %.1f, %.3f ms, clock ~%.2f GHz, "
         "%.3f ns/wave-instr/SIMD, fp64-FMA-equiv %.1f TF/s)\n",
         kOpName[OP], cyc_per_inst, wps, ms, clk_ghz, ms * 1e6 / winst,
         winst * cus * 4 * 128.0 / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus * 4;  // 16 waves per CU = 4 per SIMD
  double *d_out;
  long long *d_cyc;
  CK(hipMalloc(&d_out, (size_t)blocks * 256 * 8 + 64 * 64 * 8));
  CK(hipMalloc(&d_cyc, (size_t)blocks * 4 * 8));
  if (run_rate<FMA64>(d_out, d_cyc, blocks) || run_rate<ADD64>(d_out, d_cyc, blocks) ||
      run_rate<MUL64>(d_out, d_cyc, blocks) || run_rate<MAX64>(d_out, d_cyc, blocks) ||
      run_rate<RNDNE64>(d_out, d_cyc, blocks) || run_rate<CVT_PAIR>(d_out, d_cyc, blocks) ||
      run_rate<LDEXP64>(d_out, d_cyc, blocks) || run_rate<AND32>(d_out, d_cyc, blocks) ||
      run_rate<ADDU32>(d_out, d_cyc, blocks) || run_rate<FMA32>(d_out, d_cyc, blocks) ||
      run_rate<MFMA16>(d_out, d_cyc, blocks) || run_rate<MFMA4>(d_out, d_cyc, blocks) ||
      run_rate<MFMA16_FMA>(d_out, d_cyc, blocks) || run_rate<MFMA4_FMA>(d_out, d_cyc, blocks) ||
      run_rate<MADI24>(d_out, d_cyc, blocks) || run_rate<BFI32>(d_out, d_cyc, blocks) ||
      run_rate<LSHLADD>(d_out, d_cyc, blocks) || run_rate<SUBCLAMP>(d_out, d_cyc, blocks) ||
      run_rate<PERMLANE16>(d_out, d_cyc, blocks) || run_rate<MOV32>(d_out, d_cyc, blocks) ||
      run_rate<CVTF64I32>(d_out, d_cyc, blocks) || run_rate<FRMANT64>(d_out, d_cyc, blocks))
    return 1;
  // one wave per SIMD: latency-bound chains (8 independent) for reference
  printf("-- 1 wave per SIMD --\n");
  if (run_rate<FMA64>(d_out, d_cyc, cus) || run_rate<MFMA16>(d_out, d_cyc, cus) ||
      run_rate<MFMA4>(d_out, d_cyc, cus))
    return 1;
  std::vector<double> h(64 * 64);
  for (int which = 0; which < 2; ++which) {
    if (which == 0) hipLaunchKernelGGL(layout4_kernel, dim3(1), dim3(64), 0, 0, d_out);
    else hipLaunchKernelGGL(layout4b_kernel, dim3(1), dim3(64), 0, 0, d_out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost));
    printf("mfma_f64_4x4x4 %s one-hot: hot lane -> [out lane = other-operand lane]\n",
           which == 0 ? "A" : "B");
    for (int hot = 0; hot < 64; ++hot) {
      printf("  %2d:", hot);
      for (int l = 0; l < 64; ++l)
        if (h[hot * 64 + l] != 0.0) printf(" %d=%d", l, (int)h[hot * 64 + l] - 1000);
      printf("\n");
    }
  }
  int *d_i;
  CK(hipMalloc(&d_i, 4 * 64 * 4));
  hipLaunchKernelGGL(permlane_kernel, dim3(1), dim3(64), 0, 0, d_i);
  CK(hipDeviceSynchronize());
  std::vector<int> hi(4 * 64);
  CK(hipMemcpy(hi.data(), d_i, hi.size() * 4, hipMemcpyDeviceToHost));
  const char *nm[] = {"permlane16_swap(x=100+l, y=200+l)[0]", "permlane16_swap[1]",
                      "permlane32_swap[0]", "permlane32_swap[1]"};
  for (int r = 0; r < 4; ++r) {
    printf("%s:", nm[r]);
    for (int l = 0; l < 64; ++l) printf(" %d", hi[r * 64 + l]);
    printf("\n");
  }
  return 0;
}

// scripts/mfma_layout.hip -- probe the lane layout of v_mfma_f64_4x4x4f64 (4 blocks
// of 4x4x4) on gfx950: for every lane p, one MFMA with A = e_p (one-hot) and
// B[lane] = 2^lane, and one with A[lane] = 2^lane and B = e_p; D (one double per
// lane) is printed.  D[lane] = sum_k A[i][k] B[k][j] tells which A / B lanes feed
// which D lane.  hipcc --offload-arch=gfx950 -O2 -o /tmp/mfma_layout scripts/mfma_layout.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void probe(double *outA, double *outB) {
  const int lane = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    double a = lane == p ? 1.0 : 0.0, b = ldexp(1.0, lane);
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    outA[p * 64 + lane] = d;
    a = ldexp(1.0, lane);
    b = lane == p ? 1.0 : 0.0;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    outB[p * 64 + lane] = d;
  }
}

int main() {
  double *dA, *dB;
  hipMalloc(&dA, 64 * 64 * sizeof(double));
  hipMalloc(&dB, 64 * 64 * sizeof(double));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB);
  static double hA[64 * 64], hB[64 * 64];
  hipMemcpy(hA, dA, sizeof(hA), hipMemcpyDeviceToHost);
  hipMemcpy(hB, dB, sizeof(hB), hipMemcpyDeviceToHost);
  // A one-hot at p: which D lanes are nonzero, and log2 of their value (= the B lane)
  for (int p = 0; p < 64; ++p) {
    printf("A%d:", p);
    for (int l = 0; l < 64; ++l)
      if (hA[p * 64 + l] != 0.0) printf(" %d<-%d", l, (int)std::log2(hA[p * 64 + l]));
    printf("\n");
  }
  for (int p = 0; p < 64; ++p) {
    printf("B%d:", p);
    for (int l = 0; l < 64; ++l)
      if (hB[p * 64 + l] != 0.0) printf(" %d<-%d", l, (int)std::log2(hB[p * 64 + l]));
    printf("\n");
  }
  return 0;
}

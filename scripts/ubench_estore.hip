// E store-pattern microbenchmark: row-major 16-column tiles (4 rows x
// 128 B per store instruction, as emission_u_kernel writes E) against tile-major
// (512 contiguous bytes per instruction).  hipcc --offload-arch=gfx950 -O3 -o /tmp/wr
// scripts/ubench_estore.hip; profiles/r05aj_ubench_estore.txt
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
// E: rows x cols doubles, row-major (ld = cols).  Pattern A (current): wave writes a
// 16-col tile of 128 rows as 32 instructions of 4 rows x 16 cols (4 x 128 B segments).
// Pattern B (tile-major): the same values contiguous per tile (512 B per instruction).
__global__ void wrA(double *E, int rows, long long cols, int ntile) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const int kl = lane >> 4, cl = lane & 15;
  for (int t = wave; t < ntile; t += nw) {
    double *Ec = E + (long long)t * 16 + cl;
#pragma unroll 8
    for (int q = 0; q < rows / 4; ++q) Ec[(long long)(4 * q + kl) * cols] = (double)q;
  }
}
__global__ void wrB(double *E, int rows, long long cols, int ntile) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int t = wave; t < ntile; t += nw) {
    double *Et = E + (long long)t * 16 * rows + lane;
#pragma unroll 8
    for (int q = 0; q < rows / 4; ++q) Et[q * 64] = (double)q;
  }
}
int main() {
  const int rows = 128; const long long cols = 800000; const int ntile = cols / 16;
  double *E; hipMalloc(&E, rows * cols * 8);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int pat = 0; pat < 2; ++pat)
    for (int rep = 0; rep < 4; ++rep) {
      hipEventRecord(a);
      if (pat == 0) hipLaunchKernelGGL(wrA, dim3(768), dim3(256), 0, 0, E, rows, cols, ntile);
      else hipLaunchKernelGGL(wrB, dim3(768), dim3(256), 0, 0, E, rows, cols, ntile);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      printf("pattern %c: %.3f ms  %.2f TB/s\n", pat ? 'B' : 'A', ms, rows * cols * 8 / ms / 1e9);
    }
  return 0;
}

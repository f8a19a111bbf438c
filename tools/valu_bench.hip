// fp64 VALU throughput probe: independent mul+add chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CH>
__global__ __launch_bounds__(256) void k(double* out, int iters, double b) {
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = acc[c] * b + 1.0e-9;
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  double* d; hipMalloc(&d, 256 * 4096 * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int blocks : {256, 1024, 4096}) {
    const int iters = 4096;
    hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(256), 0, 0, d, iters, 0.999);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double ops = 2.0 * 16 * iters * (double)blocks * 256;  // mul + add lane-ops
    printf("blocks %5d: %.3f ms  %.2f T lane-ops/s (mul,add counted separately)\n", blocks, ms, ops / ms / 1e9);
  }
  return 0;
}

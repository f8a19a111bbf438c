// fp64 MFMA issue-rate microbenchmark: each wave runs ITERS x (MB x MB) independent
// v_mfma_f64_16x16x4_f64 on register operands.  hipcc --offload-arch=gfx950 -O3 tools/mfma_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int MB>
__global__ void k(double* out, int iters, double a0) {
  f64x4 acc[MB][MB];
  for (int m = 0; m < MB; ++m) for (int n = 0; n < MB; ++n) acc[m][n] = (f64x4){0, 0, 0, 0};
  double a[MB], b[MB];
  for (int m = 0; m < MB; ++m) { a[m] = a0 + threadIdx.x * 1e-3 + m; b[m] = a0 - m; }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int n = 0; n < MB; ++n) acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[n], acc[m][n], 0, 0, 0);
  }
  double s = 0;
  for (int m = 0; m < MB; ++m) for (int n = 0; n < MB; ++n) s += acc[m][n][0] + acc[m][n][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int MB> void run(int wgs, int threads, int iters) {
  double* out; hipMalloc(&out, (size_t)wgs * threads * 8);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<MB>, dim3(wgs), dim3(threads), 0, 0, out, 10, 1.0);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MB>, dim3(wgs), dim3(threads), 0, 0, out, iters, 1.0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double flops = (double)wgs * (threads / 64) * iters * MB * MB * 2048.0;
  printf("MB=%d wgs=%d thr=%d : %.3f ms  %.1f TFLOP/s\n", MB, wgs, threads, ms, flops / ms / 1e9);
  hipFree(out);
}
int main() {
  run<2>(256, 256, 20000); run<4>(256, 256, 5000); run<4>(512, 256, 5000);
  run<4>(1024, 256, 5000); run<2>(1024, 256, 20000); run<4>(256, 512, 5000);
  return 0;
}

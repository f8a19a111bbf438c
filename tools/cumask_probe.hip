// Which XCD does each bit of a hipExtStreamCreateWithCUMask mask select?  For every bit b of the
// first 256, a stream masked to that single CU runs a 64-block kernel; each block records its
// XCC_ID.  Prints "bit xcd" pairs (one line per bit).
//   hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe && tools/cumask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>

__global__ void k_where(int* out) {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = x & 15;
}

int main() {
  int* d = nullptr;
  if (hipMalloc(&d, 64 * sizeof(int)) != hipSuccess) return 2;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int b = 0; b < cus; ++b) {
    uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    mask[b / 32] = 1u << (b % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) return 3;
    hipLaunchKernelGGL(k_where, dim3(64), dim3(64), 0, s, d);
    int h[64];
    if (hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess) return 4;
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    int same = 1;
    for (int i = 1; i < 64; ++i) same &= h[i] == h[0];
    std::printf("%d %d%s\n", b, h[0], same ? "" : " mixed");
    (void)hipStreamDestroy(s);
  }
  return 0;
}

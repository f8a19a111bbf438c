// Operand / result map of v_mfma_i32_16x16x64_i8 on gfx950, checked with exact integer data
// (an asymmetric A and B).  Hypothesis: lane l holds A[l & 15][16 (l >> 4) + j] and
// B[16 (l >> 4) + j][l & 15] in byte j of its 16-byte fragment; D[4 (l >> 4) + r][l & 15] in
// accumulator register r.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_i8_probe.hip -o /tmp/mfma_i8_probe && /tmp/mfma_i8_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef long long i64x2 __attribute__((ext_vector_type(2)));

__global__ void k_probe(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];        // A is 16 x 64 row-major
    b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];      // B is 64 x 16 row-major
  }
  i64x2 fa, fb;
  __builtin_memcpy(&fa, a, 16);
  __builtin_memcpy(&fb, b, 16);
  i32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, fb, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; ++i) hA[i] = (int8_t)((rand() % 255) - 127);
  for (int i = 0; i < 64 * 16; ++i) hB[i] = (int8_t)((rand() % 255) - 127);
  int8_t *dA, *dB;
  int* dD;
  if (hipMalloc(&dA, sizeof(hA)) || hipMalloc(&dB, sizeof(hB)) || hipMalloc(&dD, 256 * sizeof(int))) return 2;
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  int hD[256];
  if (hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int k = 0; k < 64; ++k) s += hA[i * 64 + k] * hB[k * 16 + j];
      if (s != hD[i * 16 + j]) ++bad;
    }
  std::printf("mfma_i32_16x16x64_i8 map: %s (%d of 256 wrong)\n", bad ? "MISMATCH" : "ok", bad);
  return bad ? 1 : 0;
}

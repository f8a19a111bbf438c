// Packed lower triangle of the correlation matrix for the one RCCL all-reduce of the
// multi-GPU path (PODFS.py:1451-1455: C = np.dot(A.T, A) / ns, summed over row slabs).
//
// Packed layout: row r of the lower triangle (columns 0..r) starts at r(r+1)/2, so every row
// is contiguous both in C (row-major) and in the packed vector; the all-reduce moves
// n(n+1)/2 doubles instead of n^2.
//
//   k_pack_lower    one workgroup per row: packed[r(r+1)/2 + c] = C[r][c], c <= r
//   k_unpack_lower  one workgroup per 64 x 64 lower tile (bi >= bj): x = packed / divisor
//                   (IEEE division, numpy's `/ ns`), stored to C[r][c] and, through an LDS
//                   transpose, to C[c][r] -- both stores row-contiguous, C exactly symmetric.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "podsgen_kernels.h"
#include "podsgen_ext.h"

namespace pods {
namespace {

__device__ __forceinline__ int64_t tri_off(int64_t r) { return r * (r + 1) / 2; }

__global__ __launch_bounds__(256) void k_pack_lower(const double* __restrict__ C, int64_t ldc, int n,
                                                     double* __restrict__ packed) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const double* row = C + r * ldc;
  double* dst = packed + tri_off(r);
  for (int64_t c = threadIdx.x; c <= r; c += 256) dst[c] = row[c];
}

constexpr int UT = 64;

__global__ __launch_bounds__(256) void k_unpack_lower(const double* __restrict__ packed, int n, double divisor,
                                                       double* __restrict__ C, int64_t ldc) {
  // tile index -> (bi, bj), bj <= bi, row-major over the lower triangle of tiles
  const int64_t t = blockIdx.x;
  int64_t bi = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while (bi * (bi + 1) / 2 > t) --bi;
  while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
  const int64_t bj = t - bi * (bi + 1) / 2;
  __shared__ double tile[UT][UT + 1];
  const int tx = threadIdx.x % UT, ty = threadIdx.x / UT;  // 64 columns x 4 rows per pass
  const int64_t r0 = bi * UT, c0 = bj * UT;
  for (int rr = ty; rr < UT; rr += 4) {
    const int64_t r = r0 + rr, c = c0 + tx;
    double x = 0.0;
    if (r < n && c <= r) {
      x = packed[tri_off(r) + c] / divisor;
      C[r * ldc + c] = x;
    }
    tile[rr][tx] = x;
  }
  __syncthreads();
  // mirror: C[c][r] = x(r, c) for c < r; row c of the output tile is column c of the input
  for (int cc = ty; cc < UT; cc += 4) {
    const int64_t c = c0 + cc, r = r0 + tx;
    if (r < n && c < r) C[c * ldc + r] = tile[tx][cc];
  }
}

// snapshots i0..i1-1 of the K-tiled matrix (element (i, r) at ((r/16) ns + i) 16 + r%16) as
// rows of a (i1-i0) x rowlen row-major block: out[(i - i0) rowlen + r]
__global__ __launch_bounds__(256) void k_gather_snapshots(const double* __restrict__ AT, int ns, int64_t rowlen,
                                                           int i0, int w, double* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (int64_t)w * rowlen) return;
  const int64_t ii = idx / rowlen, r = idx - ii * rowlen;
  out[idx] = AT[(((r >> 4) * ns + i0 + ii) << 4) + (r & 15)];
}

}  // namespace

hipError_t launch_gather_snapshots(const double* AT, int ns, int64_t rowlen, int i0, int i1, double* out,
                                   hipStream_t st) {
  const int w = i1 - i0;
  if (w <= 0) return hipSuccess;
  const int64_t tot = (int64_t)w * rowlen;
  hipLaunchKernelGGL(k_gather_snapshots, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, AT, ns, rowlen,
                     i0, w, out);
  return hipGetLastError();
}

hipError_t launch_pack_lower(const double* C, int64_t ldc, int n, double* packed, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack_lower, dim3((unsigned)n), dim3(256), 0, st, C, ldc, n, packed);
  return hipGetLastError();
}

hipError_t launch_unpack_lower(const double* packed, int n, double divisor, double* C, int64_t ldc,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + UT - 1) / UT;
  hipLaunchKernelGGL(k_unpack_lower, dim3((unsigned)(nb * (nb + 1) / 2)), dim3(256), 0, st, packed, n, divisor,
                     C, ldc);
  return hipGetLastError();
}

}  // namespace pods

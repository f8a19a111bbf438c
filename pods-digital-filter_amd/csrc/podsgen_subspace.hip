// One step of the Chebyshev-filtered subspace iteration for the leading POD modes
// (podsgen/subspace.py; the eigenpairs PODFS.py:1309-1333 consumes):
//
//   out = alpha * (C Y) + beta * Y + gamma * Z        C: n x n, Y, Z, out: n x m (row-major)
//
// on fp64 MFMA (v_mfma_f64_16x16x4_f64).  A workgroup owns 16 rows x 64 columns of out; its
// 8 waves split the reduction over k into 8 contiguous ranges and their partial 16 x 64 tiles
// are summed through LDS in wave order (deterministic), the epilogue fusing the three-term
// recurrence.  Operand loads are 32-B vectors with no lane exchange: in MFMA sub-step s of a
// 16-k chunk, lane group g = lane / 16 contributes k = 16 kc + 4 g + s (A and B use the same
// k permutation, so the sum over the chunk is unchanged), and output column tile t holds the
// columns 4 (lane % 16) + t -- so a lane's A operands are one double4 of its C row and its B
// operands for all four tiles one double4 of a Y row.  The product is bandwidth/MFMA balanced
// at m = 64 (16 flop per byte of C); C (134 MB at ns = 4096) stays in the Infinity Cache across
// the filter's steps.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "podsgen_ext.h"

namespace pods {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int CB_WAVES = 8;

__device__ __forceinline__ f64x4 ld4(const double* p, int64_t base, int64_t off, int lim) {
  // p[base + off .. + 3], entries with off + i >= lim read as 0
  f64x4 v;
  if (off + 3 < lim) {
    v = *reinterpret_cast<const f64x4*>(p + base + off);
  } else {
    v[0] = off + 0 < lim ? p[base + off + 0] : 0.0;
    v[1] = off + 1 < lim ? p[base + off + 1] : 0.0;
    v[2] = off + 2 < lim ? p[base + off + 2] : 0.0;
    v[3] = off + 3 < lim ? p[base + off + 3] : 0.0;
  }
  return v;
}

__global__ __launch_bounds__(512) void k_cheb(const double* __restrict__ C, int64_t ldc, int n,
                                              const double* __restrict__ Y, const double* __restrict__ Z,
                                              int m, double alpha, double beta, double gamma,
                                              double* __restrict__ out) {
  __shared__ double red[CB_WAVES][16][64];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int g = l >> 4, li = l & 15;
  const int r0 = blockIdx.x * 16, c0 = blockIdx.y * 64;
  const int nch = (n + 15) / 16;
  const int per = (nch + CB_WAVES - 1) / CB_WAVES;
  const int kc0 = wave * per, kc1 = min(nch, kc0 + per);
  const int row = r0 + li;
  const bool rin = row < n;
  const int64_t abase = (int64_t)(rin ? row : 0) * ldc;
  f64x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
  f64x4 a, b[4], an, bn[4];
  auto load = [&](int kc, f64x4& aa, f64x4* bb) {
    const int k = kc * 16 + 4 * g;
    aa = rin ? ld4(C, abase, k, n) : f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int kr = k + s;
      bb[s] = kr < n ? *reinterpret_cast<const f64x4*>(Y + (int64_t)kr * m + c0 + 4 * li)
                     : f64x4{0.0, 0.0, 0.0, 0.0};
    }
  };
  if (kc0 < kc1) load(kc0, a, b);
  for (int kc = kc0; kc < kc1; ++kc) {
    if (kc + 1 < kc1) load(kc + 1, an, bn);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s][t], acc[t], 0, 0, 0);
    }
    a = an;
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = bn[s];
  }
  // D of tile t: column 4 li + t, row g + 4 reg
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][g + 4 * q][4 * li + t] = acc[t][q];
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * 64; e += 512) {
    const int rr = e >> 6, cc = e & 63;
    const int r = r0 + rr, c = c0 + cc;
    if (r >= n || c >= m) continue;
    double s = red[0][rr][cc];
#pragma unroll
    for (int w = 1; w < CB_WAVES; ++w) s += red[w][rr][cc];
    const int64_t o = (int64_t)r * m + c;
    double v = alpha * s;
    if (beta != 0.0) v = fma(beta, Y[o], v);
    if (gamma != 0.0) v = fma(gamma, Z[o], v);
    out[o] = v;
  }
}

}  // namespace

hipError_t launch_cheb_step(const double* C, int64_t ldc, int n, const double* Y, const double* Z, int m,
                            double alpha, double beta, double gamma, double* out, hipStream_t st) {
  if (n <= 0 || m <= 0 || m % 64 != 0) return hipErrorInvalidValue;
  if (!Z) gamma = 0.0;
  hipLaunchKernelGGL(k_cheb, dim3((unsigned)((n + 15) / 16), (unsigned)(m / 64)), dim3(512), 0, st, C, ldc, n, Y,
                     Z ? Z : Y, m, alpha, beta, gamma, out);
  return hipGetLastError();
}

}  // namespace pods

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

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "podsgen_ext.h"

namespace pods {
namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));


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

// Workgroup (256 threads) = 64 rows x 64 columns of out over one of KS ranges of k; wave w owns
// rows 16 w .. 16 w + 15.  Each C element feeds exactly one MFMA k-step of 4 column tiles
// (16 flop per byte of C), so the kernel is a stream of C at the fp64 MFMA rate (~5 TB/s): C
// is read in 64 x 64 tiles whose rows are 512 contiguous bytes (8 lanes x 64 B per row per
// load; MFMA-shaped loads -- 16 rows x 128 B per instruction -- streamed at 2.2 TB/s), staged
// through LDS together with the 64 x 64 chunk of Y that all four waves share; the next chunk
// is loaded into registers while the current one is multiplied.
// With KS > 1 each workgroup writes its partial tile and k_cheb_sum adds the KS partials in
// order (deterministic) and applies the recurrence; with KS = 1 the epilogue is applied here.
constexpr int CB_ROWS = 64;
constexpr int CB_K = 64;                 // k per chunk
constexpr int CB_CLD = CB_K + 4;         // LDS row stride of the C tile (doubles)
__global__ __launch_bounds__(256) void k_cheb(const double* __restrict__ C, int64_t ldc, int n,
                                              const double* __restrict__ Y, const double* __restrict__ Z,
                                              double alpha, double beta, double gamma, int kper,
                                              double* __restrict__ part, double* __restrict__ out) {
  __shared__ __attribute__((aligned(32))) double cs[CB_ROWS * CB_CLD];  // [row][k]
  __shared__ f64x4 ys[CB_K * 16];                                        // [k][column quad]
  const int t = threadIdx.x, wave = t >> 6, l = t & 63;
  const int g = l >> 4, li = l & 15;
  const int rb0 = blockIdx.x * CB_ROWS;
  const int ks = blockIdx.y;
  const int nch = (n + CB_K - 1) / CB_K;
  const int kc0 = ks * kper, kc1 = min(nch, kc0 + kper);
  const f64x4 zero4{0.0, 0.0, 0.0, 0.0};
  // loader mapping: C tile 64 x 64 = 1024 quads, thread t loads quads t + 256 p (p < 4):
  // row (t + 256 p) / 16, k quad (t % 16) -> 16 threads x 32 B = 512 B per row
  // Y chunk 64 x 64 = 1024 quads, thread t loads quads t + 256 p: k row (t + 256 p) / 16, quad t % 16
  f64x4 cr[4], yr[4];
  auto load = [&](int kc) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = t + 256 * p;
      const int rr = q >> 4, kq = (q & 15) * 4;
      const int r = rb0 + rr, k = kc * CB_K + kq;
      cr[p] = (kc < kc1 && r < n) ? ld4(C, (int64_t)r * ldc, k, n) : zero4;
      const int kr = kc * CB_K + rr;
      yr[p] = (kc < kc1 && kr < n) ? *reinterpret_cast<const f64x4*>(Y + (int64_t)kr * 64 + kq) : zero4;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = t + 256 * p;
      const int rr = q >> 4, kq = (q & 15) * 4;
      *reinterpret_cast<f64x4*>(&cs[rr * CB_CLD + kq]) = cr[p];
      ys[q] = yr[p];
    }
  };
  f64x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = zero4;
  const int arow = (wave * 16 + li) * CB_CLD;
  load(kc0);
  for (int kc = kc0; kc < kc1; ++kc) {
    __syncthreads();  // the previous chunk's operands have been read
    stage();
    __syncthreads();
    load(kc + 1);     // in flight during this chunk's MFMAs
#pragma unroll
    for (int kb = 0; kb < CB_K; kb += 16) {
      const f64x4 a = *reinterpret_cast<const f64x4*>(&cs[arow + kb + 4 * g]);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f64x4 b = ys[(kb + 4 * g + s) * 16 + li];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[q], acc[q], 0, 0, 0);
      }
    }
  }
  // D of column tile q: row g + 4 reg, column 4 li + q -> one double4 per (lane, reg)
  const int r0 = rb0 + wave * 16;
#pragma unroll
  for (int rg = 0; rg < 4; ++rg) {
    const int r = r0 + g + 4 * rg;
    if (r >= n) continue;
    const f64x4 v{acc[0][rg], acc[1][rg], acc[2][rg], acc[3][rg]};
    const int64_t o = (int64_t)r * 64 + 4 * li;
    if (part) {
      *reinterpret_cast<f64x4*>(part + (int64_t)ks * n * 64 + o) = v;
    } else {
      const f64x4 yv = *reinterpret_cast<const f64x4*>(Y + o);
      const f64x4 zv = *reinterpret_cast<const f64x4*>(Z + o);
      f64x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = fma(gamma, zv[e], fma(beta, yv[e], alpha * v[e]));
      *reinterpret_cast<f64x4*>(out + o) = w;
    }
  }
}

// out = alpha * sum_ks part[ks] + beta * Y + gamma * Z  (partials in order), double4 per thread
__global__ __launch_bounds__(256) void k_cheb_sum(const double* __restrict__ part, int ksn, int64_t nq,
                                                  const double* __restrict__ Y, const double* __restrict__ Z,
                                                  double alpha, double beta, double gamma,
                                                  double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // quad index
  if (i >= nq) return;
  const f64x4* P = reinterpret_cast<const f64x4*>(part);
  f64x4 s = P[i];
  for (int k = 1; k < ksn; ++k) {
    const f64x4 p = P[(int64_t)k * nq + i];
#pragma unroll
    for (int e = 0; e < 4; ++e) s[e] += p[e];
  }
  const f64x4 yv = reinterpret_cast<const f64x4*>(Y)[i];
  const f64x4 zv = reinterpret_cast<const f64x4*>(Z)[i];
  f64x4 w;
#pragma unroll
  for (int e = 0; e < 4; ++e) w[e] = fma(gamma, zv[e], fma(beta, yv[e], alpha * s[e]));
  reinterpret_cast<f64x4*>(out)[i] = w;
}

// ---- small dense pieces of the iteration: Gram matrices, Cholesky QR, block rotations ----
// (rocBLAS/rocSOLVER take 60-220 us for these n x 64 shapes: tools/topk_probe.py profile)
constexpr int GR_WG = 64;  // workgroups of a Gram product (partials summed in this order)

// part[w] = Y[rows_w]^T Z[rows_w], 64 x 64, on fp64 MFMA.  Each wave sums 4 rows per MFMA
// k-step over its row range; lane (li = l % 16, g = l / 16) loads Y and Z row k0 + g, columns
// 4 li .. 4 li + 3 (one double4 each), and tile (ti, tj) uses element ti of Y's and tj of Z's:
// tile row li is G row 4 li + ti, tile column li is G column 4 li + tj, so the D register q of
// the tile lands at G[4 (g + 4 q) + ti][4 li + tj].  The 4 waves' partials sum through LDS.
__global__ __launch_bounds__(256) void k_gram_mfma(const double* __restrict__ Y, const double* __restrict__ Z,
                                                   int n, int rows_per, double* __restrict__ part) {
  __shared__ double red[3][64 * 64];  // waves 1..3 park their 64 x 64 partials (wave 0 adds them)
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int g = l >> 4, li = l & 15;
  const int r0 = blockIdx.x * rows_per, r1 = min(n, r0 + rows_per);
  const int per = (r1 - r0 + 3) / 4;  // rows of this wave, a multiple of 4 apart from the tail
  const int w0 = r0 + ((per + 3) / 4 * 4) * wave, w1 = min(r1, w0 + (per + 3) / 4 * 4);
  f64x4 acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = f64x4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = w0; k0 < w1; k0 += 4) {
    const int k = k0 + g;
    const bool in = k < w1;
    const f64x4 y = in ? *reinterpret_cast<const f64x4*>(Y + (int64_t)k * 64 + 4 * li) : f64x4{0.0, 0.0, 0.0, 0.0};
    const f64x4 z = in ? *reinterpret_cast<const f64x4*>(Z + (int64_t)k * 64 + 4 * li) : f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
        acc[ti * 4 + tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(y[ti], z[tj], acc[ti * 4 + tj], 0, 0, 0);
  }
  // lane-local index of G entry: (ti, tj, q) -> G[4 (g + 4 q) + ti][4 li + tj]
  for (int w = 1; w < 4; ++w) {
    if (wave == w) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[w - 1][(e * 4 + q) * 64 + l] = acc[e][q];
    }
  }
  __syncthreads();
  if (wave == 0) {
    double* out = part + (int64_t)blockIdx.x * 64 * 64;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ti = e >> 2, tj = e & 3;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double v = acc[e][q];
        for (int w = 1; w < 4; ++w) v += red[w - 1][(e * 4 + q) * 64 + l];
        out[(4 * (g + 4 * q) + ti) * 64 + 4 * li + tj] = v;
      }
    }
  }
}

// G = the partials summed in workgroup order (deterministic)
__global__ __launch_bounds__(256) void k_gram_reduce(const double* __restrict__ part, int np, int m,
                                                     double* __restrict__ G) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= m * m) return;
  double s = 0.0;
  for (int w = 0; w < np; ++w) s += part[(int64_t)w * m * m + e];
  G[e] = s;
}

// One wave: G (64 x 64, symmetrised) = L L^T; Rinv = L^{-T} (upper triangular, row-major),
// so that X = Y Rinv has X^T X = I for G = Y^T Y.  Lane i holds row i of G / L in registers;
// the column of L just formed is broadcast through LDS.  A non-positive pivot gives NaN.
__global__ __launch_bounds__(64) void k_chol_inv(const double* __restrict__ G, double* __restrict__ Rinv) {
  __shared__ double col[64];
  __shared__ double Ls[64][65];
  const int i = threadIdx.x;
  double gr[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) gr[k] = 0.5 * (G[i * 64 + k] + G[k * 64 + i]);
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double d = __shfl(gr[j], j);
    const double ljj = d > 0.0 ? sqrt(d) : __builtin_nan("");
    const double lij = i == j ? ljj : gr[j] / ljj;
    gr[j] = i >= j ? lij : 0.0;
    col[i] = i > j ? lij : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = j + 1; k < 64; ++k) gr[k] = fma(-lij, col[k], gr[k]);
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int k = 0; k < 64; ++k) Ls[i][k] = gr[k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // lane c: column c of L^{-T} = R^{-1} (R = L^T): back substitution x_t for t = c .. 0,
  // x_c = 1 / R[c][c], x_t = -(sum_{k = t+1..c} R[t][k] x_k) / R[t][t], R[t][k] = L[k][t]
  const int c = i;
  double x[64];
#pragma unroll
  for (int t = 63; t >= 0; --t) {
    double s = t == c ? 1.0 : 0.0;
#pragma unroll
    for (int k = t + 1; k < 64; ++k) s = k <= c ? fma(-Ls[k][t], x[k], s) : s;
    x[t] = t <= c ? s / Ls[t][t] : 0.0;
  }
#pragma unroll
  for (int t = 0; t < 64; ++t) Rinv[t * 64 + c] = x[t];
}

// out = Y M (M m x m row-major); 16 rows per workgroup, a thread per (row, m/16 columns)
__global__ __launch_bounds__(256) void k_right_mul(const double* __restrict__ Y, const double* __restrict__ Mx,
                                                   int n, int m, double* __restrict__ out) {
  extern __shared__ double sh[];
  double* Ms = sh;          // m x m
  double* ys = sh + m * m;  // 16 x m
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * 16;
  for (int e = t; e < m * m; e += 256) Ms[e] = Mx[e];
  for (int e = t; e < 16 * m; e += 256) ys[e] = r0 + e / m < n ? Y[(int64_t)r0 * m + e] : 0.0;
  __syncthreads();
  const int cpt = m / 16;
  const int rr = t / 16, cb = t % 16;
  const int r = r0 + rr;
  if (r >= n) return;
  for (int q = 0; q < cpt; ++q) {
    const int c = cb + 16 * q;  // 16 consecutive threads store 16 consecutive columns
    double s0 = 0.0, s1 = 0.0;
    for (int k = 0; k < m; k += 2) {
      s0 = fma(ys[rr * m + k], Ms[k * m + c], s0);
      s1 = fma(ys[rr * m + k + 1], Ms[(k + 1) * m + c], s1);
    }
    out[(int64_t)r * m + c] = s0 + s1;
  }
}

}  // namespace

int gram_slices(int n) { return GR_WG; }

hipError_t launch_gram(const double* Y, const double* Z, int n, double* part, double* G, hipStream_t st) {
  const int rows_per = ((n + GR_WG - 1) / GR_WG + 15) / 16 * 16;
  hipLaunchKernelGGL(k_gram_mfma, dim3(GR_WG), dim3(256), 0, st, Y, Z, n, rows_per, part);
  hipLaunchKernelGGL(k_gram_reduce, dim3(16), dim3(256), 0, st, part, GR_WG, 64, G);
  return hipGetLastError();
}

hipError_t launch_chol_inv(const double* G, double* Rinv, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_inv, dim3(1), dim3(64), 0, st, G, Rinv);
  return hipGetLastError();
}

hipError_t launch_right_mul(const double* Y, const double* M, int n, int m, double* out, hipStream_t st) {
  if (m % 16) return hipErrorInvalidValue;
  const size_t lds = (size_t)(m * m + 16 * m) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_right_mul),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_right_mul, dim3((unsigned)((n + 15) / 16)), dim3(256), lds, st, Y, M, n, m, out);
  return hipGetLastError();
}

int cheb_splits(int n) {
  const int rb = (n + CB_ROWS - 1) / CB_ROWS;
  const int nch = (n + CB_K - 1) / CB_K;
  static const int target = std::getenv("PODS_CHEB_WG") ? std::atoi(std::getenv("PODS_CHEB_WG")) : 512;
  int ks = std::max(1, std::min(32, (target + rb / 2) / rb));  // ~2 workgroups per CU
  return std::max(1, std::min(ks, nch / 2));                 // >= 2 chunks per split
}

hipError_t launch_cheb_step(const double* C, int64_t ldc, int n, const double* Y, const double* Z, int m,
                            double alpha, double beta, double gamma, double* part, double* out, hipStream_t st) {
  if (n <= 0 || m != 64) return hipErrorInvalidValue;
  if (!Z) {
    Z = Y;
    gamma = 0.0;
  }
  const int ks = cheb_splits(n);
  const int nch = (n + CB_K - 1) / CB_K;
  const int kper = (nch + ks - 1) / ks;
  const int ksn = (nch + kper - 1) / kper;
  const dim3 grid((unsigned)((n + CB_ROWS - 1) / CB_ROWS), (unsigned)ksn);
  if (ksn == 1) {
    hipLaunchKernelGGL(k_cheb, grid, dim3(256), 0, st, C, ldc, n, Y, Z, alpha, beta, gamma, kper,
                       (double*)nullptr, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_cheb, grid, dim3(256), 0, st, C, ldc, n, Y, Z, alpha, beta, gamma, kper, part, out);
  const int64_t nq = (int64_t)n * 16;
  hipLaunchKernelGGL(k_cheb_sum, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, part, ksn, nq, Y, Z, alpha,
                     beta, gamma, out);
  return hipGetLastError();
}

}  // namespace pods

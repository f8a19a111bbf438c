// Kernels of the Chebyshev-filtered subspace iteration for the leading POD modes
// (podsgen/subspace.py; the eigenpairs PODFS.py:1309-1333 consumes):
//
//   k_cheb / k_cheb_sum   out = alpha (C Y) + beta Y + gamma Z on fp64 MFMA (v_mfma_f64_16x16x4),
//                         C from a 64 x 64-tiled copy (k_tile_c), split-K partials summed in
//                         order (deterministic), the filter's three-term recurrence fused into
//                         the epilogue
//   k_gram_mfma / _reduce 64 x 64 Gram matrices Y^T Z on fp64 MFMA
//   k_chol_inv            one wave: Cholesky of the Gram and R^{-1} (Cholesky QR)
//   k_right_mul           Y M or Z - Y M for a 64 x 64 M (CholQR's Y R^{-1}, Rayleigh-Ritz
//                         rotations and residual blocks)
//
// MFMA operand mapping (f64 16x16x4: A[l%16][l/16], B[l/16][l%16], D[l/16 + 4 r][l%16]): in
// sub-step s of a 16-k block, lane group g = l/16 contributes k = 16 kb + 4 g + s (A and B use
// the same k permutation, so a block's sum is unchanged), and column tile q holds columns
// 4 (l%16) + q -- so a lane's operands are whole 32-B pairs of LDS slots, no lane exchange.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

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
constexpr int CB_ROWS = 64;  // rows per workgroup = tile edge
constexpr int CB_K = 64;     // k per chunk = tile edge
// LDS images in 16-byte slots, bank-conflict-free for the MFMA operand reads (ds_read_b128 lane
// groups, checked exhaustively): C tile row r, k pair kk at r * 36 + r / 8 + kk; Y chunk row kr,
// column pair cc at kr * 32 + kr / 4 + cc.  (Unpadded, the B reads of lane groups g and g + 1
// hit the same banks: 2-way conflicts on every operand fetch.)
__device__ __forceinline__ int cs_slot(int r, int kk) { return r * 36 + (r >> 3) + kk; }
__device__ __forceinline__ int ys_slot(int kr, int cc) { return kr * 32 + (kr >> 2) + cc; }
constexpr int CS_SLOTS = 64 * 36 + 8;
constexpr int YS_SLOTS = 64 * 32 + 16;

// C re-laid out once per matrix into 64 x 64 tiles, tile (rb, kb) contiguous (32 KB, rows of
// 512 B), zero-padded to whole tiles: a workgroup's operand stream is then one contiguous
// range.  In row-major C the same stream is 64 rows x 512 B per chunk, 32 KB apart: every
// variant of the kernel on that layout ran at ~2 TB/s (65 us per step at ns = 4096).
__global__ __launch_bounds__(256) void k_tile_c(const double* __restrict__ C, int64_t ldc, int n, int nt,
                                                double* __restrict__ Ct) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // quad index in the tiled copy
  const int64_t tile = q >> 10, w = q & 1023;
  if (tile >= (int64_t)nt * nt) return;
  const int rb = (int)(tile / nt), kb = (int)(tile % nt);
  const int r = rb * 64 + (int)(w >> 4), k = kb * 64 + (int)(w & 15) * 4;
  const f64x4 v = r < n ? ld4(C, (int64_t)r * ldc, k, n) : f64x4{0.0, 0.0, 0.0, 0.0};
  reinterpret_cast<f64x4*>(Ct)[q] = v;
}

// Workgroup (256 threads) = 64 rows x 64 columns of out over one of KS ranges of k; wave w owns
// rows 16 w .. 16 w + 15.  Each C element feeds exactly one MFMA k-step of 4 column tiles
// (16 flop per byte of C): the kernel streams C at the fp64 MFMA rate, one 32 KB tile per
// chunk staged through LDS with the 64 x 64 chunk of Y that all four waves share; the next
// chunk is loaded into registers while the current one is multiplied.
// With KS > 1 each workgroup writes its partial tile and k_cheb_sum adds the KS partials in
// order (deterministic) and applies the recurrence; with KS = 1 the epilogue is applied here.
// Measured the same (55-58 us per step with the partial sum, r3): the C operand loaded
// straight into the MFMA registers from a copy laid out in operand order with only Y through
// LDS, either staged by ds_write or streamed by LDS-DMA into a 2-stage ring with one barrier
// per chunk; scheduling fences that keep each block's LDS reads 16 MFMAs ahead; two chunks of
// register prefetch; 4 or 16 K splits.  The fp64 MFMA pipe is busy 45 % of the kernel
// (profiles/r3/mfma_util_syrk_c3.json).  Measured slower in r4 (tools/cheb_bench.py, one call):
// every wave streaming its own operands from L2 straight into the MFMA registers, no LDS and no
// barriers, 140 against 57 us (four waves each pull the whole Y chunk: 512 MB of L2 reads per
// step); the split-K sum fused into this kernel (the last workgroup of a row block adds the
// partials), 127 us with an agent-scope release per workgroup (an XCD L2 write-back each) and
// 63.7 us with sc1 partial stores and loads (the last workgroup's loads are a serial tail).
__global__ __launch_bounds__(256) void k_cheb(const double* __restrict__ Ct, int nt, int n,
                                              const double* __restrict__ Y, const double* __restrict__ Z,
                                              double alpha, double beta, double gamma, int kper,
                                              double* __restrict__ part, double* __restrict__ out) {
  __shared__ double2 cs[CS_SLOTS];  // C tile [row][k]
  __shared__ double2 ys[YS_SLOTS];  // Y chunk [k][column]
  const int t = threadIdx.x, wave = t >> 6, l = t & 63;
  const int g = l >> 4, li = l & 15;
  const int rb = blockIdx.x;
  const int ks = blockIdx.y;
  const int kc0 = ks * kper, kc1 = min(nt, kc0 + kper);
  const f64x4 zero4{0.0, 0.0, 0.0, 0.0};
  const f64x4* Cq = reinterpret_cast<const f64x4*>(Ct) + (int64_t)rb * nt * 1024;
  // loader: tile quad q = t + 256 p -> row q / 16, k quad q % 16; Y chunk quad q -> k row q / 16
  // the loads of chunk kc + 1 are issued while chunk kc is multiplied (two chunks ahead
  // measured no faster: 55.8 vs 54.7 us per step)
  constexpr int PF = 1;
  f64x4 cr[PF][4], yr[PF][4];
  auto load = [&](int kc, int u) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = t + 256 * p;
      cr[u][p] = kc < kc1 ? Cq[(int64_t)kc * 1024 + q] : zero4;
      const int kr = kc * CB_K + (q >> 4);
      yr[u][p] = (kc < kc1 && kr < n) ? *reinterpret_cast<const f64x4*>(Y + (int64_t)kr * 64 + (q & 15) * 4)
                                      : zero4;
    }
  };
  auto stage = [&](int u) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int q = t + 256 * p;
      const int sc = cs_slot(q >> 4, (q & 15) * 2), sy = ys_slot(q >> 4, (q & 15) * 2);
      cs[sc] = double2{cr[u][p][0], cr[u][p][1]};
      cs[sc + 1] = double2{cr[u][p][2], cr[u][p][3]};
      ys[sy] = double2{yr[u][p][0], yr[u][p][1]};
      ys[sy + 1] = double2{yr[u][p][2], yr[u][p][3]};
    }
  };
  f64x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = zero4;
  const int arow = wave * 16 + li;
#pragma unroll
  for (int u = 0; u < PF; ++u) load(kc0 + u, u);
  for (int kb0 = kc0; kb0 < kc1; kb0 += PF)
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int kc = kb0 + u;
    if (kc >= kc1) break;
    __syncthreads();  // the previous chunk's operands have been read
    stage(u);
    __syncthreads();
    load(kc + PF, u);  // in flight during the next PF chunks' MFMAs
    // operands of a 16-k block (A: 4 doubles, B: 4 x 4) are read from LDS one block ahead, so
    // the 16 MFMAs of a block issue back to back in accumulator-rotating order (each
    // accumulator every 4th MFMA: dependent f64 MFMAs two apart ran the loop at half rate)
    {
      double a[4], b[4][4], an[4], bn[4][4];
      auto rd = [&](int kb, double* aa, double (*bb)[4]) {
        const int sa = cs_slot(arow, (kb + 4 * g) / 2);
        const double2 a0 = cs[sa], a1 = cs[sa + 1];
        aa[0] = a0.x; aa[1] = a0.y; aa[2] = a1.x; aa[3] = a1.y;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int sb = ys_slot(kb + 4 * g + s, 2 * li);
          const double2 b0 = ys[sb], b1 = ys[sb + 1];
          bb[s][0] = b0.x; bb[s][1] = b0.y; bb[s][2] = b1.x; bb[s][3] = b1.y;
        }
      };
      rd(0, a, b);
#pragma unroll
      for (int kb = 0; kb < CB_K; kb += 16) {
        if (kb + 16 < CB_K) rd(kb + 16, an, bn);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s][q], acc[q], 0, 0, 0);
        if (kb + 16 < CB_K) {
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            a[s] = an[s];
#pragma unroll
            for (int q = 0; q < 4; ++q) b[s][q] = bn[s][q];
          }
        }
      }
    }
  }
  // D of column tile q: row g + 4 reg, column 4 li + q -> one double4 per (lane, reg)
  const int r0 = rb * CB_ROWS + wave * 16;
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

// G = the partials summed in workgroup order (deterministic); all NP loads of a thread are
// issued before the first add (a rolled load-add loop waited one L2 round trip per partial)
template <int NP>
__global__ __launch_bounds__(256) void k_gram_reduce(const double* __restrict__ part, int m,
                                                     double* __restrict__ G) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= m * m) return;
  double v[NP];
#pragma unroll
  for (int w = 0; w < NP; ++w) v[w] = part[(int64_t)w * m * m + e];
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < NP; ++w) s += v[w];
  G[e] = s;
}

__device__ __forceinline__ double rdlane(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

// One wave: G (64 x 64, symmetrised) = L L^T; Rinv = L^{-T} (upper triangular, row-major),
// so that X = Y Rinv has X^T X = I for G = Y^T Y.  A non-positive pivot gives NaN.
// Lane i holds row i of G (the factorisation's trailing rows) and column i of Z = L^{-1}
// (forward substitution) in registers.  Step j takes the pivot from lane j (readlane), forms
// column j of L, broadcasts it through LDS, and applies it to BOTH: the trailing update
// g_ik -= l_ij l_kj and the substitution s_k -= l_kj z_j (k > j), whose z_j = s_j / l_jj is
// final at step j.  (Factorisation, then a separate back substitution: 74 us; fused: the
// substitution rides on the factorisation's column loads, tools/chol_bench.hip.)
__global__ __launch_bounds__(64) void k_chol_inv(const double* __restrict__ G, double* __restrict__ Rinv) {
  __shared__ double col[2][64];
  __shared__ double Zs[64][65];   // Zs[t][c] = Z[c][t] = Rinv[t][c]
  const int i = threadIdx.x;
  double gr[64], sv[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    gr[k] = 0.5 * (G[i * 64 + k] + G[k * 64 + i]);
    sv[k] = k == i ? 1.0 : 0.0;
  }
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double d = rdlane(gr[j], j);
    const double ljj = d > 0.0 ? sqrt(d) : __builtin_nan("");
    const double r = 1.0 / ljj;
    const double lij = gr[j] * r;   // lanes i > j: L[i][j] (other lanes' values are never read)
    const double zj = sv[j] * r;    // Z[j][i]
    Zs[i][j] = zj;
    col[j & 1][i] = lij;
    // the fences keep each step's column reads after its column write (and out of the
    // previous steps: hoisted, they take the kernel past 256 VGPRs)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = j + 1; k < 64; ++k) {
      const double lk = col[j & 1][k];
      gr[k] = fma(-lij, lk, gr[k]);
      sv[k] = fma(-zj, lk, sv[k]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int t = 0; t < 64; ++t) Rinv[t * 64 + i] = Zs[t][i];
}

// out = Y M (M m x m row-major), or Z - Y M with Z; 16 rows per workgroup, a thread per
// (row, m/16 columns)
__global__ __launch_bounds__(256) void k_right_mul(const double* __restrict__ Y, const double* __restrict__ Mx,
                                                   const double* __restrict__ Z, int n, int m,
                                                   double* __restrict__ out) {
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
    const int64_t o = (int64_t)r * m + c;
    out[o] = Z ? Z[o] - (s0 + s1) : s0 + s1;
  }
}

}  // namespace

int gram_slices(int n) { return GR_WG; }

hipError_t launch_gram(const double* Y, const double* Z, int n, double* part, double* G, hipStream_t st) {
  const int rows_per = ((n + GR_WG - 1) / GR_WG + 15) / 16 * 16;
  hipLaunchKernelGGL(k_gram_mfma, dim3(GR_WG), dim3(256), 0, st, Y, Z, n, rows_per, part);
  hipLaunchKernelGGL(k_gram_reduce<GR_WG>, dim3(16), dim3(256), 0, st, part, 64, G);
  return hipGetLastError();
}

hipError_t launch_chol_inv(const double* G, double* Rinv, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_inv, dim3(1), dim3(64), 0, st, G, Rinv);
  return hipGetLastError();
}

hipError_t launch_right_mul(const double* Y, const double* M, const double* Z, int n, int m, double* out,
                            hipStream_t st) {
  if (m % 16) return hipErrorInvalidValue;
  const size_t lds = (size_t)(m * m + 16 * m) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_right_mul),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_right_mul, dim3((unsigned)((n + 15) / 16)), dim3(256), lds, st, Y, M, Z, n, m, out);
  return hipGetLastError();
}

int cheb_splits(int n) {
  const int nt = (n + 63) / 64;
  // ~2 workgroups per CU (at n = 4096: 8 splits; 4 and 16 measured 58 and 61 against 55 us)
  const int ks = std::max(1, std::min(32, (512 + nt / 2) / nt));
  return std::max(1, std::min(ks, nt / 2));                          // >= 2 chunks per split
}

size_t cheb_tiled_doubles(int n) {
  const size_t nt = (size_t)(n + 63) / 64;
  return nt * nt * 64 * 64;
}

hipError_t launch_tile_c(const double* C, int64_t ldc, int n, double* Ct, hipStream_t st) {
  const int nt = (n + 63) / 64;
  const int64_t quads = (int64_t)nt * nt * 1024;
  hipLaunchKernelGGL(k_tile_c, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, st, C, ldc, n, nt, Ct);
  return hipGetLastError();
}

hipError_t launch_cheb_step(const double* Ct, int n, const double* Y, const double* Z, int m, double alpha,
                            double beta, double gamma, double* part, double* out, hipStream_t st) {
  if (n <= 0 || m != 64) return hipErrorInvalidValue;
  if (!Z) {
    Z = Y;
    gamma = 0.0;
  }
  const int nt = (n + 63) / 64;
  const int ks = cheb_splits(n);
  const int kper = (nt + ks - 1) / ks;
  const int ksn = (nt + kper - 1) / kper;
  const dim3 grid((unsigned)nt, (unsigned)ksn);
  auto kern = k_cheb;
  if (ksn == 1) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, Ct, nt, n, Y, Z, alpha, beta, gamma, kper, (double*)nullptr,
                       out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, Ct, nt, n, Y, Z, alpha, beta, gamma, kper, part, out);
  const int64_t nq = (int64_t)n * 16;
  hipLaunchKernelGGL(k_cheb_sum, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, part, ksn, nq, Y, Z, alpha,
                     beta, gamma, out);
  return hipGetLastError();
}

}  // namespace pods

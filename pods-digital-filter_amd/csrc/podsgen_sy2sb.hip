// Two-stage symmetric eigensolver for correlation matrices too large for the on-chip
// tridiagonalisation (pods_syev, n <= 4096): PODFS.py:1309-1310 at BASELINE configs 4/5
// (ns = 8192, 16384), where rocSOLVER dsyevd takes 0.67 s / several s.
//
//   stage 1  dense -> band (lower bandwidth B): per panel of B columns
//            k_pqr      Householder QR of the m x B panel below the band, rows spread over NW
//                       co-resident workgroups with ONE cross-CU hop per column (partial Gram
//                       rows + the pivot row are published, every workgroup forms the reflector
//                       redundantly); writes the explicit V (m x B), tau and R, and
//                       (one more hop: partial V^T V) T (dlarft 'F','C')
//            k_ay2      Y = A22 V on fp64 MFMA (split K)      \
//            k_xt       X = Y T                                |  W = X - 1/2 V T^T V^T X
//            k_z/k_zm   Z = V^T X, M = 1/2 T^T Z               |  (LAPACK dsytrd blocking)
//            k_w        W = X - V M                           /
//            k_upd      A22 -= V W^T + W V^T on fp64 MFMA, lower tiles mirrored (exactly
//                       symmetric)
//   stage 2  band -> tridiagonal by bulge chasing (k_sbtrd): sweep s annihilates column s
//            below the subdiagonal with Householders of length <= B, chasing the bulge down;
//            sweeps run concurrently on different workgroups, task (s, k) starting once
//            sweep s-1 has finished its task k+2 (the last task whose elements it shares)
//   eigenvalues  Sturm bisection of the tridiagonal (podsgen_eigen.hip)
//   vectors  inverse iteration on the BAND matrix (k_band_invit: banded LU with partial
//            pivoting of B - lambda I in an LDS window, two solves), cluster MGS (k_orth),
//            then Y <- Q1 Y with the stage-1 panels (k_bt_z / k_bt_t / k_bt_u).
// The algorithm's index bookkeeping is prototyped in tools/twostage_proto.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <cstdlib>

#include "podsgen_kernels.h"

namespace pods {
namespace sb {

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double ld_c(const double* p) {
  const unsigned long long u = __hip_atomic_load(
      const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(p)), __ATOMIC_RELAXED,
      __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ void st_c(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_f(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_f(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Pipelined coherent accesses (MI355X_MICROARCH.md "Valid forms": sc1 stores drained before
// the flag, sc1 loads after the poll): raw buffer loads/stores with the sc1 policy bit, no
// per-access wait (the agent-scope atomics above serialise: one round trip each).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double* base, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, (int)(n * 8), 0x00020000);
}
__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t r, int idx) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, (1u << 31) | 16u);
  return __builtin_bit_cast(double, q);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, int idx, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(
      __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v), r, idx * 8, 0, 16u);
}

constexpr int SPIN_LIMIT = 1 << 22;

// tagged granules: the tag rides in the two lowest mantissa bits of the published double
__device__ __forceinline__ double tagged(double v, uint32_t tag) {
  const long long b = (__double_as_longlong(v) & ~3ll) | (long long)(tag & 3u);
  return __longlong_as_double(b);
}
__device__ __forceinline__ bool tag_ok(double v, uint32_t tag) {
  return ((uint32_t)__double2loint(v) & 3u) == (tag & 3u);
}
// consumers use the value with the tag cleared: a published 0.0 stays 0.0 (tagged, it would be
// a denormal that passes dlarfg's sigma != 0 test) and every workgroup still sees equal bits
__device__ __forceinline__ double untag(double v) {
  return __longlong_as_double(__double_as_longlong(v) & ~3ll);
}

// ---------------------------------------------------------------------------------------
// k_pqr<B>: Householder QR of the panel P = A[r0:r0+m, c0:c0+B] (row-major A, ld lda).
// Workgroup w holds panel rows [w*RP, min((w+1)*RP, m)) in LDS.  Column j: partial
// s_k = sum_{r>j, local} P[r][j] P[r][k] (k >= j) and, from the owner of row j, P[j][k],
// are published; after the hop every workgroup sums the partials in workgroup order
// (identical bits everywhere), forms beta, tau, v = [1; P[j+1:, j] / (alpha - beta)] and
// w_k = v^T P[:, k] = P[j][k] + s_k / (alpha - beta), and updates its rows.
// Outputs: Vx (m x B explicit, unit diagonal, zeros above), tau (B), R into A's panel rows
// [0, B) (zeros below the diagonal and in rows >= B).
// ---------------------------------------------------------------------------------------
template <int B>
__global__ __launch_bounds__(256, 1) void k_pqr(double* __restrict__ A, int64_t lda, int r0, int c0, int m,
                                               int RP, int NW, double* __restrict__ pub,
                                               uint32_t* __restrict__ flags, uint32_t epoch, uint32_t seq0,
                                               uint32_t* __restrict__ abortw, double* __restrict__ Vx,
                                               double* __restrict__ tau, double* __restrict__ gpart,
                                               double* __restrict__ Tout, int64_t* __restrict__ ptrace) {
  static_assert(B == 32, "k_pqr: one half-wave per panel row group (lane = column)");
  constexpr int RG = 256 / B;   // 8 row groups (half-waves)
  constexpr int NR = 256 / RG;  // rows per thread: RP <= 256
  constexpr int LDP = B + 1;
  __shared__ double red[RG][B];
  __shared__ double S[B], rowjb[2][B], taul[B];
  __shared__ double gsum[64 * B];
  // column j of each row group, written by the lane holding it (kq == j) during column j-1's
  // update and read back by its half-wave (same wave: no barrier) in place of 32 shuffles
  __shared__ __attribute__((aligned(16))) double colb[RG][NR];
  __shared__ double G[B][LDP], Ts[B][LDP];
  const int w = blockIdx.x, t = threadIdx.x;
  const int kq = t % B, rg = t / B;
  const int g0 = w * RP, g1 = min(g0 + RP, m);
  const int nl = max(g1 - g0, 0);
  const int src0 = (t & 63) & ~(B - 1);  // lane 0 of this half-wave
  // P[i] = panel element (local row rg + RG*i, column kq), in registers
  double P[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = rg + RG * i;
    P[i] = r < nl ? A[(int64_t)(r0 + g0 + r) * lda + c0 + kq] : 0.0;
  }
  const int kc = min(m, B);
  int64_t* ptr = (ptrace && w == 0 && t == 0) ? ptrace : nullptr;  // diagnostics: per-column stamps
  auto stamp = [&](int j, int q) {
    if (ptr) ptr[j * 8 + q] = (int64_t)__builtin_amdgcn_s_memrealtime();
  };
  if (kq == 0) {
#pragma unroll
    for (int i = 0; i < NR; ++i) colb[rg][i] = P[i];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int j = 0; j < kc; ++j) {
    stamp(j, 0);
    double* rowj = rowjb[j & 1];  // double-buffered: no barrier at the end of the column
    // column j of my rows (lane j of the half-wave), broadcast from colb
    double pj[NR];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < NR; i += 2) {
      const double2 q = *reinterpret_cast<const double2*>(&colb[rg][i]);
      pj[i] = q.x;
      pj[i + 1] = q.y;
    }
    // rows rg + RG i with i >= B / RG lie past row B > j in every workgroup, and rows past
    // the panel hold zeros: only the first B / RG slots need the row conditions
    constexpr int IG = B / RG;
    double acc = 0.0, acc1 = 0.0;
#pragma unroll
    for (int i = 0; i < IG; ++i) {
      const int gr = g0 + rg + RG * i;
      if (gr > j && rg + RG * i < nl) acc = fma(pj[i], P[i], acc);
    }
#pragma unroll
    for (int i = IG; i < NR; i += 2) {
      acc = fma(pj[i], P[i], acc);
      acc1 = fma(pj[i + 1], P[i + 1], acc1);
    }
    acc += acc1;
    red[rg][kq] = kq >= j ? acc : 0.0;
    // the pivot row's owner keeps row j for the publish
    if (j >= g0 && j < g1 && rg == (j - g0) % RG) {
      const int i = (j - g0) / RG;
      double pr = 0.0;
#pragma unroll
      for (int q = 0; q < NR; ++q)
        if (q == i) pr = P[q];
      rowj[kq] = pr;
    }
    stamp(j, 1);
    __syncthreads();  // B1: the row-group partials are in red
    stamp(j, 2);
    // Hand-off without flags: every published double carries the column's tag in its two
    // lowest mantissa bits (the sequence number c = 16 panel + j/2 + 1 differs by 1 from the
    // previous write to the same slot, and the slots are zeroed per call), so consumers spin
    // on the data itself; no drain, no flag round trip.
    const __amdgpu_buffer_rsrc_t rpub = rsrc(pub, (int64_t)2 * NW * 2 * B);
    const int pbase = ((j & 1) * NW + w) * 2 * B;
    const uint32_t tag = seq0 + (uint32_t)(j >> 1);
    if (t < B) {
      double sp = 0.0;
#pragma unroll
      for (int q = 0; q < RG; ++q) sp += red[q][t];
      bst(rpub, pbase + t, tagged(sp, tag));
      if (j >= g0 && j < g1) bst(rpub, pbase + B + t, tagged(rowj[t], tag));
    }
    stamp(j, 3);
    {
      const int qb = (j & 1) * NW * 2 * B;
      const int own = j / RP;  // the workgroup holding pivot row j
      int spin = 0;
      for (;;) {
        bool ok = true;
        for (int e = t; e < NW * B; e += 256) {
          const double v = bld(rpub, qb + (e / B) * 2 * B + (e % B));
          ok = ok && tag_ok(v, tag);
          gsum[e] = untag(v);
        }
        if (t < B) {
          const double v = bld(rpub, qb + own * 2 * B + B + t);
          ok = ok && tag_ok(v, tag);
          rowj[t] = untag(v);
        }
        if (__all(ok)) break;
        if (++spin > SPIN_LIMIT) {
          st_f(abortw, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    stamp(j, 4);
    __syncthreads();  // B2: every partial and the pivot row are in LDS
    {  // S[k] = sum over workgroups: 8 interleaved partial sums (fixed order everywhere)
      double sacc = 0.0;
      for (int q = rg; q < NW; q += RG) sacc += gsum[q * B + kq];
      red[rg][kq] = sacc;
    }
    __syncthreads();  // B3
    if (t < B) {
      double sacc = red[0][t];
#pragma unroll
      for (int q = 1; q < RG; ++q) sacc += red[q][t];
      S[t] = sacc;
    }
    __syncthreads();  // B3b
    stamp(j, 5);
    // ---- reflector (dlarfg), redundantly in every thread -----------------------------
    const double alpha = rowj[j], sigma = S[j];
    double beta = alpha, tj = 0.0, scal = 0.0;
    if (sigma != 0.0) {
      beta = -copysign(sqrt(fma(alpha, alpha, sigma)), alpha);
      tj = (beta - alpha) / beta;
      scal = 1.0 / (alpha - beta);
    }
    if (t == 0) {
      taul[j] = tj;
      if (w == 0) tau[j] = tj;
    }
    const double wk = (kq > j) ? fma(scal, S[kq], rowj[kq]) : 0.0;
    const double f = -tj * wk;
#pragma unroll
    for (int i = 0; i < IG; ++i) {
      const int gr = g0 + rg + RG * i;
      if (gr < j) continue;
      const double v = gr == j ? 1.0 : scal * pj[i];
      if (kq > j) P[i] = fma(f, v, P[i]);
      else if (kq == j) P[i] = gr == j ? beta : v;
    }
    {  // rows past B: P <- P + f v (columns k > j; f = 0 below), v itself in column j
      const double fe = kq > j ? f : 0.0;
      const bool cj = kq == j;
#pragma unroll
      for (int i = IG; i < NR; ++i) {
        const double v = scal * pj[i];
        const double u = fma(fe, v, P[i]);
        P[i] = cj ? v : u;
      }
    }
    if (kq == j + 1) {  // the next column, for this half-wave
#pragma unroll
      for (int i = 0; i < NR; i += 2)
        *reinterpret_cast<double2*>(&colb[rg][i]) = make_double2(P[i], P[i + 1]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    stamp(j, 6);
    // no barrier here: rowj alternates, S and red are rewritten only after the next B1
  }
  if (ptr) ptr[kc * 8] = (int64_t)__builtin_amdgcn_s_memrealtime();
  // ---- outputs: explicit V and R; V (explicit) kept in registers for the Gram ----------
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = rg + RG * i;
    const int gr = g0 + r;
    if (r < nl) {
      const double pv = P[i];
      const double v = kq >= kc ? 0.0 : (gr > kq ? pv : (gr == kq ? 1.0 : 0.0));
      Vx[(int64_t)gr * B + kq] = v;
      A[(int64_t)(r0 + gr) * lda + c0 + kq] = (gr <= kq && gr < B) ? pv : 0.0;
      P[i] = v;
    } else {
      P[i] = 0.0;
    }
  }
  // ---- T (dlarft 'F','C'): G = V^T V (partials per workgroup) -> workgroup 0 -------------
  // thread (b = kq, rg): sum over its rows of V[r][a] V[r][b] for every a (V[r][a] from lane a)
  {
    double gacc[B];
#pragma unroll
    for (int aa = 0; aa < B; ++aa) gacc[aa] = 0.0;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
#pragma unroll
      for (int aa = 0; aa < B; ++aa) gacc[aa] = fma(__shfl(P[i], src0 + aa), P[i], gacc[aa]);
    }
    // reduce over the 8 row groups through LDS, one a-block at a time
    const __amdgpu_buffer_rsrc_t rgp = rsrc(gpart, (int64_t)NW * B * B);
    for (int a0 = 0; a0 < B; a0 += 8) {
#pragma unroll
      for (int aa = 0; aa < 8; ++aa) gsum[(rg * 8 + aa) * B + kq] = gacc[a0 + aa];
      __syncthreads();
      {
        const int aa = t / B, b = t % B;  // 256 threads = 8 a's x 32 b's
        double g = 0.0;
#pragma unroll
        for (int q = 0; q < RG; ++q) g += gsum[(q * 8 + aa) * B + b];
        bst(rgp, w * B * B + (a0 + aa) * B + b, g);
      }
      __syncthreads();
    }
  }
  drain();
  __syncthreads();
  const uint32_t wantg = epoch * 256u + 255u;
  if (t == 0) st_f(flags + w, wantg);
  if (w != 0) return;
  if (t < NW) {
    int spin = 0;
    while ((int)(ld_f(flags + t) - wantg) < 0) {
      if (++spin > SPIN_LIMIT) {
        st_f(abortw, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  {
    const __amdgpu_buffer_rsrc_t rgp = rsrc(gpart, (int64_t)NW * B * B);
    for (int e = t; e < B * B; e += 256) {
      double g = 0.0;
      for (int q = 0; q < NW; ++q) g += bld(rgp, q * B * B + e);
      G[e / B][e % B] = g;
      Ts[e / B][e % B] = 0.0;
    }
  }
  __syncthreads();
  for (int i = 0; i < B; ++i) {
    const double ti = i < kc ? taul[i] : 0.0;
    double v = 0.0;
    if (t < i) {
      for (int q = t; q < i; ++q) v = fma(Ts[t][q], G[q][i], v);
      v = -ti * v;
    }
    __syncthreads();
    if (t < i) Ts[t][i] = v;
    if (t == i) Ts[i][i] = ti;
    __syncthreads();
  }
  for (int e = t; e < B * B; e += 256) Tout[e] = Ts[e / B][e % B];
  if (t >= kc && t < B) tau[t] = 0.0;
}

// s = ((p_0 + p_1) + p_2) + ... over n partials at stride `stride` (the order of a plain loop),
// with the loads issued eight at a time so they are in flight together.
__device__ __forceinline__ double sum_partials(const double* __restrict__ p, int64_t stride, int n) {
  double s = 0.0;
  int q = 0;
  for (; q + 8 <= n; q += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)(q + u) * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; q < n; ++q) s += p[(int64_t)q * stride];
  return s;
}

// Y_s = A22[:, k-slice s] Vx[k-slice s, :], bandwidth-shaped: 64 x B output block per
// workgroup, K staged 32 at a time through LDS with the next slice's A / V loads in flight
// (registers) while the current one feeds the MFMAs.  Enough (row block, split) pairs to put
// several workgroups on every CU (the A22 read is the kernel's whole cost: ~m^2 doubles).
template <int B>
__global__ __launch_bounds__(256) void k_ay2(const double* __restrict__ A, int64_t lda, int r0, int m,
                                             const double* __restrict__ Vx, int kchunk,
                                             double* __restrict__ Y) {
  constexpr int KC = 32, LDA_S = KC + 2, LDV = B + 2;
  constexpr int AL = 64 * KC / 256;  // A loads per thread per slice: 8
  constexpr int VL = KC * B / 256;   // V loads per thread per slice: 4
  __shared__ double As[64 * LDA_S];
  __shared__ double Vs[KC * LDV];
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const int fr = lane & 15, fk = lane >> 4;
  const int i0 = blockIdx.x * 64;
  const int k0 = blockIdx.y * kchunk, k1 = min(m, k0 + kchunk);
  f64x4 acc[B / 16];
#pragma unroll
  for (int c = 0; c < B / 16; ++c) acc[c] = (f64x4){0.0, 0.0, 0.0, 0.0};
  double ra[AL], rv[VL];
  auto load = [&](int kb) {
#pragma unroll
    for (int u = 0; u < AL; ++u) {
      const int e = t + 256 * u, r = e / KC, k = e % KC;
      const int gi = i0 + r, gk = kb + k;
      ra[u] = (gi < m && gk < k1) ? A[(int64_t)(r0 + gi) * lda + r0 + gk] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < VL; ++u) {
      const int e = t + 256 * u, k = e / B, c = e % B;
      const int gk = kb + k;
      rv[u] = gk < k1 ? Vx[(int64_t)gk * B + c] : 0.0;
    }
  };
  if (k0 < k1) load(k0);
  for (int kb = k0; kb < k1; kb += KC) {
    __syncthreads();  // the previous slice's fragments are consumed
#pragma unroll
    for (int u = 0; u < AL; ++u) {
      const int e = t + 256 * u;
      As[(e / KC) * LDA_S + e % KC] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < VL; ++u) {
      const int e = t + 256 * u;
      Vs[(e / B) * LDV + e % B] = rv[u];
    }
    __syncthreads();
    if (kb + KC < k1) load(kb + KC);  // in flight under this slice's MFMAs
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const double a = As[(16 * wv + fr) * LDA_S + kk + fk];
#pragma unroll
      for (int c = 0; c < B / 16; ++c) {
        const double b = Vs[(kk + fk) * LDV + 16 * c + fr];
        acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
      }
    }
  }
  double* Yb = Y + (int64_t)blockIdx.y * m * B;
#pragma unroll
  for (int c = 0; c < B / 16; ++c)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int gi = i0 + 16 * wv + fk + 4 * reg;
      if (gi < m) Yb[(int64_t)gi * B + 16 * c + fr] = acc[c][reg];
    }
}

// X = (sum_s Y_s) T, 256/B rows per block.
template <int B>
__global__ __launch_bounds__(256) void k_xt(const double* __restrict__ Y, int KS, int m,
                                            const double* __restrict__ T, double* __restrict__ X) {
  constexpr int RB = 256 / B;
  __shared__ double Ts[B][B + 1];
  __shared__ double Ys[RB][B + 1];
  const int t = threadIdx.x, rr = t / B, c = t % B;
  for (int e = t; e < B * B; e += 256) Ts[e / B][e % B] = T[e];
  const int i = blockIdx.x * RB + rr;
  double s = 0.0;
  if (i < m)
    s = sum_partials(Y + (int64_t)i * B + c, (int64_t)m * B, KS);
  Ys[rr][c] = s;
  __syncthreads();
  if (i >= m) return;
  double x = 0.0;
  for (int l = 0; l <= c; ++l) x = fma(Ys[rr][l], Ts[l][c], x);  // T upper triangular
  X[(int64_t)i * B + c] = x;
}

// Partials of Z = Vx^T X over row chunks: block q handles rows [q*chunk, ...).
template <int B>
__global__ __launch_bounds__(256) void k_z(const double* __restrict__ Vx, const double* __restrict__ X, int m,
                                           int chunk, double* __restrict__ Zp) {
  constexpr int RT = 32;
  __shared__ double Vs[RT][B + 1];
  __shared__ double Xs[RT][B + 1];
  const int t = threadIdx.x;
  constexpr int PER = B * B / 256;  // entries per thread
  double acc[PER > 0 ? PER : 1];
#pragma unroll
  for (int q = 0; q < (PER > 0 ? PER : 1); ++q) acc[q] = 0.0;
  const int a0 = blockIdx.x * chunk, a1 = min(m, a0 + chunk);
  for (int rb = a0; rb < a1; rb += RT) {
    for (int e = t; e < RT * B; e += 256) {
      const int r = e / B, c = e % B;
      const bool ok = rb + r < a1;
      Vs[r][c] = ok ? Vx[(int64_t)(rb + r) * B + c] : 0.0;
      Xs[r][c] = ok ? X[(int64_t)(rb + r) * B + c] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < (PER > 0 ? PER : 1); ++q) {
      const int e = t + 256 * q;
      if (e < B * B) {
        const int a = e / B, b = e % B;
        double s = acc[q];
        for (int r = 0; r < RT; ++r) s = fma(Vs[r][a], Xs[r][b], s);
        acc[q] = s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < (PER > 0 ? PER : 1); ++q) {
    const int e = t + 256 * q;
    if (e < B * B) Zp[(int64_t)blockIdx.x * B * B + e] = acc[q];
  }
}

// M = 1/2 T^T Z, Z = sum of the nz partials (in order).
template <int B>
__global__ __launch_bounds__(256) void k_zm(const double* __restrict__ Zp, int nz, const double* __restrict__ T,
                                            double* __restrict__ M) {
  __shared__ double Z[B][B + 1];
  const int t = threadIdx.x;
  for (int e = t; e < B * B; e += 256) {
    double s = 0.0;
    s = sum_partials(Zp + e, (int64_t)B * B, nz);
    Z[e / B][e % B] = s;
  }
  __syncthreads();
  __shared__ double Tl[B][B + 1];
  for (int e = t; e < B * B; e += 256) Tl[e / B][e % B] = T[e];
  __syncthreads();
  for (int e = t; e < B * B; e += 256) {
    const int a = e / B, b = e % B;
    double s = 0.0;
    for (int l = 0; l <= a; ++l) s = fma(Tl[l][a], Z[l][b], s);  // (T^T)[a][l] = T[l][a], l <= a
    M[e] = 0.5 * s;
  }
}

// W = X - Vx M
template <int B>
__global__ __launch_bounds__(256) void k_w(const double* __restrict__ X, const double* __restrict__ Vx,
                                           const double* __restrict__ M, int m, double* __restrict__ W) {
  constexpr int RB = 256 / B;
  __shared__ double Ms[B][B + 1];
  __shared__ double Vs[RB][B + 1];
  const int t = threadIdx.x, rr = t / B, c = t % B;
  for (int e = t; e < B * B; e += 256) Ms[e / B][e % B] = M[e];
  const int i = blockIdx.x * RB + rr;
  Vs[rr][c] = i < m ? Vx[(int64_t)i * B + c] : 0.0;
  __syncthreads();
  if (i >= m) return;
  double s = X[(int64_t)i * B + c];
  for (int l = 0; l < B; ++l) s = fma(-Vs[rr][l], Ms[l][c], s);
  W[(int64_t)i * B + c] = s;
}

// A22 <- A22 - V W^T - W V^T on lower 64x64 tiles (fp64 MFMA, K = 2B), each tile written
// to its place and, transposed through LDS, to the mirrored upper tile.
template <int B>
__global__ __launch_bounds__(256) void k_upd(double* __restrict__ A, int64_t lda, int r0, int m,
                                             const double* __restrict__ Vx, const double* __restrict__ W) {
  constexpr int K2 = 2 * B, LD = K2 + 2;
  // Ls | Rs during the MFMAs, then the 64 x 65 transpose staging (aliased: 2 blocks per CU)
  __shared__ double sh_upd[2 * 64 * LD];
  double* Ls = sh_upd;
  double* Rs = sh_upd + 64 * LD;
  double (*Ot)[65] = reinterpret_cast<double (*)[65]>(sh_upd);
  static_assert(64 * 65 <= 2 * 64 * LD, "transpose staging fits the operand buffers");
  const int L = blockIdx.x;
  int ti = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
  while (ti * (ti + 1) / 2 > L) --ti;
  const int tj = L - ti * (ti + 1) / 2;
  const int i0 = ti * 64, j0 = tj * 64;
  const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const int fr = lane & 15, fk = lane >> 4;
  // the A tile's loads go out first: they overlap the V / W staging and the MFMAs
  double aold[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int li = 16 * wv + fk + 4 * reg, lj = 16 * c + fr;
      const int gi = i0 + li, gj = j0 + lj;
      aold[c][reg] = (gi < m && gj < m) ? A[(int64_t)(r0 + gi) * lda + r0 + gj] : 0.0;
    }
  // L row i = [V_i, W_i], R row j = [W_j, V_j]: sum_k L_ik R_jk = V_i.W_j + W_i.V_j.
  // All 2 x 16 operand loads of a thread go out before any LDS store (a rolled load -> store
  // loop paid one L2 round trip per element pair: 26 us per tile, 2 TB/s for the kernel).
  static_assert(K2 == 64, "thread t stages column k = t % 64 of rows 4 it + t / 64");
  {
    constexpr int NIT = 64 * K2 / 256;
    const int k = t & (K2 - 1), rb = t >> 6;
    const double* lsrc = k < B ? Vx + k : W + (k - B);
    const double* rsrc = k < B ? W + k : Vx + (k - B);
    double lv[NIT], rv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = 4 * it + rb;
      const int gi = i0 + r, gj = j0 + r;
      lv[it] = gi < m ? lsrc[(int64_t)gi * B] : 0.0;
      rv[it] = gj < m ? rsrc[(int64_t)gj * B] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int r = 4 * it + rb;
      Ls[r * LD + k] = lv[it];
      Rs[r * LD + k] = rv[it];
    }
  }
  __syncthreads();
  f64x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = (f64x4){0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int kk = 0; kk < K2; kk += 4) {
    const double a = Ls[(16 * wv + fr) * LD + kk + fk];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const double b = Rs[(16 * c + fr) * LD + kk + fk];
      acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave's fragments are read before Ot overwrites them
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int li = 16 * wv + fk + 4 * reg, lj = 16 * c + fr;
      const int gi = i0 + li, gj = j0 + lj;
      double v = 0.0;
      if (gi < m && gj < m) {
        v = aold[c][reg] - acc[c][reg];
        if (ti > tj || lj <= li) A[(int64_t)(r0 + gi) * lda + r0 + gj] = v;
      }
      Ot[li][lj] = v;
    }
  if (ti == tj) {
    __syncthreads();
    // diagonal tile: the upper half from the lower half (exact symmetry)
    for (int e = t; e < 64 * 64; e += 256) {
      const int li = e / 64, lj = e % 64;
      const int gi = i0 + li, gj = j0 + lj;
      if (lj > li && gi < m && gj < m) A[(int64_t)(r0 + gi) * lda + r0 + gj] = Ot[lj][li];
    }
    return;
  }
  __syncthreads();
  for (int e = t; e < 64 * 64; e += 256) {
    const int li = e / 64, lj = e % 64;  // upper tile element (j0 + li, i0 + lj) = lower (i0 + lj, j0 + li)
    const int gi = j0 + li, gj = i0 + lj;
    if (gi < m && gj < m) A[(int64_t)(r0 + gi) * lda + r0 + gj] = Ot[lj][li];
  }
}

// Band storage: band[c * LDB + d] = A[c + d][c], d in [0, LDB) (LDB = 2B: the band plus the
// bulge space of stage 2).
template <int B>
__global__ void k_band(const double* __restrict__ A, int64_t lda, int n, double* __restrict__ band) {
  constexpr int LDB = 2 * B;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * LDB) return;
  const int c = (int)(e / LDB), d = (int)(e % LDB);
  band[e] = (d <= B && c + d < n) ? A[(int64_t)(c + d) * lda + c] : 0.0;
}

// ---------------------------------------------------------------------------------------
// Stage 2, windowed: k_sbtrd_win<B, G>.  Bulge chasing in tasks (s, k):
// Task (s, k): rows R_k = [r0, r1), r0 = s+1+k*B (k = 0: the column s itself is the target);
// the Householder annihilates A[r0+1:r1, col] (col = s for k = 0, else the first column of
// the previous bulge, s+1+(k-1)*B) and is applied to A[R_k, col:r0] (left), A[R_k, R_k]
// (both sides) and A[r1:r1+B, R_k] (right; the new bulge).
// Task (s, k) follows (s-1, k+2).  (One wave per task over L2, each task handed off through
// memory, took 198 against ~100 ms at n = 8192.)  The tasks are scheduled so the chase runs
// out of LDS:
//   * a workgroup runs a GROUP of G consecutive sweeps s0 .. s0+G-1 in lock step: at step
//     tau, task wave g runs task (s0+g, tau - 3g).  The 3-task lag is the chase's dependency
//     ((s, k) after (s-1, k+2)) and the tasks of one step touch disjoint band elements, so
//     one workgroup barrier per step orders everything;
//   * the group's band columns live in an LDS ring of W = 8B column slots of 64 doubles
//     (element (row, cc) at slot(cc) * 64 + row - cc: a task lane reading down its column, or
//     a task row across columns, meets 32 different bank pairs), in blocks
//     b = [s0 + bB, s0 + (b+1)B): block b is first touched at step b - 1, and is final for
//     this group after step b + 4 (the trailing sweep's next column has passed it);
//   * a LOADER wave requests block tau+3 by LDS-DMA during step tau into the slots of block
//     tau-5, once the WRITER has read those, and makes sure block tau+2 has landed before the
//     step's barrier (a fixed vmcnt: every step issues exactly one block of DMA, past the
//     matrix into a junk slot);
//   * the WRITER wave writes block tau-5 back (one block of 16-B stores every step, into a
//     scratch block when none is due) and publishes gprog[q] = the end of the block it stored
//     one step earlier, after draining those stores;
//   * a POLLER wave polls gprog[q-1] (the previous group's written-back boundary) into LDS,
//     where the loader waits for it.
//   Workgroup w runs groups w, w + P, ... (persistent grid).
// ---------------------------------------------------------------------------------------
// Cross-lane helpers for one wave64 (gfx950): lane l's partner l ^ 32 and l ^ 16 by the
// permlane swaps, a 32-lane sum by a DPP butterfly (xor 1, 2, then the mirrors, which pair
// lanes holding equal partial sums) and the permlane16 swap; a lane broadcast by readlane.
__device__ __forceinline__ double lane_read(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}
__device__ __forceinline__ double lane_xor32(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const bool up = __lane_id() >= 32;
  return __hiloint2double((int)(up ? b[0] : b[1]), (int)(up ? a[0] : a[1]));
}
__device__ __forceinline__ double lane_xor16(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const bool odd = (__lane_id() >> 4) & 1;
  return __hiloint2double((int)(odd ? b[0] : b[1]), (int)(odd ? a[0] : a[1]));
}
template <int CTL>
__device__ __forceinline__ double lane_dpp(double x) {
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(x), CTL, 0xf, 0xf, false),
                          __builtin_amdgcn_mov_dpp(__double2loint(x), CTL, 0xf, 0xf, false));
}
__device__ __forceinline__ double lane_sum32(double x) {
  x += lane_dpp<0xB1>(x);   // quad_perm [1, 0, 3, 2]: l ^ 1
  x += lane_dpp<0x4E>(x);   // quad_perm [2, 3, 0, 1]: l ^ 2
  x += lane_dpp<0x141>(x);  // row_half_mirror: the other quad of the eight
  x += lane_dpp<0x140>(x);  // row_mirror: the other eight of the row
  x += lane_xor16(x);
  return x;
}

// sum over qq of a[qq] * b[qq], two interleaved chains
__device__ __forceinline__ double dot16(const double (&a)[16], const double (&b)[16]) {
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int qq = 0; qq < 16; qq += 2) {
    s0 = fma(a[qq], b[qq], s0);
    s1 = fma(a[qq + 1], b[qq + 1], s1);
  }
  return s0 + s1;
}

template <int B, int G>
struct SbWin {
  static constexpr int LDB = 2 * B;
  static constexpr int NBLK = 8;               // ring blocks: tau-5 .. tau+2 (+ tau+3 reusing tau-5)
  static constexpr int W = NBLK * B;
  static constexpr int NT = 64 * (G + 3);      // G task waves, loader, writer, poller
  static constexpr int PER = B * LDB / 2 / 64;  // 16-B pieces per lane per block: 16
  static constexpr size_t lds_bytes = (size_t)(LDB + W * LDB + 2 * LDB + G * 2 * B) * sizeof(double);
};

template <int B, int G>
__global__ __launch_bounds__(64 * (G + 3), 1) void k_sbtrd_win(double* __restrict__ band, int n, int qbeg,
                                                                int qend, uint32_t* __restrict__ gprog,
                                                                uint32_t* __restrict__ abortw,
                                                                double* __restrict__ scratch,
                                                                int64_t* __restrict__ wtr, int wq0) {
  static_assert(B == 32, "the task maps a 32 x 32 block onto one wave (lane = column, half of the rows)");
  using P = SbWin<B, G>;
  constexpr int LDB = P::LDB, W = P::W, H = B / 2, PER = P::PER;
  constexpr int LOADER = G, WRITER = G + 1, POLLER = G + 2;
  extern __shared__ __attribute__((aligned(1024))) double sb_sh[];
  double* ring = sb_sh + LDB;         // [W][LDB], after a zero pad: stray task reads stay finite
  double* junk = ring + W * LDB;       // two slots: the DMA target past the matrix
  double* wv_all = junk + 2 * LDB;     // per task wave: vs[B], wvec[B]
  __shared__ int s_avail, s_wread;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c = lane & (B - 1), h = lane >> 5;
  typedef double double2v __attribute__((ext_vector_type(2)));
  const int nbytes = n * LDB * 8;
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(band, 0, nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(scratch + (int64_t)blockIdx.x * B * LDB, 0,
                                                                       B * LDB * 8, 0x00020000);
  const uint32_t ring_lds = (uint32_t)(uintptr_t)ring, junk_lds = (uint32_t)(uintptr_t)junk;
  // Every LDS double a task may read is finite: the pad, the ring and the vectors start at zero
  // and only ever receive band values, so a task reads whole rows/columns unmasked and lets
  // zero entries of v (and of w) cancel what lies outside its block; its stores outside the
  // block go to a junk slot per lane instead of being masked.
  for (int i = t; i < (int)(P::lds_bytes / sizeof(double)); i += P::NT) sb_sh[i] = 0.0;
  const int jk = W * LDB + lane;  // this lane's junk element (ring-relative)
  // element d of band column cc in the ring
  auto ri = [&](int cc, int d) -> int { return (cc % W) * LDB + d; };
  auto ntask = [&](int s) -> int { return s < n - 2 ? (n - 2 - s + B - 1) / B : 0; };
  // groups [qbeg, qend) of this launch; every group before qbeg finished in an earlier launch
  for (int q = qbeg + blockIdx.x; q < qend; q += gridDim.x) {
    const int s0 = q * G;  // even: the two columns of one DMA share an even slot pair
    const int gq = min(G, n - 2 - s0);
    const int tend = ntask(s0) + 3 * (gq - 1);
    const int nblk = (n - s0 + B - 1) / B;
    auto blk_end = [&](int b) -> int { return min(n, s0 + (b + 1) * B); };
    if (t == 0) {
      s_avail = q == qbeg ? n : 0;
      s_wread = -1;
    }
    __syncthreads();
    auto dma_blk = [&](int b) {  // 16 DMA instructions, always
      const int half = lane >> 5, p2 = 2 * (lane & 31);
      const bool real = b < nblk;
#pragma unroll
      for (int i = 0; i < B / 2; ++i) {
        const int cc0 = s0 + b * B + 2 * i;
        const int cc = cc0 + half;
        const double* src = band + (int64_t)min(cc, n - 1) * LDB + p2;
        const uint32_t dst = real ? ring_lds + (uint32_t)((cc0 % W) * LDB * 8) : junk_lds;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)dst, 16, 0, 16);
      }
    };
    auto store_blk = [&](int b) {  // 16 store instructions, always
      const bool real = b >= 0 && b < nblk;
      // lane l holds 16 B of every two columns: column cb + 2u + l / 32, doubles 2 (l % 32) + {0, 1}
      const int cb = s0 + b * B;
      double2v tmp[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int cc = cb + 2 * u + (lane >> 5);
        tmp[u] = real ? *reinterpret_cast<const double2v*>(ring + ri(cc, 2 * (lane & 31))) : (double2v){0.0, 0.0};
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the ring reads are done ...
      if (lane == 0) __hip_atomic_store(&s_wread, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int cc = cb + 2 * u + (lane >> 5);
        const auto v = __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b128(rb, 0, 0, 0)), tmp[u]);
        if (real)
          __builtin_amdgcn_raw_buffer_store_b128(v, rb, cc < n ? (cc * LDB + 2 * (lane & 31)) * 8 : nbytes, 0, 16u);
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, rsc, (lane + 64 * u) * 16, 0, 0u);
      }
    };
    auto lds_wait = [&](int* word, int need) {
      int spin = 0;
      while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need && ++spin < SPIN_LIMIT)
        __builtin_amdgcn_s_sleep(1);
    };
    auto poll_until = [&](int need) {  // poller
      need = min(need, n);
      if (lane == 0 && q > qbeg) {
        int got = __hip_atomic_load(&s_avail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP), spin = 0;
        while (got < need) {
          got = (int)ld_f(gprog + q - 1);
          if (got >= need) break;
          if (++spin > SPIN_LIMIT || ld_f(abortw) != 0) {
            st_f(abortw, 1u);
            got = n;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(&s_avail, got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    };
    // ---- prologue: blocks 0 .. 2 requested, 0 and 1 landed --------------------------------
    if (wave == POLLER) poll_until(blk_end(2));
    __syncthreads();
    if (wave == LOADER) {
#pragma unroll
      for (int b = 0; b < 3; ++b) dma_blk(b);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // blocks 0, 1 landed; 2 may fly
    }
    __syncthreads();
    int prev = -1;  // block stored one step ago (writer)
    int64_t* tq = (wtr && q >= wq0 && q < wq0 + 4) ? wtr + (int64_t)(q - wq0) * 512 * 12 : nullptr;
    for (int tau = 0; tau < tend; ++tau) {
      int64_t* tr = (tq && tau < 512 && lane == 0) ? tq + tau * 12 : nullptr;
      if (wave == LOADER) {
        // block tau+3 into the slots of block tau-5 once the writer has read them; block
        // tau+2 (first touched at step tau+1) must land within this step: tau+3 may fly
        if (tr) tr[0] = (int64_t)__builtin_amdgcn_s_memrealtime();
        lds_wait(&s_avail, blk_end(tau + 3));
        if (tr) tr[1] = (int64_t)__builtin_amdgcn_s_memrealtime();
        if (tau >= 5) lds_wait(&s_wread, tau - 5);
        if (tr) tr[2] = (int64_t)__builtin_amdgcn_s_memrealtime();
        dma_blk(tau + 3);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        if (tr) tr[3] = (int64_t)__builtin_amdgcn_s_memrealtime();
      } else if (wave == WRITER) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the block stored one step ago
        if (tr) tr[4] = (int64_t)__builtin_amdgcn_s_memrealtime();
        if (lane == 0 && prev >= 0 && prev < nblk) st_f(gprog + q, (uint32_t)blk_end(prev));
        prev = tau - 5;
        store_blk(tau - 5);  // final after step tau-1; a scratch block while tau < 5
      } else if (wave == POLLER) {
        poll_until(blk_end(tau + 4));
      } else if (wave < gq) {
        const int s = s0 + wave, k = tau - 3 * wave;
        if (k >= 0 && k < ntask(s)) {
          const int r0 = s + 1 + k * B;
          const int r1 = min(r0 + B, n), len = r1 - r0;
          const int col = k == 0 ? s : r0 - B;
          const int nl = r0 - col;
          const int r2 = min(r1 + B, n), nr = r2 - r1;
          int64_t* tw = (wave == 0) ? tr : nullptr;
          if (tw) tw[6] = (int64_t)__builtin_amdgcn_s_memrealtime();
          double* wvec = wv_all + wave * 2 * B + B;
          // Ring addresses: element (row, cc) at slot(cc) * LDB + row - cc.  L and the lower half
          // of D are read down one column per lane (immediate offsets); the upper half of D and R
          // down one row per lane, whose slot steps by one per element and may wrap once.
          const int ih = H * h;
          const int bL = ((col + c) % W) * LDB + r0 + ih - col - c;
          const int bD = ((r0 + c) % W) * LDB + ih - c;
          const int u0 = (r0 + ih) % W;
          const int bU = u0 * LDB + c - ih, thr = W - u0;
          // branch-free selects (sign masks): a select the compiler turns into control flow
          // keeps 16 exec masks live across the phase
          auto pick = [](int m, int a, int b) -> int { return b + ((a - b) & m); };  // m ? a : b
          auto iu = [&](int qq) -> int { return bU + (LDB - 1) * qq - (W * LDB & ((thr - 1 - qq) >> 31)); };
          const int limL = c < nl ? len - ih : 0;   // qq < limL: a live element of L
          const int limI = len - ih;                // qq < limI: row i inside the block
          const int limD = c < len ? limI : 0;
          const int limR = c < nr ? limI : 0;
          // ih - c, opaque: otherwise the 16 lane-constant masks (ih + qq >= c) are hoisted
          // out of the whole kernel loop and spilled
          int dh = ih - c;
          asm volatile("" : "+v"(dh));
          // ---- every read of the task up front: its L, D and R regions are disjoint ---------
          // (the reflector column col is read by every lane: v is formed where it is used)
          const int b0 = (col % W) * LDB + r0 - col;  // column col, row r0
          // a full task (k > 0, no tail) stores every element it holds; the others send the
          // elements outside their block to the junk slot
          const bool full = k > 0 && len == B && nr == B;
          double L[H], V[H], Dd[H], R[H];
          int ad[H];  // D: column c below the diagonal, row c above it (the mirror element)
#pragma unroll
          for (int qq = 0; qq < H; ++qq) {
            ad[qq] = pick((dh + qq) >> 31, iu(qq), bD + qq);
            L[qq] = ring[bL + qq];
            V[qq] = ring[b0 + ih + qq];
            Dd[qq] = ring[ad[qq]];
            R[qq] = ring[iu(qq) + len];
          }
          const double x0 = ring[b0];
          const double xc = ring[b0 + c];
          if (tw) tw[7] = (int64_t)__builtin_amdgcn_s_memrealtime();
          // ---- the reflector ------------------------------------------------------------------
          double sq0 = 0.0, sq1 = 0.0;
#pragma unroll
          for (int qq = 0; qq < H; qq += 2) {
            if (ih + qq >= 1 && qq < limI) sq0 = fma(V[qq], V[qq], sq0);
            if (qq + 1 < limI) sq1 = fma(V[qq + 1], V[qq + 1], sq1);
          }
          double sq = sq0 + sq1;
          sq += lane_xor32(sq);
          double beta = x0, tau_h = 0.0, scal = 0.0;
          if (sq != 0.0) {
            beta = -copysign(sqrt(fma(x0, x0, sq)), x0);
            tau_h = (beta - x0) / beta;
            scal = 1.0 / (x0 - beta);
          }
          double v[H];
#pragma unroll
          for (int qq = 0; qq < H; ++qq) v[qq] = qq < limI ? (ih + qq == 0 ? 1.0 : V[qq] * scal) : 0.0;
          const double vc = c < len ? (c == 0 ? 1.0 : xc * scal) : 0.0;
          if (tw) tw[8] = (int64_t)__builtin_amdgcn_s_memrealtime();
          // ---- left block: the reflector applied to rows R_k of columns col .. r0-1 -----------
          {
            double d = dot16(v, L);
            d += lane_xor32(d);
            const double f = tau_h * d;
#pragma unroll
            for (int qq = 0; qq < H; ++qq) L[qq] = c == 0 ? (ih + qq == 0 ? beta : 0.0) : fma(-f, v[qq], L[qq]);
            if (full) {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[bL + qq] = L[qq];
            } else {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[pick((qq - limL) >> 31, bL + qq, jk)] = L[qq];
            }
          }
          if (tw) tw[9] = (int64_t)__builtin_amdgcn_s_memrealtime();
          // ---- right: the rows below (the new bulge) ----------------------------------------
          {
            double d = dot16(R, v);
            d += lane_xor32(d);
            const double f = tau_h * d;
#pragma unroll
            for (int qq = 0; qq < H; ++qq) R[qq] = fma(-f, v[qq], R[qq]);
            if (full) {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[iu(qq) + len] = R[qq];
            } else {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[pick((qq - limR) >> 31, iu(qq) + len, jk)] = R[qq];
            }
          }
          // ---- both sides on the diagonal block ---------------------------------------------
          {
            double pc = dot16(Dd, v);
            pc += lane_xor32(pc);
            pc *= tau_h;
            double pv = h == 0 ? pc * vc : 0.0;
            pv = lane_sum32(pv);
            pv += lane_xor32(pv);
            const double wc = fma(-0.5 * tau_h * pv, vc, pc);
            if (h == 0) wvec[c] = c < len ? wc : 0.0;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (tw) tw[10] = (int64_t)__builtin_amdgcn_s_memrealtime();
            // D - (v w' + w v'), symmetric in (i, c) bit for bit: the lane holding the mirror
            // element computes and stores the same value to the same address
#pragma unroll
            for (int qq = 0; qq < H; ++qq) {
              const double wi = wvec[ih + qq];
              Dd[qq] = Dd[qq] - (v[qq] * wc + wi * vc);
            }
            if (full) {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[ad[qq]] = Dd[qq];
            } else {
#pragma unroll
              for (int qq = 0; qq < H; ++qq) ring[pick((qq - limD) >> 31, ad[qq], jk)] = Dd[qq];
            }
          }
        }
        if (wave == 0 && tr) tr[5] = (int64_t)__builtin_amdgcn_s_memrealtime();
      }
      __syncthreads();  // step tau done; block tau+2 (first touched at step tau+1) landed
    }
    // ---- epilogue: the blocks not yet written back, then the group is done ----------------
    if (wave == LOADER) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave == WRITER) {
      for (int b = max(0, tend - 5); b < nblk; ++b) store_blk(b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) st_f(gprog + q, (uint32_t)n);
    }
    __syncthreads();  // the ring is reused by the next group of this workgroup
  }
}

// D, E of the reduced band (band[c*LDB + 0], band[c*LDB + 1]).
template <int B>
__global__ void k_tri_out(const double* __restrict__ band, int n, double* __restrict__ D, double* __restrict__ E) {
  constexpr int LDB = 2 * B;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  D[c] = ld_c(band + (int64_t)c * LDB);
  if (c < n - 1) E[c] = ld_c(band + (int64_t)c * LDB + 1);
}

// ---------------------------------------------------------------------------------------
// Inverse iteration on the band matrix Bm (the stage-1 band, lower bandwidth B, in `band`
// before stage 2 ran -- a separate copy) for lam_desc[k], one workgroup per eigenvalue.
// LU with partial pivoting of Bm - lam I (dgbtrf: kl = B, ku = 2B after the row swaps),
// kept as U rows (n x (2B+1)) and L multipliers (n x B) + pivots in the workspace; the
// active (B+1) x (2B+1) window lives in LDS.  Two solves from a fixed start vector
// (dstein's), normalised.
// ---------------------------------------------------------------------------------------
template <int B>
__global__ __launch_bounds__(256) void k_band_invit(const double* __restrict__ bnd, int n,
                                                    const double* __restrict__ lam_desc,
                                                    double* __restrict__ work, int* __restrict__ ipiv_all,
                                                    double* __restrict__ Y, int ldy) {
  static_assert(2 * B <= 64, "the backward solve keeps 2B values in one wave");
  constexpr int LDB = 2 * B, KU = 2 * B, WC = KU + 1, WR = B + 1;
  // circular window: matrix row j+r in row slot (j+r) % WR, column j+c in slot (j+c) % WC
  __shared__ double win[WR][WC + 1];
  __shared__ double lmul[WR];
  __shared__ int piv_i;
  __shared__ double red[8];
  const int k = blockIdx.x, t = threadIdx.x;
  const double lam = lam_desc[k];
  double* U = work + (int64_t)k * n * (WC + B + 1);  // n x WC, then L (n x B), then x (n)
  double* Lm = U + (int64_t)n * WC;
  double* x = Lm + (int64_t)n * B;
  int* ipiv = ipiv_all + (int64_t)k * n;
  auto bval = [&](int i, int j) -> double {  // (Bm - lam I)[i][j]
    if (i < 0 || j < 0 || i >= n || j >= n) return 0.0;
    const int d = i - j;
    if (d > B || d < -B) return 0.0;
    const double v = d >= 0 ? bnd[(int64_t)j * LDB + d] : bnd[(int64_t)i * LDB - d];
    return i == j ? v - lam : v;
  };
  double nrm = 0.0;
  for (int e = t; e < n; e += 256) nrm = fmax(nrm, fabs(bnd[(int64_t)e * LDB]) + 2.0 * fabs(bnd[(int64_t)e * LDB + 1]));
  for (int o = 32; o >= 1; o >>= 1) nrm = fmax(nrm, __shfl_xor(nrm, o));
  if ((t & 63) == 0) red[t >> 6] = nrm;
  __syncthreads();
  nrm = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double floor_ = 2.220446049250313e-16 * fmax(nrm, 1e-300);
  for (int e = t; e < WR * WC; e += 256) {
    const int r = e / WC, c = e % WC;
    win[r][c] = bval(r, c);
  }
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    const int nrow = min(B, n - 1 - j);
    const int sj = j % WR, cj = j % WC;
    // the row entering at the end of this step (independent of the elimination): load now
    const double nrv = t < WC ? bval(j + 1 + B, j + 1 + t) : 0.0;
    if (t < 64) {
      double best = -1.0;
      int bi = 0;
      if (t <= nrow) {
        best = fabs(win[(j + t) % WR][cj]);
        bi = t;
      }
      for (int o = 32; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      if (t == 0) piv_i = bi;
    }
    __syncthreads();
    const int pr = piv_i;
    const int sp = (j + pr) % WR;
    if (pr != 0 && t < WC) {
      const double a = win[sj][t];
      win[sj][t] = win[sp][t];
      win[sp][t] = a;
    }
    __syncthreads();
    double d0 = win[sj][cj];
    if (fabs(d0) < floor_) d0 = d0 < 0.0 ? -floor_ : floor_;
    if (t >= 1 && t <= nrow) lmul[t] = win[(j + t) % WR][cj] / d0;
    if (t < WC) U[(int64_t)j * WC + t] = t == 0 ? d0 : win[sj][(j + t) % WC];
    if (t == 0) ipiv[j] = j + pr;
    __syncthreads();
    if (t < B) Lm[(int64_t)j * B + t] = (t + 1 <= nrow) ? lmul[t + 1] : 0.0;
    for (int e = t; e < nrow * KU; e += 256) {
      const int r = 1 + e / KU, c = 1 + e % KU;
      const int sr = (j + r) % WR, sc = (j + c) % WC;
      win[sr][sc] = fma(-lmul[r], win[sj][sc], win[sr][sc]);
    }
    __syncthreads();
    // row j leaves: its slot takes matrix row j+1+B; column slot cj becomes column j+1+2B
    if (t < WC) win[sj][(j + 1 + t) % WC] = nrv;
    if (t >= 1 && t <= B) win[(j + t) % WR][cj] = 0.0;
    __syncthreads();
  }
  // ---- two solves from a pseudo-random start (dlarnv-like), one wave, register windows ---
  // The start depends on k as well: members of an exactly degenerate cluster (a zero block,
  // I + u u^T) then reach different vectors of the eigenspace, which k_orth orthonormalises
  // (one start for all k gave identical vectors there, and the cluster collapsed).
  for (int e = t; e < n; e += 256) {
    uint32_t hh = (uint32_t)e * 2654435761u ^ (0x9e3779b9u + (uint32_t)k * 0x85ebca6bu);
    hh ^= hh >> 15; hh *= 2246822519u; hh ^= hh >> 13; hh *= 3266489917u; hh ^= hh >> 16;
    x[e] = (double)hh * (2.0 / 4294967296.0) - 1.0;
  }
  __syncthreads();
  for (int it = 0; it < 2; ++it) {
    if (t < 64) {
      const int lane = t;
      // The loads of both solves do not depend on the recurrence: they run PD rows ahead
      // in registers (a load inside the chain cost one memory round trip per row).
      constexpr int PD = 8;
      // forward: lanes 0..B hold x[j..j+B] (lane 0 = x[j])
      double wv = lane <= B && lane < n ? x[lane] : 0.0;
      {
        double lq[PD], xq[PD];
        int pq[PD];
        auto fetch = [&](int d, int j) {
          const bool in = j < n;
          lq[d] = (in && lane >= 1 && lane <= B) ? Lm[(int64_t)j * B + lane - 1] : 0.0;
          xq[d] = (in && j + 1 + B < n) ? x[j + 1 + B] : 0.0;
          pq[d] = in ? ipiv[j] - j : 0;
        };
#pragma unroll
        for (int d = 0; d < PD; ++d) fetch(d, d);
        for (int j0 = 0; j0 < n; j0 += PD) {
#pragma unroll
          for (int d = 0; d < PD; ++d) {
            const int j = j0 + d;
            if (j < n) {
              const int p = __builtin_amdgcn_readfirstlane(pq[d]);
              const double v0 = lane_read(wv, 0), vp = lane_read(wv, p);
              if (lane == 0) wv = vp;
              if (lane == p) wv = v0;
              const double xj = lane_read(wv, 0);
              if (lane >= 1 && lane <= B) wv = fma(-lq[d], xj, wv);
              if (lane == 0) x[j] = xj;
              const double nxt = __shfl_down(wv, 1);
              wv = lane < B ? nxt : xq[d];
            }
            fetch(d, j + PD);
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      // backward: lanes 0..2B-1 hold x[j+1..j+2B]
      double wb = 0.0;
      {
        double uq[PD], dq[PD], xq[PD];
        auto fetch = [&](int d, int j) {
          const bool in = j >= 0;
          uq[d] = (in && j + 1 + lane < n) ? U[(int64_t)j * WC + 1 + lane] : 0.0;
          dq[d] = in ? U[(int64_t)j * WC] : 1.0;
          xq[d] = in ? x[j] : 0.0;  // the forward result: row j is rewritten only at step j
        };
#pragma unroll
        for (int d = 0; d < PD; ++d) fetch(d, n - 1 - d);
        for (int j0 = n - 1; j0 >= 0; j0 -= PD) {
#pragma unroll
          for (int d = 0; d < PD; ++d) {
            const int j = j0 - d;
            if (j >= 0) {
              double sdot = uq[d] * wb;
              for (int o = 32; o >= 1; o >>= 1) sdot += __shfl_xor(sdot, o);
              const double xj = (xq[d] - sdot) / dq[d];
              if (lane == 0) x[j] = xj;
              const double up = __shfl_up(wb, 1);
              wb = lane == 0 ? xj : up;
            }
            fetch(d, j - PD);
          }
        }
      }
    }
    __syncthreads();
    double mx = 0.0;
    for (int e = t; e < n; e += 256) mx = fmax(mx, fabs(x[e]));
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    double ss = 0.0;
    for (int e = t; e < n; e += 256) {
      const double v = x[e] / mx;
      ss = fma(v, v, ss);
    }
    for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
    if ((t & 63) == 0) red[4 + (t >> 6)] = ss;
    __syncthreads();
    const double nrm2 = sqrt(red[4] + red[5] + red[6] + red[7]);
    for (int e = t; e < n; e += 256) x[e] = x[e] / mx / nrm2;
    __syncthreads();
  }
  for (int e = t; e < n; e += 256) Y[(int64_t)e * ldy + k] = x[e];
}

// Back-transformation Y[r0:] <- Q_p Y[r0:] = Y - Vx (T (Vx^T Y)), panels applied last first.
// k_bt_z: partial Vx^T Y over row chunks -> Zp; k_bt_u: Z = sum, Z2 = T Z, Y -= Vx Z2.
template <int B>
__global__ __launch_bounds__(256) void k_bt_z(const double* __restrict__ Vx, const double* __restrict__ Y, int ldy,
                                              int r0, int m, int nvec, int chunk, double* __restrict__ Zp) {
  // thread (a = column of V, g = row group of 256/B): partial sums over rows r = g (mod 256/B)
  // of V[r][a] * Y[r][c] for every c (nvec <= 64 accumulators), then an LDS reduction
  constexpr int RG = 256 / B;
  __shared__ double red[RG][B][65];
  const int t = threadIdx.x, a = t % B, g = t / B;
  const int a0 = blockIdx.x * chunk, a1 = min(m, a0 + chunk);
  double acc[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) acc[c] = 0.0;
  for (int r = a0 + g; r < a1; r += RG) {
    const double v = Vx[(int64_t)r * B + a];
    const double* yr = Y + (int64_t)(r0 + r) * ldy;
#pragma unroll
    for (int c = 0; c < 64; ++c)
      if (c < nvec) acc[c] = fma(v, yr[c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < 64; ++c)
    if (c < nvec) red[g][a][c] = acc[c];
  __syncthreads();
  for (int e = t; e < B * nvec; e += 256) {
    const int aa = e / nvec, c = e % nvec;
    double s2 = 0.0;
    for (int q = 0; q < RG; ++q) s2 += red[q][aa][c];
    Zp[(int64_t)blockIdx.x * B * nvec + e] = s2;
  }
}

template <int B>
__global__ __launch_bounds__(256) void k_bt_t(const double* __restrict__ T, const double* __restrict__ Zp, int nz,
                                              int nvec, double* __restrict__ Z2) {
  extern __shared__ double shz[];
  double* Z = shz;  // B x nvec
  const int t = threadIdx.x;
  for (int e = t; e < B * nvec; e += 256) {
    double s = 0.0;
    s = sum_partials(Zp + e, (int64_t)B * nvec, nz);
    Z[e] = s;
  }
  __syncthreads();
  for (int e = t; e < B * nvec; e += 256) {
    const int a = e / nvec, c = e % nvec;
    double s = 0.0;
    for (int l = a; l < B; ++l) s = fma(T[a * B + l], Z[l * nvec + c], s);  // T upper
    Z2[e] = s;
  }
}

template <int B>
__global__ __launch_bounds__(256) void k_bt_u(const double* __restrict__ Vx, const double* __restrict__ Z2g,
                                              double* __restrict__ Y, int ldy, int r0, int m, int nvec) {
  extern __shared__ double shz[];
  double* Z2 = shz;  // B x nvec
  const int t = threadIdx.x;
  for (int e = t; e < B * nvec; e += 256) Z2[e] = Z2g[e];
  __syncthreads();
  const int64_t tot = (int64_t)m * nvec;
  for (int64_t e = (int64_t)blockIdx.x * 256 + t; e < tot; e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / nvec), c = (int)(e % nvec);
    double s = Y[(int64_t)(r0 + r) * ldy + c];
    for (int l = 0; l < B; ++l) s = fma(-Vx[(int64_t)r * B + l], Z2[l * nvec + c], s);
    Y[(int64_t)(r0 + r) * ldy + c] = s;
  }
}

}  // namespace sb

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
int sy2sb_band() { return 32; }
int syev2_max_n() { return 16384; }

size_t sy2sb_work_doubles(int n, int nvec, SyevdPlan* plan) {
  constexpr int B = 32;
  SyevdPlan p{};
  p.B = B;
  p.np = 0;
  int64_t vx = 0;
  for (int c0 = 0; c0 < n - B - 1; c0 += B) {
    vx += (int64_t)(n - c0 - B) * B;
    ++p.np;
  }
  p.KS = 16;   // k_ay2 K splits (at most; fewer for short trailing blocks)
  p.NZ = 128;  // row chunks of the V^T X / V^T Y partial products
  p.RP = 256;
  const int64_t nn = (int64_t)n * n;
  p.off_aw = 0;
  p.off_vx = p.off_aw + nn;
  p.off_t = p.off_vx + vx;
  p.off_tau = p.off_t + (int64_t)std::max(p.np, 1) * B * B;
  p.off_y = p.off_tau + (int64_t)std::max(p.np, 1) * B;
  p.off_x = p.off_y + (int64_t)p.KS * n * B;
  p.off_w = p.off_x + (int64_t)n * B;
  p.off_zp = p.off_w + (int64_t)n * B;
  p.off_m = p.off_zp + (int64_t)std::max<int64_t>(p.NZ * B * B, (int64_t)p.NZ * B * std::max(nvec, 1));
  p.off_pub = p.off_m + (int64_t)B * std::max(B, nvec);
  p.off_band = p.off_pub + 2LL * 64 * 2 * B;
  p.off_band0 = p.off_band + (int64_t)n * 2 * B;
  p.off_de = p.off_band0 + (int64_t)n * 2 * B;
  p.off_deg = p.off_de + 4LL * n + 8;
  p.off_inv = p.off_deg + 2LL * n + 2;
  p.off_end = p.off_inv + (int64_t)std::max(nvec, 1) * ((int64_t)n * (2 * B + 1 + B) + n);
  p.off_end += 256LL * B * 2 * B;  // k_sbtrd_win's per-workgroup scratch block (the last 4 MB)
  if (plan) *plan = p;
  return (size_t)p.off_end;
}

// ---- launch_syevd2 in stages, so a caller can spread one eigenvalues-only solve over several
// calls (pods_eigvals_* for n > 4096): begin, panel ranges of stage 1, the band, sweep-group
// ranges of the bulge chase, the eigenvalues.  launch_syevd2 runs them back to back.
hipError_t syevd2_begin(const double* C, int n, double* ws, const SyevdPlan& p, uint32_t* flags, hipStream_t st) {
  constexpr int B = 32;
  hipError_t e = hipMemcpyAsync(ws + p.off_aw, C, (size_t)n * n * sizeof(double), hipMemcpyDeviceToDevice, st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(flags + 128, 0, (size_t)n * sizeof(uint32_t), st);  // the chase's sweep counters
  if (e != hipSuccess) return e;
  // k_pqr's tagged hand-off slots start from tag 0 (the first column's tag is 1)
  return hipMemsetAsync(ws + p.off_pub, 0, (size_t)2 * 64 * 2 * B * sizeof(double), st);
}

// stage 1, panels [pi0, pi1) (panel pi reduces columns 32 pi .. 32 pi + 31 to the band)
hipError_t syevd2_panels(int n, double* ws, const SyevdPlan& p, uint32_t* flags, uint32_t epoch, int pi0, int pi1,
                         hipStream_t st) {
  constexpr int B = 32;
  double* Aw = ws + p.off_aw;
  uint32_t* pflags = flags;        // 64 panel-QR flags
  uint32_t* abortw = flags + 64;   // [0] panel QR, [1] stage 2
  hipError_t e = hipSuccess;
  int64_t vxo = 0;
  for (int r = 0; r < pi0; ++r) vxo += (int64_t)(n - r * B - B) * B;
  pi1 = std::min(pi1, p.np);
  for (int pi = pi0; pi < pi1; ++pi) {
    const int c0 = pi * B;
    const int r0 = c0 + B, m = n - r0;
    double* Vx = ws + p.off_vx + vxo;
    double* T = ws + p.off_t + (int64_t)pi * B * B;
    double* tau = ws + p.off_tau + (int64_t)pi * B;
    const int NW = std::max(1, std::min(64, (m + p.RP - 1) / p.RP));
    const int RP = (m + NW - 1) / NW;
    // PODS_PQR_TRACE=pi: per-column phase stamps of workgroup 0 in panel pi (diagnostics, stderr)
    const char* pqt = std::getenv("PODS_PQR_TRACE");
    int64_t* ptrace = nullptr;
    if (pqt && std::atoi(pqt) == pi) {
      e = hipMallocAsync(reinterpret_cast<void**>(&ptrace), (B * 8 + 1) * sizeof(int64_t), st);
      if (e == hipSuccess) e = hipMemsetAsync(ptrace, 0, (B * 8 + 1) * sizeof(int64_t), st);
      if (e != hipSuccess) return e;
    }
    e = check_persistent(reinterpret_cast<const void*>(&sb::k_pqr<B>), 256, 0, NW, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sb::k_pqr<B>, dim3(NW), dim3(256), 0, st, Aw, (int64_t)n, r0, c0, m, RP, NW,
                       ws + p.off_pub, pflags, epoch * 1024u + (uint32_t)pi, 16u * (uint32_t)pi + 1u, abortw, Vx,
                       tau, ws + p.off_zp, T, ptrace);
    if (ptrace) {
      int64_t h[B * 8 + 1];
      e = hipMemcpyAsync(h, ptrace, sizeof(h), hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      (void)hipFreeAsync(ptrace, st);
      if (e != hipSuccess) return e;
      double a[7] = {0, 0, 0, 0, 0, 0, 0};
      for (int j = 0; j < B; ++j) {
        const int64_t* R = h + j * 8;
        const int64_t nx = j + 1 < B ? h[(j + 1) * 8] : h[B * 8];
        for (int q = 0; q < 6; ++q) a[q] += (R[q + 1] - R[q]) * 0.01;
        a[6] += (nx - R[6]) * 0.01;
      }
      std::fprintf(stderr,
                   "k_pqr panel %d (m = %d, NW = %d, RP = %d) per column us: shfl+dot %.2f B1 %.2f publish %.2f "
                   "hop %.2f B2+sum+B3 %.2f reflector+update %.2f B4 %.2f; total %.2f\n",
                   pi, m, NW, RP, a[0] / B, a[1] / B, a[2] / B, a[3] / B, a[4] / B, a[5] / B, a[6] / B,
                   (h[B * 8] - h[0]) * 0.01 / B);
    }
    // ~4 workgroups per CU for the A22 read: K splits of >= 256 columns
    const int ks = std::max(1, std::min(p.KS, (1024 + (m + 63) / 64 - 1) / ((m + 63) / 64)));
    const int kchunk = ((m + ks - 1) / ks + 31) / 32 * 32;
    const int ksn = (m + kchunk - 1) / kchunk;
    hipLaunchKernelGGL(sb::k_ay2<B>, dim3((m + 63) / 64, ksn), dim3(256), 0, st, Aw, (int64_t)n, r0, m, Vx,
                       kchunk, ws + p.off_y);
    hipLaunchKernelGGL(sb::k_xt<B>, dim3((m + 256 / B - 1) / (256 / B)), dim3(256), 0, st, ws + p.off_y, ksn, m,
                       T, ws + p.off_x);
    const int nzc = std::max(1, std::min(p.NZ, (m + 63) / 64));
    const int zchunk = (m + nzc - 1) / nzc;
    const int nzn = (m + zchunk - 1) / zchunk;
    hipLaunchKernelGGL(sb::k_z<B>, dim3(nzn), dim3(256), 0, st, Vx, ws + p.off_x, m, zchunk, ws + p.off_zp);
    hipLaunchKernelGGL(sb::k_zm<B>, dim3(1), dim3(256), 0, st, ws + p.off_zp, nzn, T, ws + p.off_m);
    hipLaunchKernelGGL(sb::k_w<B>, dim3((m + 256 / B - 1) / (256 / B)), dim3(256), 0, st, ws + p.off_x, Vx,
                       ws + p.off_m, m, ws + p.off_w);
    const int tiles = (m + 63) / 64;
    hipLaunchKernelGGL(sb::k_upd<B>, dim3(tiles * (tiles + 1) / 2), dim3(256), 0, st, Aw, (int64_t)n, r0, m, Vx,
                       ws + p.off_w);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    vxo += (int64_t)m * B;
  }
  return hipSuccess;
}

hipError_t syevd2_band(int n, double* ws, const SyevdPlan& p, bool keep_band0, hipStream_t st) {
  constexpr int B = 32;
  double* band = ws + p.off_band;
  const int64_t nb = (int64_t)n * 2 * B;
  hipLaunchKernelGGL(sb::k_band<B>, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, ws + p.off_aw, (int64_t)n, n,
                     band);
  if (!keep_band0) return hipGetLastError();
  return hipMemcpyAsync(ws + p.off_band0, band, (size_t)nb * sizeof(double), hipMemcpyDeviceToDevice, st);
}

int syevd2_groups(int n) { return n > 2 ? (n - 2 + 1) / 2 : 0; }  // sweep groups of two (GW = 2)

// stage 2, sweep groups [q0, q1): one persistent launch; every group before q0 is done
hipError_t syevd2_chase(int n, double* ws, const SyevdPlan& p, uint32_t* flags, int q0, int q1, hipStream_t st) {
  constexpr int B = 32;
  constexpr int GW = 2;
  using SW = sb::SbWin<B, GW>;
  q1 = std::min(q1, syevd2_groups(n));
  if (q1 <= q0) return hipSuccess;
  uint32_t* abortw = flags + 64;
  uint32_t* prog = flags + 128;
  const int cus = std::max(1, stream_cus(st));  // a CU-masked stream offers only its CUs
  int P = std::max(1, std::min(q1 - q0, cus));
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&sb::k_sbtrd_win<B, GW>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)SW::lds_bytes);
  if (e != hipSuccess) return e;
  e = check_persistent(reinterpret_cast<const void*>(&sb::k_sbtrd_win<B, GW>), SW::NT, SW::lds_bytes, P, st);
  if (e != hipSuccess) return e;
  // PODS_SBWIN_TRACE=q0: per-step timestamps of groups q0 .. q0+3 (diagnostics, stderr)
  const char* wts = std::getenv("PODS_SBWIN_TRACE");
  int64_t* wtr = nullptr;
  const size_t wtn = 4 * 512 * 12;
  if (wts) {
    e = hipMallocAsync(reinterpret_cast<void**>(&wtr), wtn * sizeof(int64_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(wtr, 0, wtn * sizeof(int64_t), st);
    if (e != hipSuccess) return e;
  }
  const int wq0 = wts ? std::atoi(wts) : 0;
  hipLaunchKernelGGL((sb::k_sbtrd_win<B, GW>), dim3(P), dim3(SW::NT), SW::lds_bytes, st, ws + p.off_band, n, q0, q1,
                     prog, abortw + 1, ws + p.off_end - 256LL * B * 2 * B, wtr, wq0);
  if (wtr) {
    std::vector<int64_t> h(wtn);
    e = hipMemcpyAsync(h.data(), wtr, wtn * sizeof(int64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFreeAsync(wtr, st);
    if (e != hipSuccess) return e;
    for (int g = 0; g < 4; ++g) {
      const int64_t* T = h.data() + (size_t)g * 512 * 12;
      double a[6] = {0, 0, 0, 0, 0, 0};
      int cnt = 0;
      double ph[5] = {0, 0, 0, 0, 0};
      int pc = 0;
      for (int k = 0; k + 1 < 512 && T[(k + 1) * 12] != 0; ++k, ++cnt) {
        const int64_t* R = T + k * 12;
        a[0] += (R[1] - R[0]) * 0.01;           // loader: wait for the previous group
        a[1] += (R[2] - R[1]) * 0.01;           // loader: wait for the writer's read
        a[2] += (R[3] - R[2]) * 0.01;           // loader: DMA issue + landing
        a[3] += (R[4] - R[0]) * 0.01;           // writer: store drain
        a[4] += (R[5] - R[0]) * 0.01;           // task wave 0
        a[5] += (T[(k + 1) * 12] - R[0]) * 0.01;  // step to step
        if (R[6] != 0) {
          ph[0] += (R[6] - R[0]) * 0.01;  // task start
          for (int z = 1; z < 5; ++z) ph[z] += (R[6 + z] - R[5 + z]) * 0.01;
          ++pc;
        }
      }
      pc = std::max(pc, 1);
      std::fprintf(stderr, "sbwin group %d task phases us: start %.2f loads %.2f reflector %.2f left %.2f right+w %.2f\n", wq0 + g,
                   ph[0] / pc, ph[1] / pc, ph[2] / pc, ph[3] / pc, ph[4] / pc);
      const double lag = g > 0 ? (T[0] - h[(size_t)(g - 1) * 512 * 12]) * 0.01 : 0.0;
      cnt = std::max(cnt, 1);
      std::fprintf(stderr,
                   "sbwin group %d: %d steps, start lag %.2f us; per step us: avail %.2f wread %.2f dma %.2f "
                   "drain %.2f task %.2f step %.2f\n",
                   wq0 + g, cnt, lag, a[0] / cnt, a[1] / cnt, a[2] / cnt, a[3] / cnt, a[4] / cnt, a[5] / cnt);
    }
  }
  return hipGetLastError();
}

// all n eigenvalues of the band's tridiagonal (descending)
hipError_t syevd2_eigvals(int n, double* ws, const SyevdPlan& p, int* grid_cnt, double* lam_desc, hipStream_t st) {
  constexpr int B = 32;
  double* D = ws + p.off_de;
  double* E = D + n;
  double* bounds = D + 2 * (int64_t)n;
  hipLaunchKernelGGL(sb::k_tri_out<B>, dim3((n + 255) / 256), dim3(256), 0, st, ws + p.off_band, n, D, E);
  return launch_tri_eigvals(D, E, n, bounds, lam_desc, grid_cnt, st, reinterpret_cast<double2*>(ws + p.off_deg));
}

hipError_t launch_syevd2(const double* C, int n, int nvec, double* ws, const SyevdPlan& p, uint32_t* flags,
                         uint32_t epoch, int* ipiv, int* grid_cnt, double* lam_desc, double* vec, hipStream_t st) {
  constexpr int B = 32;
  hipError_t e = syevd2_begin(C, n, ws, p, flags, st);
  if (e == hipSuccess) e = syevd2_panels(n, ws, p, flags, epoch, 0, p.np, st);
  if (e == hipSuccess) e = syevd2_band(n, ws, p, nvec > 0, st);
  if (e == hipSuccess) e = syevd2_chase(n, ws, p, flags, 0, syevd2_groups(n), st);
  if (e == hipSuccess) e = syevd2_eigvals(n, ws, p, grid_cnt, lam_desc, st);
  if (e != hipSuccess || nvec <= 0) return e;
  double* band0 = ws + p.off_band0;
  double* bounds = ws + p.off_de + 2 * (int64_t)n;
  double* inv = ws + p.off_inv;
  hipLaunchKernelGGL(sb::k_band_invit<B>, dim3(nvec), dim3(256), 0, st, band0, n, lam_desc, inv, ipiv, vec, nvec);
  e = launch_orth(lam_desc, bounds, n, nvec, vec, nvec, st);
  if (e != hipSuccess) return e;
  // Y <- Q_0 Q_1 ... Q_{np-1} Y
  for (int q = p.np - 1; q >= 0; --q) {
    int64_t off = 0;
    for (int r = 0; r < q; ++r) off += (int64_t)(n - r * B - B) * B;
    const int r0 = q * B + B, m = n - r0;
    const double* Vx = ws + p.off_vx + off;
    const double* T = ws + p.off_t + (int64_t)q * B * B;
    const int nz0 = std::min(p.NZ, std::max(1, m / 64));
    const int chunk = (m + nz0 - 1) / nz0;
    const int nz = (m + chunk - 1) / chunk;
    hipLaunchKernelGGL(sb::k_bt_z<B>, dim3(nz), dim3(256), 0, st, Vx, vec, nvec, r0, m, nvec, chunk, ws + p.off_zp);
    const size_t lds = (size_t)B * nvec * sizeof(double);
    hipLaunchKernelGGL(sb::k_bt_t<B>, dim3(1), dim3(256), lds, st, T, ws + p.off_zp, nz, nvec, ws + p.off_m);
    const int gu = std::max(1, std::min(512, (int)(((int64_t)m * nvec + 255) / 256)));
    hipLaunchKernelGGL(sb::k_bt_u<B>, dim3(gu), dim3(256), lds, st, Vx, ws + p.off_m, vec, nvec, r0, m, nvec);
  }
  return hipGetLastError();
}

}  // namespace pods

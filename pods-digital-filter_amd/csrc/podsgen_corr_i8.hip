// The POD correlation C = A^T A (PODFS.py:1455, `np.dot(A.T, A)` after main() :1492-1495's
// centring) as EXACT integer arithmetic on the int8 matrix cores (v_mfma_i32_16x16x64_i8),
// reconstructed by the Chinese remainder theorem (Ozaki scheme II, integer-modular form).
//
//   1. scale: one power of two 2^s for the whole matrix from max |a - mean| (k_mean folds that
//      maximum into its pass; k_absdev when the mean came from the host), chosen so every
//      scaled element rounds to an integer a' with |a'| <= 2^b; b = 52 at C3 / C4, 51 at C5,
//      so no element loses more than 2^-(b+1) of max |a - mean| (fp64 keeps 2^-53 of |a|);
//   2. k_residues: a' mod m_l for NMOD = 16 pairwise-coprime odd moduli m_l <= 255, as balanced
//      int8 (|r| <= 127), K-tiled [K/64][ns][64] per modulus;
//   3. k_syrk_i8: for every modulus, the int8 SYRK of the residues on 256 x 256 lower tiles,
//      int32 accumulators (exact: every 2048 K-steps they are reduced mod m before they could
//      overflow), written as one byte mod m_l per element (split-K partials summed mod m_l);
//   4. k_crt: per element, Garner's mixed-radix digits of the 16 residues and the exact
//      128-bit integer C' = sum a'_i a'_j (|C'| <= K 2^2b < M/2, M = prod m_l ~ 2^124.7),
//      converted to double once and scaled by 2^-2s (and / ns).
// The products are exact, so the only rounding is the scaling of the inputs (step 1) and the
// final conversion; against the fp64 SYRK (k_syrk_g128) the results differ by ~1e-15 of
// max |C| (tests/test_gpu_corr_i8.py).  The fp64 MFMA SYRK stays selectable
// (pods_set_corr_mode / PODS_CORR=f64).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "podsgen_kernels.h"

namespace pods {
namespace i8 {

constexpr int NMOD = 16;

struct ModTables {
  int m[NMOD];
  int p18[NMOD], p36[NMOD];  // 2^18, 2^36 mod m
  int off[NMOD];             // -(2^52) mod m
  int p11[NMOD][5];          // 2^(11 k) mod m
  int p14[NMOD][4];          // 2^(14 k) mod m, balanced to [-(m-1)/2, (m-1)/2]
  int inv[NMOD][NMOD];       // inv[k][l] = m_k^-1 mod m_l (k != l)
};
constexpr int pow2mod(int e, int m) {
  int r = 1 % m;
  for (int i = 0; i < e; ++i) r = (r * 2) % m;
  return r;
}
constexpr int invmod(int a, int m) {
  a %= m;
  for (int x = 1; x < m; ++x)
    if ((a * x) % m == 1) return x;
  return 0;
}
constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }
constexpr ModTables make_tables() {
  ModTables t{};
  const int mm[NMOD] = {255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 211, 199, 197, 193, 191, 181};
  for (int l = 0; l < NMOD; ++l) {
    t.m[l] = mm[l];
    t.p18[l] = pow2mod(18, mm[l]);
    t.p36[l] = pow2mod(36, mm[l]);
    t.off[l] = (mm[l] - pow2mod(52, mm[l])) % mm[l];
    for (int k = 0; k < 5; ++k) t.p11[l][k] = pow2mod(11 * k, mm[l]);
    for (int k = 0; k < 4; ++k) {
      const int c = pow2mod(14 * k, mm[l]);
      t.p14[l][k] = c > mm[l] / 2 ? c - mm[l] : c;
    }
  }
  for (int l = 0; l < NMOD; ++l)
    for (int k = 0; k < NMOD; ++k) t.inv[k][l] = k == l ? 0 : invmod(mm[k], mm[l]);
  return t;
}
constexpr ModTables kT = make_tables();
constexpr bool coprime_all() {
  for (int a = 0; a < NMOD; ++a)
    for (int b = a + 1; b < NMOD; ++b)
      if (gcd_c(kT.m[a], kT.m[b]) != 1) return false;
  return true;
}
static_assert(coprime_all(), "moduli must be pairwise coprime");
constexpr unsigned __int128 prod_m() {
  unsigned __int128 p = 1;
  for (int l = 0; l < NMOD; ++l) p *= (unsigned)kT.m[l];
  return p;
}
constexpr unsigned __int128 kM = prod_m();
constexpr double kLog2M = 124.689;  // log2(prod m_l), rounded down
static_assert((kM >> 124) == 1, "prod m_l in [2^124, 2^125)");

// a runtime modulus (the SYRK's workgroup-uniform one)
__device__ __forceinline__ int modulus(int l) {
  int r = 0;
#pragma unroll
  for (int k = 0; k < NMOD; ++k)
    if (k == l) r = kT.m[k];
  return r;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// the scale exponent s: max |a - mean| * 2^s < 2^b
__device__ __forceinline__ int scale_exp(double dev, int bbits) {
  return dev > 0.0 ? bbits - 1 - ilogb(dev) : 0;
}

// ---- max |fl(a - mean)| when the mean did not come from k_mean ----------------------------
__global__ __launch_bounds__(256) void k_absdev(const double* __restrict__ AT, int ns, int64_t rowlen,
                                                int64_t rowpad, const double* __restrict__ mean,
                                                unsigned long long* __restrict__ devmax) {
  const int64_t n = rowpad * (int64_t)ns;
  double mx = 0.0;
  for (int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x; f < n; f += (int64_t)gridDim.x * 256) {
    const int64_t r = (f / ((int64_t)ns << 4)) * 16 + (f & 15);
    if (r < rowlen) mx = fmax(mx, fabs(AT[f] - mean[r]));
  }
  unsigned long long u = (unsigned long long)__double_as_longlong(mx > 0.0 ? mx : 0.0);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long v = __shfl_xor(u, o);
    u = v > u ? v : u;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(devmax, u);
}

// ---- residues ------------------------------------------------------------------------------
// Thread (chunk kc, snapshot i, quarter q) converts the 16 rows r = 64 kc + 16 q + e of snapshot
// i (one 128-B run of the K-tiled fp64 A) and writes 16 bytes per modulus at
// R_l[kc][i][16 q ..]: a wave covers 16 snapshots x 64 rows = 1 KB contiguous per modulus.
// V: 0 = unsigned 11-bit limbs, the mean per lane (any ns); 8 = signed 14-bit limbs (two packed
// ops fewer per element pair and modulus) with the wave's mean through LDS (ns % 16 == 0, the
// default: 3.72 vs 4.37 ms at C3, profiles/r5/residues_ab.log).  r5 counters
// (profiles/r5/residues_pmc.json): ~2,000 VALU instructions per wave (4 cycles each) make a ~3 ms
// VALU floor at C3 -- not the HBM traffic, as r4 thought -- and the 16 per-lane mean loads of the
// r4 kernel, each behind its own branch and vmcnt(0), were two thirds of its L1 accesses and most
// of its load stalls.  (Measured and removed in r6 as A/B variants: signed limbs with per-lane
// means, unsigned limbs with the LDS mean, 8 elements per thread at 52 VGPRs -- none faster.)
template <int V>
__device__ __forceinline__ void residues_body(const double* __restrict__ AT, int ns, int64_t rowlen,
                                              int64_t rowpad, const double* __restrict__ mean,
                                              const double* __restrict__ devmax, int bbits, int64_t kc0,
                                              int64_t nkc, int8_t* __restrict__ R, int64_t ms, int64_t cs) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q = (int)(t & 3);
  const int64_t rest = t >> 2;
  if (rest >= nkc * ns) return;
  const int i = (int)(rest % ns);
  const int64_t kcl = rest / ns;
  const int64_t r0 = (kc0 + kcl) * 64 + q * 16;
  double a[16];
  // a - mean (main() :1494) past rowlen 0: the 16 mean loads unconditional (clamped index) and
  // issued together -- guarded one by one they compiled to 16 branches each ending in a
  // vmcnt(0), i.e. 16 serial memory round trips per wave, the kernel's bound (r5: 4.6 ms)
  auto sub_mean = [&](double (&x)[16]) {
    double mv[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) mv[e] = mean[r0 + e < rowlen ? r0 + e : rowlen - 1];
#pragma unroll
    for (int e = 0; e < 16; ++e) x[e] = r0 + e < rowlen ? x[e] - mv[e] : 0.0;
  };
  if constexpr (V == 8) {
    // the mean through LDS (ns % 16 == 0: one K chunk per wave): one 8-B load per lane fetches
    // the wave's 64 mean values, instead of 16 per-lane loads of 4 distinct slices (two thirds of
    // the kernel's L1 accesses)
    extern __shared__ __attribute__((aligned(16))) char res_lds[];
    double* M = reinterpret_cast<double*>(res_lds) + (threadIdx.x >> 6) * 64;
    const int lane = threadIdx.x & 63;
    const int64_t rm = (kc0 + kcl) * 64 + lane;
    M[lane] = mean[rm < rowlen ? rm : rowlen - 1];
    if (r0 < rowpad) {
      const double2* src = reinterpret_cast<const double2*>(AT + ((((r0 >> 4) * ns) + i) << 4));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double2 v = src[e];
        a[2 * e] = v.x;
        a[2 * e + 1] = v.y;
      }
      __builtin_amdgcn_wave_barrier();
      const double2* mq = reinterpret_cast<const double2*>(M + q * 16);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double2 mv = mq[e];
        a[2 * e] = r0 + 2 * e < rowlen ? a[2 * e] - mv.x : 0.0;
        a[2 * e + 1] = r0 + 2 * e + 1 < rowlen ? a[2 * e + 1] - mv.y : 0.0;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) a[e] = 0.0;
    }
  } else if (r0 < rowpad) {
    const double2* src = reinterpret_cast<const double2*>(AT + ((((r0 >> 4) * ns) + i) << 4));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double2 v = src[e];
      a[2 * e] = v.x;
      a[2 * e + 1] = v.y;
    }
    sub_mean(a);
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = 0.0;
  }
  const int sg = scale_exp(*devmax, bbits);
  // modulus l's bytes of this thread: R + l * ms + kcl * cs + i * 64 + q * 16 (ms, cs: the
  // modulus and K-chunk strides of the residue layout, see launch_corr_i8)
  int8_t* const rb = R + kcl * cs;
  const uint32_t doff = (uint32_t)(i * 64 + q * 16);
  // the byte of r + 1.5 * 2^23 (|r| <= 127) is r's two's-complement byte: pack 16 of them
  auto store16 = [&](const f32x2 (&sv)[8], int l) {
    uint32_t w[4];
#pragma unroll
    for (int pq = 0; pq < 4; ++pq) {
      const f32x2 u = sv[2 * pq], v = sv[2 * pq + 1];
      const uint32_t h0 = __builtin_amdgcn_perm(__float_as_uint(u.y), __float_as_uint(u.x), 0x0C0C0400u);
      const uint32_t h1 = __builtin_amdgcn_perm(__float_as_uint(v.y), __float_as_uint(v.x), 0x0C0C0400u);
      w[pq] = h0 | (h1 << 16);
    }
    int8_t* base = rb + (int64_t)l * ms;
    *reinterpret_cast<uint4*>(base + doff) = make_uint4(w[0], w[1], w[2], w[3]);
  };
  constexpr float MAG = 12582912.0f;  // 1.5 * 2^23
  if constexpr (V == 8) {
    // a' as four SIGNED 14-bit limbs, split in fp64 (every step exact): h = rint(a' 2^-28),
    // lo = a' - h 2^28 (|lo| <= 2^27), d3 = rint(h 2^-14), d2 = h - d3 2^14, d1 = rint(lo 2^-14),
    // d0 = lo - d1 2^14: |d0|, |d1|, |d2| <= 2^13, |d3| <= 2^10.  Per modulus, with the balanced
    // c_k = 2^14k mod m (|c_k| <= 127): s = d0 + c1 d1 + c2 d2 + c3 d3, |s| < 2^21.1, exact in
    // f32; q = rint(s / m) by one fma with 1.5 * 2^23 (|s fl(1/m) - s/m| <= 2^21.1 / 181 * 2^-24
    // < 2^-10.3 < 1/(2m), and s/m is never within 1/(2m) of a half-integer), r = s - q m.  Seven
    // packed ops per element pair and modulus (nine with unsigned 11-bit limbs + the offset).
    f32x2 F[4][8];
#pragma unroll
    for (int e = 0; e < 16; e += 2) {
      float d[4][2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const double ap = rint(ldexp(a[e + h2], sg));
        const double hh = rint(ap * 0x1p-28);
        const double lo = __builtin_fma(-hh, 0x1p28, ap);
        const double d3 = rint(hh * 0x1p-14), d1 = rint(lo * 0x1p-14);
        d[3][h2] = (float)d3;
        d[2][h2] = (float)__builtin_fma(-d3, 0x1p14, hh);
        d[1][h2] = (float)d1;
        d[0][h2] = (float)__builtin_fma(-d1, 0x1p14, lo);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) F[k][e / 2] = (f32x2){d[k][0], d[k][1]};
    }
    sfor<0, NMOD>([&](auto L) {
      constexpr int l = decltype(L)::value;
      constexpr float m = (float)kT.m[l], inv = 1.0f / (float)kT.m[l];
      constexpr float c1 = (float)kT.p14[l][1], c2 = (float)kT.p14[l][2], c3 = (float)kT.p14[l][3];
      f32x2 sv[8];
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[1][pr], (f32x2){c1, c1}, F[0][pr]);
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[2][pr], (f32x2){c2, c2}, sv[pr]);
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[3][pr], (f32x2){c3, c3}, sv[pr]);
      f32x2 qv[8];
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) qv[pr] = __builtin_elementwise_fma(sv[pr], (f32x2){inv, inv}, (f32x2){MAG, MAG});
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) qv[pr] = qv[pr] - (f32x2){MAG, MAG};
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(-qv[pr], (f32x2){m, m}, sv[pr]);
#pragma unroll
      for (int pr = 0; pr < 8; ++pr) sv[pr] = sv[pr] + (f32x2){MAG, MAG};
      store16(sv, l);
    });
    return;
  }
  // z = a' + 2^52 in [0, 2^53] as five 11-bit limbs z_k, held as exact f32
  float Fs[5][16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const double z = rint(ldexp(a[e], sg)) + 0x1p52;
    const double h = floor(z * 0x1p-32);
    const uint32_t lo = (uint32_t)__builtin_fma(-h, 0x1p32, z), hi = (uint32_t)h;
    Fs[0][e] = (float)(lo & 0x7FFu);
    Fs[1][e] = (float)((lo >> 11) & 0x7FFu);
    Fs[2][e] = (float)(((lo >> 22) | (hi << 10)) & 0x7FFu);
    Fs[3][e] = (float)((hi >> 1) & 0x7FFu);
    Fs[4][e] = (float)(hi >> 12);
  }
  f32x2 F[5][8];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) F[k][pr] = (f32x2){Fs[k][2 * pr], Fs[k][2 * pr + 1]};
  // per modulus m: s = sum_k z_k (2^11k mod m) + (-2^52 mod m) < 2^21.4, exact in f32.  The
  // quotient q = rint(s / m) comes from one fma, s * fl(1/m) + 1.5 * 2^23, rounded once to an
  // integer: |s fl(1/m) - s/m| <= (s/m) 2^-24 < 2^-10 < 1/(2m), and s/m (m odd) is never within
  // 1/(2m) of a half-integer, so it is exact; r = s - q m is the balanced residue, and
  // r + 1.5 * 2^23 holds r's two's-complement byte in its low mantissa bits (|r| <= 127)
  sfor<0, NMOD>([&](auto L) {
    constexpr int l = decltype(L)::value;
    constexpr float m = (float)kT.m[l], inv = 1.0f / (float)kT.m[l], o = (float)kT.off[l];
    constexpr float c1 = (float)kT.p11[l][1], c2 = (float)kT.p11[l][2], c3 = (float)kT.p11[l][3],
                    c4 = (float)kT.p11[l][4];
    // stage by stage over the 8 element pairs: independent packed ops back to back (no nops)
    f32x2 sv[8];
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[1][pr], (f32x2){c1, c1}, F[0][pr]);
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[2][pr], (f32x2){c2, c2}, sv[pr]);
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[3][pr], (f32x2){c3, c3}, sv[pr]);
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(F[4][pr], (f32x2){c4, c4}, sv[pr]);
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = sv[pr] + (f32x2){o, o};
    f32x2 qv[8];
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) qv[pr] = __builtin_elementwise_fma(sv[pr], (f32x2){inv, inv}, (f32x2){MAG, MAG});
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) qv[pr] = qv[pr] - (f32x2){MAG, MAG};
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = __builtin_elementwise_fma(-qv[pr], (f32x2){m, m}, sv[pr]);
#pragma unroll
    for (int pr = 0; pr < 8; ++pr) sv[pr] = sv[pr] + (f32x2){MAG, MAG};
    store16(sv, l);
  });
}

#define PODS_RES_ARGS const double* __restrict__ AT, int ns, int64_t rowlen, int64_t rowpad, \
    const double* __restrict__ mean, const double* __restrict__ devmax, int bbits, int64_t kc0, int64_t nkc, \
    int8_t* __restrict__ R, int64_t ms, int64_t cs
#define PODS_RES_PASS AT, ns, rowlen, rowpad, mean, devmax, bbits, kc0, nkc, R, ms, cs
// (r6: a cap of 4, 5 or 8 waves per SIMD instead of 3 -- 90-102 VGPRs -- left the whole pods_corr
// at 26.0-26.2 ms either way, profiles/r6/residues_occupancy_ab.log: the pass is VALU-bound)
#ifndef PODS_RES_WPE
#define PODS_RES_WPE 3
#endif
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, PODS_RES_WPE))) void k_residues(PODS_RES_ARGS) {
  residues_body<V>(PODS_RES_PASS);
}
#undef PODS_RES_ARGS
#undef PODS_RES_PASS

// ---- the int8 SYRK -----------------------------------------------------------------------

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_byte_addr) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)lds_byte_addr,
                                   16, 0, 0);
}

constexpr int TB = 256;            // tile rows / columns
constexpr int KC = 64;             // K bytes per chunk (one MFMA K step)
constexpr int PANEL = TB * KC;     // 16 KB: one chunk of 256 rows
constexpr int FOLD = 2048;         // K steps between the mod-m reductions of the accumulators
__device__ __forceinline__ int swz(int quartet) { return (0x78 >> (2 * quartet)) & 3; }

// One 256 x 256 tile of one modulus' residue SYRK over one K split.  8 waves as 2 x 4, each
// 128 x 64 = 8 x 4 blocks of v_mfma_i32_16x16x64_i8 (lane l: A[l&15][16(l>>4)+j],
// B[16(l>>4)+j][l&15]; D[4(l>>4)+r][l&15]).  Both operands are rows of the same K-tiled residue
// matrix, so a fragment is 16 consecutive 64-B rows of one K chunk.  Operands stream by LDS-DMA
// into an NST-stage ring (counted vmcnt + one barrier per K step); the fragments of step t+1
// are read between the two halves of step t's MFMAs.  A diagonal tile (SAME) loads one panel and
// reads it as both operands.  items: {bi, bj, split, -} (bi < 0: an empty slot that keeps the
// item count a multiple of 8).  DIAG (measurement only): 1 = no MFMAs, 2 = no operand traffic.
// Soft XCD pacing (the persistent SYRK): one lane of the workgroup counts it in and waits until
// all nslot workgroups of its XCD have arrived `epoch` times, or a bounded spin has passed.  It
// only paces the workgroups that share an L2 (so they read the same K window of the same panels);
// no data moves through it, so a timeout (a workgroup not resident yet) costs time, never
// correctness.  Raw s_barrier (no memory drain) around it; vector atomics only.
__device__ __forceinline__ void pace_xcd(unsigned* ctr, unsigned& epoch, unsigned nslot) {
  ++epoch;
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = epoch * nslot;
    for (int spin = 0; spin < (1 << 14); ++spin) {
      if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_s_barrier();
}


template <int NST, int DIAG, bool SAME, int ILV, int LD = 0>
__device__ __forceinline__ void syrk_tile(const int8_t* __restrict__ base, int64_t cstride, int ns, int nt, int i0,
                                          int j0, int m, char* smem, uint8_t* __restrict__ dst, int ldp,
                                          int accumulate) {
  constexpr int STG = 2 * PANEL;
  constexpr int Q = SAME ? 2 : 4;  // DMA instructions per wave per stage
  // DMA lead in K steps beyond the one being read: NST - 2, or with LD = 1 NST - 1 (the slot of
  // step t itself is refilled during step t: its fragments were read during step t - 1 and are
  // waited for before step t's barrier), one more stage in flight
  constexpr int D = NST - 2 + LD;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // LDS rows are 64 B (four 16-B slots); row R keeps logical slot s at physical slot
  // s ^ g((R >> 2) & 3), g = {0, 2, 3, 1}: ds_read_b128 serves a wave in the lane groups
  // {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32), and with this g the four 4-row quartets
  // of every group land on four different 16-B bank columns (conflict-free).  The DMA writes
  // each wave-instruction's 1 KB linearly, so the swizzle is applied to the source address.
  int64_t xo[2], yo[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rw = (wave * 2 + q) * 16 + (lane >> 2);
    const int ls = (lane & 3) ^ swz((rw >> 2) & 3);
    xo[q] = (int64_t)min(i0 + rw, ns - 1) * KC + ls * 16;
    yo[q] = (int64_t)min(j0 + rw, ns - 1) * KC + ls * 16;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  // piece q of step t's DMA (q < 2: the row panel, 2-3: the column panel)
  auto piece = [&](int t, int q) {
    if constexpr (DIAG == 2) return;
    const uint32_t sb = lds0 + (uint32_t)((t % NST) * STG);
    const int8_t* g = base + (int64_t)(DIAG == 3 || DIAG == 4 ? (t & 7) : t) * cstride;  // DIAG 3/4: an L2-resident K window
    if (q < 2) dma16(g + xo[q], sb + (wave * 2 + q) * 1024);
    else dma16(g + yo[q - 2], sb + PANEL + (wave * 2 + q - 2) * 1024);
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int q = 0; q < Q; ++q) piece(t, q);
  };
  i32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (i32x4){0, 0, 0, 0};
  const int wr = wave >> 2, wc = wave & 3;
  // a diagonal tile's waves (0, 2) and (0, 3) hold rows 0-127 x columns 128-255: strictly upper,
  // never stored -- they only load their share of the panel
  const bool idle = SAME && wr == 0 && wc >= 2;
  const int fo = (lane & 15) * KC + (((lane >> 4) ^ swz((lane >> 2) & 3)) * 16);  // row lane&15, slot lane>>4
  auto read = [&](int t, i32x4 (&av)[8], i32x4 (&bv)[4]) {
    const char* st = smem + (t % NST) * STG;
    const char* X = st + wr * 128 * KC + fo;
    const char* Y = st + (SAME ? 0 : PANEL) + wc * 64 * KC + fo;
#pragma unroll
    for (int a = 0; a < 8; ++a) av[a] = *reinterpret_cast<const i32x4*>(X + a * 16 * KC);
#pragma unroll
    for (int b = 0; b < 4; ++b) bv[b] = *reinterpret_cast<const i32x4*>(Y + b * 16 * KC);
  };
  // the MFMA rows a0 .. a0+3; with dt >= 0, DMA piece qb + k / qs of step dt after row a0 + k for
  // every k that is a multiple of qs (ILV variants: the pieces go among the MFMAs instead of back
  // to back after the barrier, where every wave of the CU would issue them at once)
  auto mma_rows = [&](const i32x4 (&av)[8], const i32x4 (&bv)[4], int a0, int dt, int qb, int qs) {
#pragma unroll
    for (int a = a0; a < a0 + 4; ++a) {
      if constexpr (DIAG == 1 || DIAG == 4) {
        acc[a][0] += av[a] ^ bv[a & 3];
      } else {
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[a], bv[b], acc[a][b], 0, 0, 0);
      }
      if constexpr (ILV != 0) {
        const int k = a - a0;
        if (dt >= 0 && k % qs == 0 && qb + k / qs < Q) {
          __builtin_amdgcn_sched_barrier(0);
          piece(dt, qb + k / qs);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };
  auto fold = [&](int t) {
    if ((t + 1) % FOLD == 0 && t + 1 < nt) {
      // |acc| stays < m + 2048 * 64 * 127^2 < 2^31
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][r] %= m;
    }
  };
  // step t: every wave waits for stage t+1, one barrier, the DMA of stage t + D + 1 into the
  // slot of step t - 1 (read during step t - 1's MFMAs, consumed by them), then step t's MFMAs
  // with the reads of step t+1 between their halves -- the wait the compiler puts at the loop
  // head (lgkmcnt(0)) then finds those reads long complete.  With ILV the DMA pieces go among
  // the MFMA rows: issued back to back right after the barrier, all 8 waves of the CU stall on
  // them at once (an LDS-DMA issue costs ~60-185 cycles) while the MFMA pipes idle
#pragma unroll
  for (int t = 0; t <= D; ++t)
    if (t < nt) issue(t);
  if (D < nt) wait_vm<Q * D>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  i32x4 a0[8], b0[4], a1[8], b1[4];
  if (!idle) read(0, a0, b0);
  // ILV: 0 = the DMA pieces of step t + D + 1 back to back after the barrier; 1 = one after each
  // of the first Q MFMA rows; 2 = after every second row over both halves; 4 = after the rows of
  // the second half (behind the reads of step t + 1)
  auto step = [&](int t, const i32x4 (&ac)[8], const i32x4 (&bc)[4], i32x4 (&an)[8], i32x4 (&bn)[4]) {
    if (t + 1 < nt) {
      if (t + D < nt) wait_vm<Q * (D - 1)>();
      else wait_vm<0>();
      if constexpr (LD == 1) __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's reads of slot t done
      if constexpr (DIAG != 5) __builtin_amdgcn_s_barrier();  // DIAG 5 (measurement only): no per-step barrier
      __builtin_amdgcn_sched_barrier(0);
      if (ILV == 0 || idle)
        if (t + D + 1 < nt) issue(t + D + 1);
    }
    if (idle) return;
    const int dt = ILV != 0 && t + D + 1 < nt ? t + D + 1 : -1;
    mma_rows(ac, bc, 0, ILV == 4 ? -1 : dt, 0, ILV == 2 ? 2 : 1);
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < nt) read(t + 1, an, bn);
    __builtin_amdgcn_sched_barrier(0);
    mma_rows(ac, bc, 4, ILV == 2 || ILV == 4 ? dt : -1, ILV == 2 ? 2 : 0, ILV == 2 ? 2 : 1);
    fold(t);
  };
  int t = 0;
  for (; t + 1 < nt; t += 2) {
    step(t, a0, b0, a1, b1);
    step(t + 1, a1, b1, a0, b0);
  }
  if (t < nt) step(t, a0, b0, a1, b1);
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = i0 + wr * 128 + a * 16 + 4 * fq + r;
        const int gj = j0 + wc * 64 + b * 16 + fr;
        if (gi < ns && gj <= gi) {
          int v = acc[a][b][r] % m;
          if (v < 0) v += m;
          uint8_t* p = dst + (int64_t)gi * ldp + gj;
          if (accumulate) {
            v += *p;
            if (v >= m) v -= m;
          }
          *p = (uint8_t)v;
        }
      }
}

#ifdef PODS_DIAG
// The launch-per-item grid form (r4; the persistent kernel replaced it in r5) and its
// measurement-only variants (DIAG: wrong results): the diagnostic library only (tools/lib_variants.sh
// diag), never libpodsgen.so.
template <int NST, int DIAG = 0, int ILV = 0>
__global__ __launch_bounds__(512, 1) void k_syrk_i8(const int8_t* __restrict__ R, int ns, int64_t ms, int64_t cs,
                                                    int kcs,
                                                    const int4* __restrict__ items, int nitems, int nsplit,
                                                    uint8_t* __restrict__ P, int64_t pslab, int ldp, int accumulate,
                                                    int xcd_ranges) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  int b = blockIdx.x;
  if (xcd_ranges) {  // block b runs on XCD b % 8: give each XCD a contiguous range of the work
    const int nb = gridDim.x, xcd = b & 7, q = nb >> 3, rr = nb & 7;
    b = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  }
  const int l = b / nitems;
  const int4 it = items[b - l * nitems];
  if (it.x < 0) return;
  const int bi = it.x, bj = it.y, sp = it.z;
  const int8_t* base = R + (int64_t)l * ms + (int64_t)sp * kcs * cs;
  uint8_t* dst = P + (int64_t)(l * nsplit + sp) * pslab;
  const int m = modulus(l);
  if (bi == bj)
    syrk_tile<NST, DIAG, true, ILV>(base, cs, ns, kcs, bi * TB, bj * TB, m, smem, dst, ldp, accumulate);
  else
    syrk_tile<NST, DIAG, false, ILV>(base, cs, ns, kcs, bi * TB, bj * TB, m, smem, dst, ldp, accumulate);
}

#endif  // PODS_DIAG

// The persistent, XCD-paced form (r5): one 512-thread workgroup per CU, workgroup b on XCD b % 8
// (dispatch deals blocks round-robin over the XCDs) as slot b / 8 of nslot.  XCD x's items (its
// share of every modulus' lower tiles and K splits, host-ordered so that one round -- nslot
// consecutive items -- is a compact block of tiles of one modulus and split) are taken in rounds,
// slot s taking item r * nslot + s of round r, with a soft pacing point after every round: the
// workgroups that share an L2 then stream the same K window of the same panels (the
// launch-per-item form let them drift apart over the 17 rounds at C3, and the XCD's 4 MB L2 held
// the union of their windows: 54 % hits).  5-stage ring, the DMA pieces among the first MFMA rows
// (ILV 1), one more stage in flight (LD 1).
template <int NST, int ILV, int LD>
__global__ __launch_bounds__(512, 1) void k_syrk_i8_paced(const int8_t* __restrict__ R, int ns, int64_t ms, int64_t cs,
                                                          int kcs, const int4* __restrict__ xitems, int per_xcd,
                                                          int nsplit, uint8_t* __restrict__ P, int64_t pslab, int ldp,
                                                          int accumulate, unsigned* __restrict__ pace_ctr) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  unsigned* const ctr = pace_ctr + x * 32;  // one 128-B line per XCD
  const unsigned nslot = gridDim.x >> 3;
  unsigned epoch = 0;
  const int rounds = (per_xcd + (int)nslot - 1) / (int)nslot;
#pragma clang loop unroll(disable)
  for (int r = 0; r < rounds; ++r) {
    const int idx = r * (int)nslot + slot;
    const int4 it = idx < per_xcd ? xitems[(int64_t)x * per_xcd + idx] : make_int4(-1, -1, 0, 0);
    if (it.x >= 0) {
      const int bi = it.x, bj = it.y, sp = it.z, l = it.w;
      const int8_t* base = R + (int64_t)l * ms + (int64_t)sp * kcs * cs;
      uint8_t* dst = P + (int64_t)(l * nsplit + sp) * pslab;
      const int m = modulus(l);
      if (bi == bj)
        syrk_tile<NST, 0, true, ILV, LD>(base, cs, ns, kcs, bi * TB, bj * TB, m, smem, dst, ldp, accumulate);
      else
        syrk_tile<NST, 0, false, ILV, LD>(base, cs, ns, kcs, bi * TB, bj * TB, m, smem, dst, ldp, accumulate);
    }
    pace_xcd(ctr, epoch, nslot);
  }
}

// ---- CRT reconstruction ----------------------------------------------------------------------
// 16 residues 0 <= c_l < 2^16 -> the integer X in [-(M-1)/2, (M-1)/2] with X = c_l mod m_l, as a double
__device__ __forceinline__ double crt_value(const int (&c)[NMOD]) {
  // Garner's digits kept balanced, v_l in [-(m_l-1)/2, (m_l-1)/2], in f32: every operand is
  // an integer below 2^17, the quotient rint(x/m) is one fma with 1.5*2^23 (error <= 2^-15,
  // far below 1/(2m); the argument of k_residues), so each step is exact.  With balanced
  // digits Horner gives the signed X directly (|X| <= (M-1)/2).
  constexpr float MAG = 12582912.0f;
  float v[NMOD];
  sfor<0, NMOD>([&](auto L) {
    constexpr int l = decltype(L)::value;
    constexpr float ml = (float)kT.m[l], rm = 1.0f / (float)kT.m[l];
    float t = (float)c[l];
    {  // balance c_l itself
      const float q = __builtin_fmaf(t, rm, MAG) - MAG;
      t = __builtin_fmaf(-q, ml, t);
    }
    sfor<0, l>([&](auto K) {
      constexpr int k = decltype(K)::value;
      constexpr float ik = (float)kT.inv[k][l];
      const float x = (t - v[k]) * ik;  // |x| < 2^16.1, exact
      const float q = __builtin_fmaf(x, rm, MAG) - MAG;
      t = __builtin_fmaf(-q, ml, x);
    });
    v[l] = t;
  });
  __int128 X = (__int128)(int)v[NMOD - 1];
#pragma unroll
  for (int l = NMOD - 2; l >= 0; --l) X = X * kT.m[l] + (int)v[l];
  const bool neg = X < 0;
  const unsigned __int128 mag = neg ? (unsigned __int128)(-X) : (unsigned __int128)X;
  const uint64_t hi = (uint64_t)(mag >> 64), lo = (uint64_t)mag;
  double d;
  if (hi == 0) {
    d = (double)lo;
  } else {
    const int p = 127 - __builtin_clzll(hi);  // top bit of mag
    uint64_t top = (uint64_t)(mag >> (p - 63));
    // the bits below the top 64 as a sticky bit: (double)top then rounds as the whole 128-bit
    // value would (the rounding position is bit 10 of top), so C' is rounded to double once
    top |= (mag << (128 - (p - 63))) != 0 ? 1u : 0u;
    d = ldexp((double)top, p - 63);
  }
  return neg ? -d : d;
}

// C[i][j] (lower 64 x 64 tiles, mirrored through LDS as k_syrk_reduce) from the partials:
// thread (row r, column quad) loads each modulus' / split's 4 residues of its row as one u32
// (P rows padded to ldp, a multiple of 64)
__global__ __launch_bounds__(256) void k_crt(const uint8_t* __restrict__ P, int nsplit, int64_t pslab, int ldp,
                                             int ns, const double* __restrict__ devmax, int bbits,
                                             double* __restrict__ C, int64_t ldc, int divide) {
  __shared__ double tile[64][65];
  const int L = blockIdx.x;
  int ti = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
  while (ti * (ti + 1) / 2 > L) --ti;
  const int tj = L - ti * (ti + 1) / 2;
  const int cq = threadIdx.x & 15, rq = threadIdx.x >> 4;
  const int sg = scale_exp(*devmax, bbits);
  const double dn = (double)ns;
#pragma unroll 1
  for (int it = 0; it < 4; ++it) {
    const int r = rq + 16 * it;
    const int i = ti * 64 + r, jb = tj * 64 + 4 * cq;
    double val[4] = {0.0, 0.0, 0.0, 0.0};
    if (i < ns) {
      // the splits' bytes summed in 16-bit fields: even bytes (entries 0, 2), odd (1, 3)
      uint32_t ev[NMOD], od[NMOD];
      const uint8_t* src = P + (int64_t)i * ldp + jb;
#pragma unroll
      for (int l = 0; l < NMOD; ++l) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(src + (int64_t)(l * nsplit) * pslab);
        ev[l] = v & 0x00FF00FFu;
        od[l] = (v >> 8) & 0x00FF00FFu;
      }
      for (int sp = 1; sp < nsplit; ++sp)
#pragma unroll
        for (int l = 0; l < NMOD; ++l) {
          const uint32_t v = *reinterpret_cast<const uint32_t*>(src + (int64_t)(l * nsplit + sp) * pslab);
          ev[l] += v & 0x00FF00FFu;
          od[l] += (v >> 8) & 0x00FF00FFu;
        }
#pragma unroll 1
      for (int k = 0; k < 4; ++k) {
        const int j = jb + k;
        if (j < ns && (ti > tj || j <= i)) {
          int cr[NMOD];
          const int sh = 16 * (k >> 1);
          sfor<0, NMOD>([&](auto Lm) {
            constexpr int l = decltype(Lm)::value;
            cr[l] = (int)((((k & 1) ? od[l] : ev[l]) >> sh) & 0xFFFFu);  // < 2^16: crt_value reduces
          });
          double v = ldexp(crt_value(cr), -2 * sg);
          if (divide) v = v / dn;
          C[(int64_t)i * ldc + j] = v;
          val[k] = v;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[r][4 * cq + k] = val[k];
  }
  __syncthreads();
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll 4
  for (int r = r0; r < 64; r += 4) {
    const int i = tj * 64 + r, j = ti * 64 + c;
    const bool ok = i < ns && j < ns && (ti > tj || r < c);
    if (ok) C[(int64_t)i * ldc + j] = tile[c][r];
  }
}

}  // namespace i8

// ---- host ------------------------------------------------------------------------------------
namespace {
constexpr int I8_KSUB = 1;  // K chunks per split are a multiple of this
}

int corr_i8_nmod() { return i8::NMOD; }

int corr_i8_plan(int ns, int64_t rowlen, int64_t rowpad, int64_t budget_bytes, CorrI8Plan* out, int force_split) {
  if (ns <= 0 || rowlen <= 0 || rowpad < rowlen || !out) return -1;
  CorrI8Plan p{};
  // b: 2 |C'| <= 2 K 2^2b < M
  const int b = (int)std::floor((i8::kLog2M - 1.0 - std::log2((double)rowlen)) / 2.0);
  p.bbits = std::min(52, b);
  if (p.bbits < 40) return -1;  // K beyond ~2^43: more moduli needed
  const int64_t nkc = (rowpad + i8::KC - 1) / i8::KC;
  const int64_t per_chunk = (int64_t)i8::NMOD * ns * i8::KC;  // residue bytes per K chunk
  int64_t cmax = std::max<int64_t>(I8_KSUB * 64, budget_bytes / per_chunk);
  // k_residues addresses one modulus' residues with a 32-bit offset (< chunks * ns * 64): keep
  // a launch's chunks below 2^32 / (ns * 64), less the up-to-7 chunks the split rounding adds
  const int64_t cmax32 = (int64_t)0xFFFFFFFF / ((int64_t)ns * i8::KC) - 8;
  if (cmax32 < 1) return -1;
  cmax = std::min(cmax, cmax32);
  p.nlaunch = (int)((nkc + cmax - 1) / cmax);
  const int64_t per_launch = (nkc + p.nlaunch - 1) / p.nlaunch;
  const int nb = (ns + i8::TB - 1) / i8::TB;
  const int tiles = nb * (nb + 1) / 2;
  const int tiles8 = (tiles + 7) / 8 * 8;
  // K splits: fill 256 CUs (one workgroup each) with the least idle last round, >= 128 K steps
  // each (a rank's slab at N = 8, 384 K steps at C3, now takes two splits: 8.5 instead of 9
  // rounds; 3.74 vs 3.86 ms per correlation forced on one box, within the box-to-box spread)
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && per_launch / s < 128) break;
    const double items = (double)tiles * i8::NMOD * s;
    const double cost = std::ceil(items / 256.0) / s + 0.01 * s;
    if (cost < best_cost - 1e-12) {
      best_cost = cost;
      best = s;
    }
  }
  // a forced split count is capped at 8 like the planner's own: k_crt sums the splits' bytes in
  // 16-bit fields (<= 257 splits) and the item order deals splits over the 8 XCDs
  p.nsplit = force_split > 0 ? (int)std::min<int64_t>(std::min(force_split, 8), per_launch) : best;
  best = p.nsplit;
  p.kcs = (int)(((per_launch + best - 1) / best + I8_KSUB - 1) / I8_KSUB * I8_KSUB);
  p.chunks = (int64_t)p.nsplit * p.kcs;  // chunks per launch (zero-padded past rowpad)
  if (p.chunks * ns * i8::KC > (int64_t)0xFFFFFFFF) return -1;  // the 32-bit residue offsets
  p.nkc = nkc;
  p.nitems = tiles8 * p.nsplit;
  p.r_bytes = (int64_t)i8::NMOD * p.chunks * ns * i8::KC;
  p.p_bytes = (int64_t)i8::NMOD * p.nsplit * ns * ((ns + 63) / 64 * 64);
  *out = p;
  return 0;
}

// {bi, bj, split, 0} per item: each split's lower 256-tiles in Morton order, cut into 8 compact
// groups, and interleaved so that item 8k + x holds group x's k-th tile (hardware sends block b
// to XCD b % 8, so each XCD's L2 sees a compact group of tiles); padded with empty slots.
std::vector<int> corr_i8_items(int ns, const CorrI8Plan& p) {
  const int nb = (ns + i8::TB - 1) / i8::TB;
  std::vector<std::pair<uint32_t, std::pair<int, int>>> t;
  for (int bi = 0; bi < nb; ++bi)
    for (int bj = 0; bj <= bi; ++bj) {
      uint32_t key = 0;
      for (int k = 0; k < 16; ++k) key |= ((((uint32_t)bi >> k) & 1u) << (2 * k + 1)) | ((((uint32_t)bj >> k) & 1u) << (2 * k));
      t.push_back({key, {bi, bj}});
    }
  std::sort(t.begin(), t.end());
  const int tiles = (int)t.size(), per = (tiles + 7) / 8;
  // XCD lane x (grid position 8k + x; nitems is a multiple of 8) takes split x % S and Morton group
  // x / S of the 8 / S groups, so an XCD's concurrent workgroups all read one K range of one
  // modulus, on a compact block of tiles (S in {1, 2, 4, 8}; L2-miss traffic 96.9 -> 65.0 GB per
  // launch against interleaved Morton groups, r4).  (Measured and removed in r6 as A/B orders: plain
  // Morton, XCD-contiguous ranges of it -- 0.3-0.7 ms slower.)
#ifdef PODS_DIAG
  if (const char* ord = std::getenv("PODS_CORR_ORDER"); ord && ord[0] == 's') {
    // measurement only (wrong results): every item is tile (1, 0)
    std::vector<int> out;
    for (int s = 0; s < p.nsplit; ++s)
      for (int k = 0; k < per * 8; ++k) out.insert(out.end(), {nb > 1 ? 1 : 0, 0, s, 0});
    return out;
  }
#endif
  if (8 % p.nsplit == 0) {
    const int ngrp = 8 / p.nsplit, gsz = (tiles + ngrp - 1) / ngrp;
    std::vector<int> out;
    out.reserve((size_t)8 * gsz * 4);
    for (int k = 0; k < gsz; ++k)
      for (int x = 0; x < 8; ++x) {
        const int sp = x % p.nsplit, grp = x / p.nsplit, idx = grp * gsz + k;
        if (idx < tiles) {
          out.push_back(t[idx].second.first);
          out.push_back(t[idx].second.second);
        } else {
          out.push_back(-1);
          out.push_back(-1);
        }
        out.push_back(sp);
        out.push_back(0);
      }
    return out;
  }
  // other split counts (a forced PODS_CORR_SPLITS): split-major, Morton groups interleaved over XCDs
  std::vector<int> out;
  out.reserve((size_t)p.nitems * 4);
  for (int s = 0; s < p.nsplit; ++s)
    for (int k = 0; k < per; ++k)
      for (int x = 0; x < 8; ++x) {
        const int idx = x * per + k;
        if (idx < tiles) {
          out.push_back(t[idx].second.first);
          out.push_back(t[idx].second.second);
          out.push_back(s);
        } else {
          out.push_back(-1);
          out.push_back(-1);
          out.push_back(s);
        }
        out.push_back(0);
      }
  return out;
}

hipError_t launch_absdev(const double* AT, int ns, int64_t rowlen, int64_t rowpad, const double* mean,
                         double* devmax, hipStream_t st) {
  hipError_t e = hipMemsetAsync(devmax, 0, sizeof(double), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(i8::k_absdev, dim3(2048), dim3(256), 0, st, AT, ns, rowlen, rowpad, mean,
                     reinterpret_cast<unsigned long long*>(devmax));
  return hipGetLastError();
}

// The persistent kernel's table: XCD x's items of every modulus in grid order (item 8k + x of the
// grid table), empty slots dropped, as {bi, bj, split, modulus}; per_xcd items per XCD (padded
// with empty items to the longest list)
std::vector<int> corr_i8_xcd_items(const std::vector<int>& items, int nitems, int* per_xcd) {
  std::vector<std::vector<int>> per(8);
  for (int l = 0; l < i8::NMOD; ++l)
    for (int k = 0; k < nitems; ++k) {
      if (items[4 * k] < 0) continue;
      per[k & 7].insert(per[k & 7].end(), {items[4 * k], items[4 * k + 1], items[4 * k + 2], l});
    }
  int px = 0;
  for (int x = 0; x < 8; ++x) px = std::max(px, (int)per[x].size() / 4);
  std::vector<int> out((size_t)8 * px * 4, -1);
  for (int x = 0; x < 8; ++x) std::copy(per[x].begin(), per[x].end(), out.begin() + (size_t)x * px * 4);
  *per_xcd = px;
  return out;
}

hipError_t launch_corr_i8(const double* AT, int ns, int64_t rowlen, int64_t rowpad, const double* mean,
                          const double* devmax, const CorrI8Plan& p, const int* items, int8_t* R, uint8_t* P,
                          double* C, int64_t ldc, int divide, hipStream_t st, hipEvent_t syrk_begin,
                          hipEvent_t syrk_end, const int* xitems, int per_xcd, unsigned* pace_ctr) {
  using namespace i8;
  if (!xitems || !pace_ctr) return hipErrorInvalidValue;
  // residue layout: modulus l's K chunk kc at R + l * ms + kc * cs, one matrix per modulus
  // ([NMOD][chunks][ns][64]); the moduli interleaved per chunk ([chunks][NMOD][ns][64], a residue
  // wave's 16 stores in one window) measured no faster (r5, profiles/r5/residue_layout_ab.log)
  const int64_t ms = p.chunks * ns * KC;
  const int64_t cs = (int64_t)ns * KC;
  const int ldp = (ns + 63) / 64 * 64;
  const int64_t pslab = (int64_t)ns * ldp;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  const int nslot = std::max(1, cus / 8);
  // The SYRK: the persistent XCD-paced kernel (k_syrk_i8_paced: 22.34 vs 22.89 ms at C3 for the
  // r4 launch-per-item grid, profiles/r5/pace_ab.log), 5 ring stages, each wave's DMA pieces one
  // after each of its first MFMA rows (ILV 1: 22.0-22.8 ms against 24.0 for the pieces back to back
  // after the barrier, profiles/r4/corr_i8_ilv_ab.log), one more stage in flight (LD 1: 21.89 vs
  // 22.12 ms, profiles/r5/syrk_lead_wide_ab.log).  (A/B variants measured equal or slower and
  // removed in r6: 4 stages, ILV 2 / 4, the r4 lead, 256 x 384 tiles, pacing points inside a tile.)
  const void* syrk = reinterpret_cast<const void*>(&k_syrk_i8_paced<5, 1, 1>);
#ifdef PODS_DIAG
  // the diagnostic library only (tools/lib_variants.sh diag): PODS_SYRK_I8 selects the r4 grid form
  // "g", or its measurement-only variants (wrong results) "9m" / "9d" / "9w" / "9x" / "9y" / "9b":
  // no MFMAs / no operand traffic / an L2-resident K window / both / the window with ILV 1 / no
  // per-step barrier
  int variant = 0;
  if (const char* v = std::getenv("PODS_SYRK_I8")) {
    if (v[0] == 'g') variant = 45;
    if (v[0] == '9') variant = v[1] == 'm' ? 91 : v[1] == 'w' ? 93 : v[1] == 'x' ? 94 : v[1] == 'y' ? 95 : v[1] == 'b' ? 96 : 92;
  }
  const void* grid_fn = variant == 91 ? reinterpret_cast<const void*>(&k_syrk_i8<4, 1>)
                      : variant == 92 ? reinterpret_cast<const void*>(&k_syrk_i8<4, 2>)
                      : variant == 93 ? reinterpret_cast<const void*>(&k_syrk_i8<4, 3>)
                      : variant == 94 ? reinterpret_cast<const void*>(&k_syrk_i8<4, 4>)
                      : variant == 95 ? reinterpret_cast<const void*>(&k_syrk_i8<4, 3, 1>)
                      : variant == 96 ? reinterpret_cast<const void*>(&k_syrk_i8<5, 5, 1>)
                      : variant == 45 ? reinterpret_cast<const void*>(&k_syrk_i8<5, 0, 1>)
                                      : nullptr;
  const size_t grid_lds = (size_t)(variant == 45 || variant == 96 ? 5 : 4) * 2 * PANEL;
  if (grid_fn) {
    e = hipFuncSetAttribute(grid_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)grid_lds);
    if (e != hipSuccess) return e;
  }
#endif
  e = hipFuncSetAttribute(syrk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(5 * 2 * PANEL));
  if (e != hipSuccess) return e;
  if (syrk_begin && p.nlaunch > 1) e = hipEventRecord(syrk_begin, st);
  if (e != hipSuccess) return e;
  for (int li = 0; li < p.nlaunch; ++li) {
    const int64_t kc0 = (int64_t)li * p.chunks;
    // residues: k_residues<8> (the wave's 64 mean values through LDS, signed 14-bit limbs) when
    // ns % 16 == 0 (a wave then covers one K chunk), else k_residues<0>
    const int64_t thr = p.chunks * ns * 4;
    const bool r8 = ns % 16 == 0;
    const void* rk = r8 ? reinterpret_cast<const void*>(&k_residues<8>) : reinterpret_cast<const void*>(&k_residues<0>);
    {
      const double* AT_ = AT;
      const double* mean_ = mean;
      const double* dm_ = devmax;
      int bb_ = p.bbits;
      int64_t kc_ = kc0, nk_ = p.chunks, ms_ = ms, cs_ = cs, rl_ = rowlen, rp_ = rowpad;
      int ns_ = ns;
      int8_t* R_ = R;
      void* rargs[] = {&AT_, &ns_, &rl_, &rp_, &mean_, &dm_, &bb_, &kc_, &nk_, &R_, &ms_, &cs_};
      e = hipLaunchKernel(rk, dim3((unsigned)((thr + 255) / 256)), dim3(256), rargs, r8 ? 4 * 512 : 0, st);
      if (e != hipSuccess) return e;
    }
    // the events bracket the SYRK launch (with several launches: the first residue pass to the last SYRK)
    if (syrk_begin && p.nlaunch == 1) e = hipEventRecord(syrk_begin, st);
    if (e != hipSuccess) return e;
#ifdef PODS_DIAG
    if (grid_fn) {
      const int ldp_ = ldp;
      const int acc_ = li > 0 ? 1 : 0;
      const int4* it_ = reinterpret_cast<const int4*>(items);
      int64_t ms_ = ms, cs_ = cs;
      int xr_ = 0;
      void* args[] = {&R, const_cast<int*>(&ns), &ms_, &cs_, const_cast<int*>(&p.kcs),
                      &it_, const_cast<int*>(&p.nitems), const_cast<int*>(&p.nsplit), &P,
                      const_cast<int64_t*>(&pslab), const_cast<int*>(&ldp_), const_cast<int*>(&acc_), &xr_};
      e = hipLaunchKernel(grid_fn, dim3((unsigned)(NMOD * p.nitems)), dim3(512), args, grid_lds, st);
      if (e != hipSuccess) return e;
      continue;
    }
#else
    (void)items;
#endif
    e = hipMemsetAsync(pace_ctr, 0, 8 * 32 * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_syrk_i8_paced<5, 1, 1>), dim3(8 * nslot), dim3(512), 5 * 2 * PANEL, st,
                       (const int8_t*)R, ns, ms, cs, p.kcs, reinterpret_cast<const int4*>(xitems), per_xcd,
                       p.nsplit, P, pslab, ldp, li > 0 ? 1 : 0, pace_ctr);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (syrk_end) e = hipEventRecord(syrk_end, st);
  if (e != hipSuccess) return e;
  const int nt = (ns + 63) / 64;
  hipLaunchKernelGGL(k_crt, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(256), 0, st, P, p.nsplit, pslab, ldp, ns,
                     devmax, p.bbits, C, ldc, divide);
  return hipGetLastError();
}

}  // namespace pods

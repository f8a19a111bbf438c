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
__global__ __launch_bounds__(256) void k_residues(const double* __restrict__ AT, int ns, int64_t rowlen,
                                                  int64_t rowpad, const double* __restrict__ mean,
                                                  const double* __restrict__ devmax, int bbits, int64_t kc0,
                                                  int64_t nkc, int8_t* __restrict__ R, int64_t lstride) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int q = (int)(t & 3);
  const int64_t rest = t >> 2;
  if (rest >= nkc * ns) return;
  const int i = (int)(rest % ns);
  const int64_t kcl = rest / ns;
  const int64_t r0 = (kc0 + kcl) * 64 + q * 16;
  double a[16];
  if (r0 < rowpad) {
    const double2* src = reinterpret_cast<const double2*>(AT + ((((r0 >> 4) * ns) + i) << 4));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const double2 v = src[e];
      a[2 * e] = v.x;
      a[2 * e + 1] = v.y;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = r0 + e < rowlen ? a[e] - mean[r0 + e] : 0.0;  // main() :1494
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) a[e] = 0.0;
  }
  const int sg = scale_exp(*devmax, bbits);
  // z = a' + 2^52 in [0, 2^53] as three limbs of 18 bits (all steps exact)
  uint32_t z0[16], z1[16], z2[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const double z = rint(ldexp(a[e], sg)) + 0x1p52;
    const double h2 = floor(z * 0x1p-36);
    const double rem = __builtin_fma(-h2, 0x1p36, z);
    const double h1 = floor(rem * 0x1p-18);
    const double h0 = __builtin_fma(-h1, 0x1p18, rem);
    z2[e] = (uint32_t)h2;
    z1[e] = (uint32_t)h1;
    z0[e] = (uint32_t)h0;
  }
  int8_t* dst = R + (kcl * ns + i) * 64 + q * 16;
  sfor<0, NMOD>([&](auto L) {
    constexpr int l = decltype(L)::value;
    constexpr uint32_t m = kT.m[l], c1 = kT.p18[l], c2 = kT.p36[l], o = kT.off[l];
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t s = z2[e] * c2 + z1[e] * c1 + z0[e] + o;  // < 2^27
      int v = (int)(s % m);
      if (v > (int)(m / 2)) v -= (int)m;
      w[e >> 2] |= ((uint32_t)v & 255u) << (8 * (e & 3));
    }
    *reinterpret_cast<uint4*>(dst + (int64_t)l * lstride) = make_uint4(w[0], w[1], w[2], w[3]);
  });
}

// ---- the int8 SYRK -----------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));

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

// One 256 x 256 tile of one modulus' residue SYRK over one K split.  8 waves as 2 x 4, each
// 128 x 64 = 8 x 4 blocks of v_mfma_i32_16x16x64_i8 (lane l: A[l&15][16(l>>4)+j],
// B[16(l>>4)+j][l&15]; D[4(l>>4)+r][l&15]).  Both operands are rows of the same K-tiled residue
// matrix, so a fragment is 16 consecutive 64-B rows = 1 KB contiguous in LDS (conflict-free
// ds_read_b128, no swizzle).  Operands stream by LDS-DMA into an NST-stage ring of KSUB chunks
// per stage (counted vmcnt + barrier, as k_syrk_g128).  items: {bi, bj, split, -} (bi < 0: an
// empty slot that keeps the item count a multiple of 8).
template <int NST, int KSUB>
__global__ __launch_bounds__(512, 1) void k_syrk_i8(const int8_t* __restrict__ R, int ns, int64_t lstride, int kcs,
                                                    const int4* __restrict__ items, int nitems, int nsplit,
                                                    uint8_t* __restrict__ P, int64_t pslab, int accumulate) {
  constexpr int STG = KSUB * 2 * PANEL;
  constexpr int Q = KSUB * 4;  // DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int l = blockIdx.x / nitems;
  const int4 it = items[blockIdx.x - l * nitems];
  if (it.x < 0) return;
  const int bi = it.x, bj = it.y, sp = it.z;
  const int i0 = bi * TB, j0 = bj * TB;
  const int nt = kcs / KSUB;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int8_t* base = R + (int64_t)l * lstride + (int64_t)sp * kcs * ns * KC;
  int64_t xo[2], yo[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int rw = (wave * 2 + q) * 16 + (lane >> 2);
    xo[q] = (int64_t)min(i0 + rw, ns - 1) * KC + (lane & 3) * 16;
    yo[q] = (int64_t)min(j0 + rw, ns - 1) * KC + (lane & 3) * 16;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const int64_t cstride = (int64_t)ns * KC;
  auto issue = [&](int t) {
    const uint32_t sb = lds0 + (uint32_t)((t % NST) * STG);
#pragma unroll
    for (int ks = 0; ks < KSUB; ++ks) {
      const int8_t* g = base + (int64_t)(t * KSUB + ks) * cstride;
#pragma unroll
      for (int q = 0; q < 2; ++q) dma16(g + xo[q], sb + (ks * 2) * PANEL + (wave * 2 + q) * 1024);
#pragma unroll
      for (int q = 0; q < 2; ++q) dma16(g + yo[q], sb + (ks * 2 + 1) * PANEL + (wave * 2 + q) * 1024);
    }
  };
  i32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (i32x4){0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nt) issue(t);
  const int m = modulus(l);
  const int wr = wave >> 2, wc = wave & 3;
  const int fo = (lane & 15) * KC + (lane >> 4) * 16;
  for (int t = 0; t < nt; ++t) {
    if (t + NST - 2 < nt) wait_vm<Q * (NST - 2)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NST - 1 < nt) issue(t + NST - 1);
    const char* st = smem + (t % NST) * STG;
#pragma unroll
    for (int ks = 0; ks < KSUB; ++ks) {
      const char* X = st + ks * 2 * PANEL + wr * 128 * KC + fo;
      const char* Y = st + (ks * 2 + 1) * PANEL + wc * 64 * KC + fo;
      i32x4 av[8], bv[4];
#pragma unroll
      for (int a = 0; a < 8; ++a) av[a] = *reinterpret_cast<const i32x4*>(X + a * 16 * KC);
#pragma unroll
      for (int b = 0; b < 4; ++b) bv[b] = *reinterpret_cast<const i32x4*>(Y + b * 16 * KC);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    if (((t + 1) * KSUB) % FOLD == 0 && t + 1 < nt) {
      // |acc| stays < m + 2048 * 64 * 127^2 < 2^31
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][r] %= m;
    }
  }
  uint8_t* dst = P + (int64_t)(l * nsplit + sp) * pslab;
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
          uint8_t* p = dst + (int64_t)gi * ns + gj;
          if (accumulate) {
            v += *p;
            if (v >= m) v -= m;
          }
          *p = (uint8_t)v;
        }
      }
}

// ---- CRT reconstruction ----------------------------------------------------------------------
// 16 residues c_l in [0, m_l) -> the integer X in (-M/2, M/2) with X = c_l mod m_l, as a double
__device__ __forceinline__ double crt_value(const int (&c)[NMOD]) {
  int v[NMOD];
  sfor<0, NMOD>([&](auto L) {
    constexpr int l = decltype(L)::value;
    constexpr int ml = kT.m[l];
    int t = c[l];
    sfor<0, l>([&](auto K) {
      constexpr int k = decltype(K)::value;
      constexpr int ik = kT.inv[k][l];
      t = ((t + ml - v[k] % ml) * ik) % ml;
    });
    v[l] = t;
  });
  unsigned __int128 X = (unsigned)v[NMOD - 1];
#pragma unroll
  for (int l = NMOD - 2; l >= 0; --l) X = X * (unsigned)kT.m[l] + (unsigned)v[l];
  const bool neg = X > (kM >> 1);
  const unsigned __int128 mag = neg ? kM - X : X;
  const uint64_t hi = (uint64_t)(mag >> 64), lo = (uint64_t)mag;
  double d;
  if (hi == 0) {
    d = (double)lo;
  } else {
    const int p = 127 - __builtin_clzll(hi);  // top bit of mag
    const uint64_t top = (uint64_t)(mag >> (p - 63));
    d = ldexp((double)top, p - 63);
  }
  return neg ? -d : d;
}

// C[i][j] (lower 64 x 64 tiles, mirrored through LDS as k_syrk_reduce) from the partials
__global__ __launch_bounds__(256) void k_crt(const uint8_t* __restrict__ P, int nsplit, int64_t pslab, int ns,
                                             const double* __restrict__ devmax, int bbits, double* __restrict__ C,
                                             int64_t ldc, int divide) {
  __shared__ double tile[64][65];
  const int L = blockIdx.x;
  int ti = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
  while (ti * (ti + 1) / 2 > L) --ti;
  const int tj = L - ti * (ti + 1) / 2;
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  const int sg = scale_exp(*devmax, bbits);
  const double dn = (double)ns;
#pragma unroll 1
  for (int q = 0; q < 16; ++q) {
    const int r = r0 + 4 * q;
    const int i = ti * 64 + r, j = tj * 64 + c;
    const bool ok = i < ns && j < ns && (ti > tj || c <= r);
    double val = 0.0;
    if (ok) {
      int cr[NMOD];
      const int64_t off = (int64_t)i * ns + j;
      sfor<0, NMOD>([&](auto Lm) {
        constexpr int l = decltype(Lm)::value;
        int s = 0;
        for (int sp = 0; sp < nsplit; ++sp) s += P[(int64_t)(l * nsplit + sp) * pslab + off];
        cr[l] = s % kT.m[l];
      });
      val = ldexp(crt_value(cr), -2 * sg);
      if (divide) val = val / dn;
      C[(int64_t)i * ldc + j] = val;
    }
    tile[r][c] = val;
  }
  __syncthreads();
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
constexpr int I8_NST = 4, I8_KSUB = 1;
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
  p.nlaunch = (int)((nkc + cmax - 1) / cmax);
  const int64_t per_launch = (nkc + p.nlaunch - 1) / p.nlaunch;
  const int nb = (ns + i8::TB - 1) / i8::TB;
  const int tiles = nb * (nb + 1) / 2;
  const int tiles8 = (tiles + 7) / 8 * 8;
  // K splits: fill 256 CUs (one workgroup each) with the least idle last round, >= 256 K steps each
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 8; ++s) {
    if (s > 1 && per_launch / s < 256) break;
    const double items = (double)tiles * i8::NMOD * s;
    const double cost = std::ceil(items / 256.0) / s + 0.01 * s;
    if (cost < best_cost - 1e-12) {
      best_cost = cost;
      best = s;
    }
  }
  p.nsplit = force_split > 0 ? (int)std::min<int64_t>(force_split, per_launch) : best;
  best = p.nsplit;
  p.kcs = (int)(((per_launch + best - 1) / best + I8_KSUB - 1) / I8_KSUB * I8_KSUB);
  p.chunks = (int64_t)p.nsplit * p.kcs;  // chunks per launch (zero-padded past rowpad)
  p.nkc = nkc;
  p.nitems = tiles8 * p.nsplit;
  p.r_bytes = (int64_t)i8::NMOD * p.chunks * ns * i8::KC;
  p.p_bytes = (int64_t)i8::NMOD * p.nsplit * ns * ns;
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

hipError_t launch_corr_i8(const double* AT, int ns, int64_t rowlen, int64_t rowpad, const double* mean,
                          const double* devmax, const CorrI8Plan& p, const int* items, int8_t* R, uint8_t* P,
                          double* C, int64_t ldc, int divide, hipStream_t st) {
  using namespace i8;
  constexpr size_t lds = (size_t)I8_NST * I8_KSUB * 2 * PANEL;
  static_assert(lds <= 160 * 1024, "LDS");
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_syrk_i8<I8_NST, I8_KSUB>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int64_t lstride = p.chunks * ns * KC;
  const int64_t pslab = (int64_t)ns * ns;
  for (int li = 0; li < p.nlaunch; ++li) {
    const int64_t kc0 = (int64_t)li * p.chunks;
    const int64_t thr = p.chunks * ns * 4;
    hipLaunchKernelGGL(k_residues, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, AT, ns, rowlen, rowpad,
                       mean, devmax, p.bbits, kc0, p.chunks, R, lstride);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_syrk_i8<I8_NST, I8_KSUB>), dim3((unsigned)(NMOD * p.nitems)), dim3(512), lds, st, R, ns,
                       lstride, p.kcs, reinterpret_cast<const int4*>(items), p.nitems, p.nsplit, P, pslab,
                       li > 0 ? 1 : 0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int nt = (ns + 63) / 64;
  hipLaunchKernelGGL(k_crt, dim3((unsigned)(nt * (nt + 1) / 2)), dim3(256), 0, st, P, p.nsplit, pslab, ns, devmax,
                     p.bbits, C, ldc, divide);
  return hipGetLastError();
}

}  // namespace pods

// gfx950 fused generator pass of the digital filter (digitalfilters.py main() :1440-1477):
// random planes -> x/y/z filter -> Lund transform -> rotation -> K-tiled snapshot store in
// one kernel.  Same numerics contract as podsgen_kernels.hip (built with -ffp-contract=off;
// bit-exact against scipy's direct correlation order and the reference's expressions).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "podsgen_kernels.h"

namespace pods {

// K-tiled snapshot layout (podsgen_kernels.hip at_off)
__device__ __forceinline__ int64_t fx_at_off(int64_t r, int64_t i, int ns) {
  return (((r >> 4) * ns + i) << 4) + (r & 15);
}

// -----------------------------------------------------------------------------------------
// Fused generator pass: x + y + z filter, Lund transform, rotation and the K-tiled snapshot
// store in ONE kernel (filter3DSciPy1D :100-140 in scipy's x -> y -> z order, adapt1d /
// adapt2prf :143-231, rotate_velocity :1119-1131), so the x-filtered planes T1 never reach
// HBM.  A workgroup owns a TJ x TK output tile and walks a chunk of steps; every thread owns
// U (component, halo point) pairs of the (TJ+NY-1) x (TK+NZ-1) halo tile and keeps their
// last NX random planes in registers (a ring: plane p sits in slot p % NX; the slot indices
// are compile-time per step phase, selected by a switch, so the ring never moves).  Per step:
//   x   t1 = sum_a R[plane i+a] * bx[NX-1-a] (a ascending, acc from 0: k_filter_x's bits),
//       while the next plane's loads are in flight (one plane ahead);
//   y   t2 over TJ rows per halo column from LDS (b ascending: k_filter_yz's bits);
//   z   out over TK columns per row (cc ascending), then Lund + rotation per point with
//       k_filter_yz's expressions, and one 128-B line per (component, row) of the tile.
// Traffic: R once from HBM (the halo overlap of neighbouring tiles is served by L2/MALL) and
// A written once -- against R + T1 written + T1 (1.75x halo) read + A for the two-pass path.
// -----------------------------------------------------------------------------------------
template <int NX, int NY, int NZ, int TJ, int TK, int NT>
struct Fxyz {
  static constexpr int HJ = TJ + NY - 1, HK = TK + NZ - 1, HP = HJ * HK;
  // pairs are dealt in 64-lane wave slots, each slot holding one component (so the plane base
  // of a slot is wave-uniform): a component's HP points take HW = ceil(HP/64) slots
  static constexpr int HW = (HP + 63) / 64;
  static constexpr int U = (3 * HW * 64 + NT - 1) / NT;  // pairs per thread
  static constexpr int YG = 4;                      // y outputs per item
  static constexpr int ZG = 2;                      // z outputs per item
  static constexpr int LDS_TAPS = (NX + NY + NZ + 1) / 2 * 2;
  static constexpr int LDS_T1 = 3 * HP;
  static constexpr int LDS_T2 = 3 * TJ * HK;
  static constexpr int LDS_Z = 3 * TJ * TK;
  static constexpr int LDS_PRM = 9 * TJ * TK;   // the tile's Lund parameters, staged once
  static constexpr int LDS_OUT = 3 * TJ * TK;   // final (u, v, w) of the step, for the stores
  // global stores per thread per step: the same count in every wave (see the store phase)
  static constexpr int NSTO = (3 * TJ * TK + NT - 1) / NT;
  static constexpr size_t lds_bytes =
      (size_t)(LDS_TAPS + LDS_T1 + LDS_T2 + LDS_Z + LDS_PRM + LDS_OUT) * sizeof(double);
};

template <int NX, int NY, int NZ, int TJ, int TK, int NT>
__global__ __launch_bounds__(NT, 1) void k_filter_xyz(
    const double* __restrict__ R, const double* __restrict__ taps, int ns, int jl, int K, int Kp,
    int64_t Sl, const double* __restrict__ lund, int64_t lund_sj, int lund_mode,
    const double* __restrict__ rot, int rotate, double* __restrict__ AT, int ntj, int ntk, int chunk) {
  using F = Fxyz<NX, NY, NZ, TJ, TK, NT>;
  constexpr int HJ = F::HJ, HK = F::HK, HP = F::HP, U = F::U, YG = F::YG, ZG = F::ZG;
  static_assert(TJ % YG == 0 && TK % ZG == 0, "tile must split into items");
  // The taps live in LDS (uniform broadcast reads): held in registers they would cost ~80
  // SGPR/VGPRs next to the NX-deep register ring.  They share the array with the stage
  // buffers, so their reads are not hoisted out of the step loop.
  extern __shared__ __attribute__((aligned(16))) double fx_sh[];
  double* tps = fx_sh;                   // bx (reversed: tps[a] = bx[NX-1-a]), by, bz (as given)
  double* t1s = fx_sh + F::LDS_TAPS;     // [3][HJ][HK]
  double* t2s = t1s + F::LDS_T1;         // [3][TJ][HK]
  double* zs = t2s + F::LDS_T2;          // [3][TJ][TK]
  double* prm = zs + F::LDS_Z;           // [9][TJ][TK]
  double* outs = prm + F::LDS_PRM;       // [3][TJ][TK]
  const int t = threadIdx.x;
  const int tile = blockIdx.x;
  const int tj = tile / ntk, tk = tile - (tile / ntk) * ntk;
  const int j0 = tj * TJ, k0 = tk * TK;  // output tile origin (slab rows, columns)
  const int i0 = blockIdx.y * chunk;
  const int i1 = min(ns, i0 + chunk);
  if (i0 >= i1) return;
  for (int e = t; e < NX + NY + NZ; e += NT) tps[e] = e < NX ? taps[NX - 1 - e] : taps[e];
  if (lund_mode >= 0) {
    const int64_t Plx = (int64_t)jl * K;
    for (int e = t; e < 9 * TJ * TK; e += NT) {
      const int q = e / (TJ * TK), pt = e - q * (TJ * TK);
      const int j = min(j0 + pt / TK, jl - 1), k = min(k0 + pt % TK, K - 1);
      prm[e] = (q < 7 || lund_mode == 1) ? lund[(int64_t)q * Plx + (int64_t)j * lund_sj + k] : 0.0;
    }
  }
  const int64_t Pl = (int64_t)jl * K;
  const int rowsp = jl + NY - 1;  // slab rows of R
  // pair u of this thread: wave slot W = wave + (NT/64) u holds component c_u = W / HW
  // (wave-uniform) and halo point pt = (W % HW) * 64 + lane at plane offset poff[u]; pairs
  // past the 3 HW slots, past HP, or outside the slab read nothing and stay 0
  constexpr int HW = F::HW;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
  // voff[u]: byte offset of the pair's point inside a plane; pairs that read nothing get an
  // offset past the buffer's range, so their raw buffer loads return 0 without a branch
  uint32_t voff[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int W = wave + (NT / 64) * u;
    const int c = W / HW;
    const int pt = (W - c * HW) * 64 + lane;
    const int hj = pt / HK, hk = pt - (pt / HK) * HK;
    const int row = j0 + hj, col = k0 + hk;
    const bool ok = c < 3 && pt < HP && row < rowsp && col < Kp;
    voff[u] = ok ? (uint32_t)(row * Kp + col) * 8u : 0xFFFFFFF0u;
  }
  const uint32_t plane_bytes = (uint32_t)(Sl * 8);
  // plane p of component c starts at stream plane sp(c, p) (main() :1361-1367, :1454-1467);
  // the buffer resource (base = that plane, range = one plane) is scalar
  auto load_plane = [&](int u, int p) -> double {
    const int W = wave + (NT / 64) * u;
    const int c = min(W / HW, 2);  // wave-uniform; slots past the components have voff out of range
    const int64_t sp = p < NX ? (int64_t)c * NX + p : (int64_t)3 * NX + 3 * (int64_t)(p - NX) + c;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(R + sp * Sl), 0, (int)plane_bytes, 0x00020000);
    const auto q = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)voff[u], 0, 0);
    return __builtin_bit_cast(double, q);
  };
  // ---- prime the ring: planes i0 .. i0+NX-2 in their slots, plane i0+NX-1 in flight ------
  double w[U][NX];
  double nxt[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int a = 0; a < NX; ++a) w[u][a] = 0.0;
  }
  for (int a = 0; a < NX - 1; ++a) {
    const int p = i0 + a;
    const int sl = p % NX;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double v = load_plane(u, p);
#pragma unroll
      for (int q = 0; q < NX; ++q)
        if (q == sl) w[u][q] = v;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) nxt[u] = load_plane(u, i0 + NX - 1);
  __syncthreads();  // taps

  for (int i = i0; i < i1; ++i) {
    // ---- x pass (phase-specialised ring indices) ------------------------------------------
    double t1[U];
    auto xstep = [&](auto PH) {
      constexpr int s = decltype(PH)::value;     // slot of plane i
      constexpr int snew = (s + NX - 1) % NX;    // slot of plane i+NX-1 (arrived in nxt)
#pragma unroll
      for (int u = 0; u < U; ++u) w[u][snew] = nxt[u];
      if (i + 1 < i1) {
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = load_plane(u, i + NX);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) t1[u] = 0.0;
#pragma unroll
      for (int a = 0; a < NX; ++a) {
        const double b = tps[a];
#pragma unroll
        for (int u = 0; u < U; ++u) t1[u] = t1[u] + w[u][(s + a) % NX] * b;
      }
    };
    switch (i % NX) {
#define PODS_XS(S_) \
  case S_:          \
    if constexpr (S_ < NX) xstep(std::integral_constant<int, S_>{}); \
    break;
      PODS_XS(0) PODS_XS(1) PODS_XS(2) PODS_XS(3) PODS_XS(4) PODS_XS(5) PODS_XS(6) PODS_XS(7)
      PODS_XS(8) PODS_XS(9) PODS_XS(10) PODS_XS(11) PODS_XS(12) PODS_XS(13) PODS_XS(14) PODS_XS(15)
      PODS_XS(16) PODS_XS(17) PODS_XS(18) PODS_XS(19) PODS_XS(20) PODS_XS(21) PODS_XS(22) PODS_XS(23)
      PODS_XS(24)
#undef PODS_XS
      default: break;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int W = wave + (NT / 64) * u;
      const int c = W / HW;
      const int pt = (W - c * HW) * 64 + lane;
      if (c < 3 && pt < HP) t1s[c * HP + pt] = t1[u];
    }
    __syncthreads();  // B1: t1 complete
    // ---- y pass: items (component, halo column, group of YG rows) ---------------------------
    for (int it = t; it < 3 * (TJ / YG) * HK; it += NT) {
      const int hk = it % HK;
      const int rest = it / HK;
      const int g = rest % (TJ / YG), c = rest / (TJ / YG);
      const double* col = t1s + (c * HJ + g * YG) * HK + hk;
      double v[YG + NY - 1];
#pragma unroll
      for (int r = 0; r < YG + NY - 1; ++r) v[r] = col[r * HK];
      double acc[YG];
#pragma unroll
      for (int jj = 0; jj < YG; ++jj) acc[jj] = 0.0;
#pragma unroll
      for (int b = 0; b < NY; ++b) {
        const double tb = tps[NX + NY - 1 - b];
#pragma unroll
        for (int jj = 0; jj < YG; ++jj) acc[jj] = acc[jj] + v[jj + b] * tb;
      }
#pragma unroll
      for (int jj = 0; jj < YG; ++jj) t2s[(c * TJ + g * YG + jj) * HK + hk] = acc[jj];
    }
    __syncthreads();  // B2: t2 complete
    // ---- z pass: items (component, row, group of ZG columns) -------------------------------
    for (int it = t; it < 3 * TJ * (TK / ZG); it += NT) {
      const int kg = it % (TK / ZG);
      const int rest = it / (TK / ZG);
      const int jj = rest % TJ, c = rest / TJ;
      const double* rowp = t2s + (c * TJ + jj) * HK + kg * ZG;
      double v[ZG + NZ - 1];
#pragma unroll
      for (int e = 0; e < ZG + NZ - 1; ++e) v[e] = rowp[e];
      double acc[ZG];
#pragma unroll
      for (int kk = 0; kk < ZG; ++kk) acc[kk] = 0.0;
#pragma unroll
      for (int cc = 0; cc < NZ; ++cc) {
        const double tb = tps[NX + NY + NZ - 1 - cc];
#pragma unroll
        for (int kk = 0; kk < ZG; ++kk) acc[kk] = acc[kk] + v[kk + cc] * tb;
      }
#pragma unroll
      for (int kk = 0; kk < ZG; ++kk) zs[(c * TJ + jj) * TK + kg * ZG + kk] = acc[kk];
    }
    __syncthreads();  // B3: z outputs complete; t1s / t2s free for the next step
    // ---- Lund + rotation: one thread per tile point, results to LDS --------------------------
    // (rot is re-materialised per step so its scalar loads stay in the loop)
    int zero = 0;
    asm volatile("" : "+s"(zero));
    const double* rot_i = rot + zero;
    for (int pt = t; pt < TJ * TK; pt += NT) {
      const double xu = zs[0 * TJ * TK + pt];
      const double xv = zs[1 * TJ * TK + pt];
      const double xw = zs[2 * TJ * TK + pt];
      double u = xu, v = xv, ww = xw;
      if (lund_mode >= 0) {  // (lund_mode < 0: the raw filter output, no rotation, as k_filter_yz)
        const double* L = prm + pt;
        constexpr int Q = TJ * TK;
        const double a00 = L[0], a10 = L[Q], a11 = L[2 * Q];
        const double a20 = L[3 * Q], a21 = L[4 * Q], a22 = L[5 * Q];
        // digitalfilters.py:174-176 (adapt1d) / :227-229 (adapt2prf), left to right, zero terms kept
        u = ((a00 * xu + 0.0 * xv) + 0.0 * xw) + L[6 * Q];
        v = (a10 * xu + a11 * xv) + 0.0 * xw;
        ww = (a20 * xu + a21 * xv) + a22 * xw;
        if (lund_mode == 1) {
          v = v + L[7 * Q];
          ww = ww + L[8 * Q];
        }
        if (rotate) {  // rotate_velocity :1119-1131, OpenBLAS dgemv order (k_filter_yz)
          const double ur = __builtin_fma(rot_i[2], ww, __builtin_fma(rot_i[0], u, rot_i[1] * v));
          const double vr = __builtin_fma(rot_i[5], ww, __builtin_fma(rot_i[3], u, rot_i[4] * v));
          const double wr = __builtin_fma(rot_i[8], ww, __builtin_fma(rot_i[6], u, rot_i[7] * v));
          u = ur;
          v = vr;
          ww = wr;
        }
      }
      outs[0 * TJ * TK + pt] = u;
      outs[1 * TJ * TK + pt] = v;
      outs[2 * TJ * TK + pt] = ww;
    }
    __syncthreads();  // B4: the step's outputs complete
    // ---- stores: NSTO unconditional stores per thread in EVERY wave --------------------------
    // Element e = (component, point) of the tile; slots past the tile or points outside the
    // inlet are clamped to a valid point of the tile and rewrite that point's own value
    // (identical bytes).  Every wave thus issues the same number of vector-memory stores, so
    // the wait for the next step's prefetched R planes (issued before these stores) can be a
    // fixed vmcnt(NSTO) instead of a drain that waits for the stores.
#pragma unroll
    for (int m = 0; m < F::NSTO; ++m) {
      int e = t + NT * m;
      e = e < 3 * TJ * TK ? e : 3 * TJ * TK - 1;
      const int c = e / (TJ * TK), pt = e - c * (TJ * TK);
      const int j = min(j0 + pt / TK, jl - 1), k = min(k0 + pt % TK, K - 1);
      const double val = outs[c * TJ * TK + (j - j0) * TK + (k - k0)];
      AT[fx_at_off((int64_t)c * Pl + (int64_t)j * K + k, i, ns)] = val;
    }
  }
}

// Fused x+y+z pass (k_filter_xyz) for the filter widths it is instantiated for; returns
// hipErrorNotSupported otherwise (the caller then runs k_filter_x2 + k_filter_yz).
template <int NX, int NY, int NZ, int TJ, int TK, int NT>
static hipError_t launch_fxyz_t(const double* R, const double* taps, int ns, int jl, int K, int Kp, int64_t Sl,
                                const double* lund, int64_t lund_sj, int lund_mode, const double* rot,
                                int rotate, double* AT, int cus, hipStream_t st) {
  using F = Fxyz<NX, NY, NZ, TJ, TK, NT>;
  const int ntj = (jl + TJ - 1) / TJ, ntk = (K + TK - 1) / TK;
  const int tiles = ntj * ntk;
  // step chunks: fill the CUs (one workgroup each), each chunk >= 4 NX steps so the ring's
  // priming (NX-1 planes) stays a small overhead
  int nch = std::max(1, (cus + tiles - 1) / tiles);
  nch = std::max(1, std::min(nch, ns / (4 * NX)));
  const int chunk = (ns + nch - 1) / nch;
  nch = (ns + chunk - 1) / chunk;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_filter_xyz<NX, NY, NZ, TJ, TK, NT>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)F::lds_bytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_filter_xyz<NX, NY, NZ, TJ, TK, NT>), dim3(tiles, nch), dim3(NT), F::lds_bytes, st, R, taps,
                     ns, jl, K, Kp, Sl, lund, lund_sj, lund_mode, rot, rotate, AT, ntj, ntk, chunk);
  return hipGetLastError();
}

bool filter_xyz_supported(int NX, int NY, int NZ) { return NX == 13 && NY == 13 && NZ == 13; }

hipError_t launch_filter_xyz(int NX, int NY, int NZ, const double* R, const double* taps, int ns, int jl, int K,
                             int Kp, int64_t Sl, const double* lund, int64_t lund_sj, int lund_mode,
                             const double* rot, int rotate, double* AT, int cus, hipStream_t st) {
  if (NX == 13 && NY == 13 && NZ == 13)
    return launch_fxyz_t<13, 13, 13, 16, 16, 512>(R, taps, ns, jl, K, Kp, Sl, lund, lund_sj, lund_mode, rot, rotate,
                                                  AT, cus, st);
  return hipErrorNotSupported;
}

}  // namespace pods

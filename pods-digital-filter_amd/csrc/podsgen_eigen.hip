// gfx950 symmetric eigensolver for the POD correlation matrix (PODFS.py:1309-1310:
// `linalg.eig(C)` + `sort_eigenvalues`): all n eigenvalues and the eigenvectors of the
// nvec largest.
//
//   k_trd      Householder tridiagonalisation (LAPACK dsytd2 'L' arithmetic) as a few
//              persistent launches (one per 512-column range).  The live matrix stays on
//              chip: workgroup g (one per CU) owns rows g, g+G, ... ; lane t of its 512
//              threads owns columns t, t+512, ... of those rows, held in VGPRs and LDS (plus,
//              for the first range at n > 2048, an L2-resident slab).  Per column j there is ONE cross-CU
//              hand-off: every workgroup publishes p = A v for its rows plus (owner only) the
//              updated row j+1, and every workgroup then recomputes the rank-2 update vector w,
//              the next column and its Householder vector redundantly from those two vectors,
//              so no second exchange (norm, dot) is needed.
//   k_bisect   all eigenvalues of T by Sturm-count multisection (16 lanes per eigenvalue).
//   k_twisted  eigenvectors of T for the wanted eigenvalues by twisted factorisation (dlar1v).
//   k_orth     modified Gram-Schmidt inside eigenvalue clusters (dstein's ORTOL rule).
//   k_larft / k_bt_*  back-transformation Y = Q Z with compact-WY blocks of 64 reflectors.
//
// FMA is requested explicitly (the file is built with -ffp-contract=off like the others).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <mutex>
#include <vector>

#include <algorithm>
#include <cfloat>
#include <cstdint>

#include "podsgen_kernels.h"

namespace pods {
namespace eig {

constexpr int TT = 512;  // k_trd workgroup: 8 waves


// ---- cross-CU hand-off primitives (MI355X_MICROARCH.md "Valid forms": sc1 payload stores,
// ---- drained, one sc1 flag per workgroup; sc1 poll; sc1 payload loads) ------------------
__device__ __forceinline__ double ld_sc1(const double* p) {
  const unsigned long long u = __hip_atomic_load(
      const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(p)),
      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_flag(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// DPP row reduction: afterwards every lane of each 16-lane row holds the row sum (the same
// bits in all 16 lanes: each step adds a pair in both orders, a+b == b+a).
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_mov<0x141>(x);  // row_half_mirror
  x += dpp_mov<0x140>(x);  // row_mirror
  return x;
}
// gfx950 cross-row swaps: permlane32_swap(a, b) -> a = {a.lo32, b.lo32}, b = {a.hi32, b.hi32};
// permlane16_swap(a, b) -> a = {a.r0, b.r0, a.r2, b.r2}, b = {a.r1, b.r1, a.r3, b.r3}.
__device__ __forceinline__ void pl32_swap(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void pl16_swap(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
// Wave sum, the same bits in every lane (exec must be full).
__device__ __forceinline__ double wave_sum(double x) {
  double y = x;
  pl32_swap(x, y);
  x = x + y;
  y = x;
  pl16_swap(x, y);
  x = x + y;
  return row16_sum(x);
}

// Workgroup sum in a fixed order; `red` alternates between two 8-double slots per call so
// no trailing barrier is needed.
template <int NW>
__device__ __forceinline__ double block_sum(double x, double* red) {
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int k = 1; k < NW; ++k) s += red[k];
  return s;
}

// A wave-uniform double (moved to SGPRs by readfirstlane).
__device__ __forceinline__ double uniform(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Reduce-scatter of RH (1, 2 or 4) per-lane values over the wave: afterwards lane row q
// (lanes 16q..16q+15) holds the wave sum of value q*RH/4 (RH = 4: value q; RH = 2: value q/2).
template <int RH>
__device__ __forceinline__ double rows_wave_sum(double (&a)[RH]) {
  double s;
  if constexpr (RH == 4) {
    double a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
    pl32_swap(a0, a2);
    pl32_swap(a1, a3);
    double s0 = a0 + a2, s1 = a1 + a3;
    pl16_swap(s0, s1);
    s = s0 + s1;
  } else if constexpr (RH == 2) {
    double a0 = a[0], a1 = a[1];
    pl32_swap(a0, a1);
    double s0 = a0 + a1, s1 = s0;
    pl16_swap(s0, s1);
    s = s0 + s1;
  } else {
    s = a[0];
    double y = s;
    pl32_swap(s, y);
    s = s + y;
    y = s;
    pl16_swap(s, y);
    s = s + y;
  }
  return row16_sum(s);
}

template <int S>
__device__ __forceinline__ double pick(const double (&v)[S], int m) {
  double r = 0.0;
#pragma unroll
  for (int k = 0; k < S; ++k)
    if (k == m) r = v[k];
  return r;
}

// dst[i] = the lane-held vector v at row r = g + G i of this workgroup, i in [I0, R) (lane r % 512,
// slot r / 512 holds it; k_trd's layout).  G = 256 (TT / 2): lane g has rows of even i at slot
// i / 2, lane g + 256 those of odd i -- compile-time registers, two lanes store.
template <int R, int S, int I0>
__device__ __forceinline__ void share_rows(double* dst, const double (&v)[S], int g, int G, int t, int n) {
  constexpr int TT_ = 512;
  if (G == TT_ / 2) {
    if (t == g) {
#pragma unroll
      for (int i = (I0 + 1) & ~1; i < R; i += 2)
        if (g + G * i < n) dst[i] = v[i >> 1];
    } else if (t == g + TT_ / 2) {
#pragma unroll
      for (int i = I0 | 1; i < R; i += 2)
        if (g + G * i < n) dst[i] = v[i >> 1];
    }
    return;
  }
#pragma unroll
  for (int i = I0; i < R; ++i) {
    const int r = g + G * i;
    if (r < n && (r & (TT_ - 1)) == t) dst[i] = pick(v, r / TT_);
  }
}

// ---- tagged 8-byte hand-off values: the two lowest mantissa bits carry the column parity
// ---- tag (j mod 4).  One 8-B sc1 store publishes value and tag together; the consumer
// ---- spins on its own loads until the tag matches -- no flag, no producer drain, one hop.
// ---- A stale entry of the same (parity) buffer is always two columns old, so two bits
// ---- suffice; the value perturbation is <= 3 ulp, below dsytd2's own rounding per step.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc8(const double* base, int n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, n * 8, 0x00020000);
}
__device__ __forceinline__ double gld(__amdgpu_buffer_rsrc_t r, int idx) {
  // volatile (bit 31) + sc1 (bit 4): re-read every spin, served by L2 but never by L1
  const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, (1u << 31) | 16u);
  return __builtin_bit_cast(double, q);
}
__device__ __forceinline__ double tagged(double v, uint32_t tag) {
  const long long b = (__double_as_longlong(v) & ~3ll) | (long long)(tag & 3u);
  return __longlong_as_double(b);
}
__device__ __forceinline__ bool tag_ok(double v, uint32_t tag) {
  return ((uint32_t)__double2loint(v) & 3u) == (tag & 3u);
}
// the value a consumer uses: tag bits cleared, so a published 0.0 stays exactly 0.0 (not a
// denormal) and every workgroup still sees identical bits
__device__ __forceinline__ double untag(double v) {
  return __longlong_as_double(__double_as_longlong(v) & ~3ll);
}
__device__ __forceinline__ void gst(__amdgpu_buffer_rsrc_t r, int idx, double v, uint32_t tag) {
  const double t = tagged(v, tag);
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), t),
                                        r, idx * 8, 0, 16u);
}

constexpr int SPIN_LIMIT = 1 << 20;  // ~1 s of polling before a workgroup raises the abort word
// The hand-off vectors are published in NREP copies, one per XCD: every consumer polls the copy
// of its own XCD, so no line is requested by more than the 32 workgroups of one XCD.
constexpr int NREP = 8;
__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 15;
}
// buffer (p or column) for replica r, column parity q; hs doubles each (TRD_HANDOFF at most)
__device__ __forceinline__ double* hbuf(double* base, int r, int q, int hs) {
  return base + ((int64_t)r * 2 + q) * hs;
}
// Lane-major hand-off layout (r6): the granule of row/column c sits at (c % 512) S + c / 512, so a
// consumer lane's S slots (columns t + 512 m) are S contiguous granules -- 16-B loads of slot pairs,
// a wave's loads one contiguous 8 S x 64-byte run -- and a workgroup's 16 rows (g + 256 i with
// G = 256) land in two runs of 8 contiguous granules per vector and copy, instead of 16 granules
// 2 KB apart.
template <int S>
__device__ __forceinline__ int hslot(int c) {
  return (c & 511) * S + (c >> 9);
}
__device__ __forceinline__ void gld2(__amdgpu_buffer_rsrc_t r, int idx, double& a, double& b) {
  // volatile (bit 31) + sc1 (bit 4), like gld: two granules (16-B aligned: idx even)
  const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, idx * 8, 0, (1u << 31) | 16u);
  typedef double d2 __attribute__((ext_vector_type(2)));
  const d2 v = __builtin_bit_cast(d2, q);
  a = v.x;
  b = v.y;
}

// -----------------------------------------------------------------------------------------
// k_trd<R, S, K, SG, SL>: one column range of the tridiagonalisation.
//
// Workgroup g (of G <= 256) owns rows r = g + G*i (i < R); lane t owns columns c = t + 512*m
// (m < S).  The column loop is cut into S ranges: range K runs columns j in
// [512K-1, 512(K+1)-1) (K = 0 starts at 0).  Throughout range K the slots m < K and the rows
// i < 2K hold nothing live (every such row/column index is <= j), so each range is its own
// launch that keeps only rows [2K, R) x slots [K, S) on chip -- the storage shrinks as the
// matrix does, and each launch is a single-exit loop with compile-time slot/row bounds.
// Between launches the live block is parked in the per-workgroup slab Wm[g][m][i][t]; the
// pending reflector v_{j-1} is re-read from V and tau from the tau array.
// Storage inside a launch: slots [K, K+SG) stay in Wm (L2-resident), the next SL slots in
// LDS, the rest in VGPRs.
// H = 1 (r6, with K = 0): the second half of range 0, columns [256, 511), run as a launch of its
// own: there row slot i = 0 (rows g < 256) and the lanes t < 256 of slot 0 hold nothing live any
// more, so the 15 live rows' slot 0 fits in LDS beside the SL = 2 slots (lanes 256..511 only,
// "Ah") and the L2 slab slot of the first half (H = 0: columns [0, 256)) is gone.
//
// Column j (dsytd2 'L'): every workgroup reads p_{j-1} = A^{(j-1)} v_{j-1} and column j of
// A^{(j-1)} (both published in column j-1 as tagged granules by the owners of the rows),
// recomputes w_{j-1}, column j of A^{(j)} and the reflector v_j redundantly (two workgroup
// reductions), applies the pending rank-2 update to its rows fused with p_j = A^{(j)} v_j,
// and publishes p_j and column j+1 of its rows.  Three workgroup barriers, one cross-CU hop.
// -----------------------------------------------------------------------------------------
template <int R, int S, int K, int SG, int SL, int H = 0>
__global__ __launch_bounds__(TT, 1) void k_trd(TrdArgs a) {
  static_assert(H == 0 || (K == 0 && SG == 0 && R == 16), "the half launch splits range 0 of the 16-row plan");
  constexpr int I0 = H ? 1 : ((2 * K < R) ? 2 * K : R);  // first live row slot
  constexpr int RL = R - I0;                    // live rows
  constexpr int SGH = SG + H;                   // slots before the LDS ones: slab (SG) or half (H)
  constexpr int SR = S - K - SGH - SL;          // register slots
  constexpr int HS = TT * S;                    // doubles per hand-off buffer (<= TRD_HANDOFF)
  static_assert(HS <= TRD_HANDOFF, "hand-off buffer");
  static_assert(SR >= 0 && RL > 0, "bad trd range configuration");
  extern __shared__ double lds[];
  double* Al = lds;                  // [SL][RL][TT]
  double* Ah = lds + SL * RL * TT;   // H: [RL][256] slot K's lanes 256..511
  double* red = Ah + H * RL * 256;   // 2 x 8 reduction slots
  double* bc = red + 16;             // 4: alpha0 (double-buffered by column parity)
  double* rsv0 = bc + 4;             // 2 x R: v_{j-1}[r_i]   (double-buffered by column parity:
  double* rsw0 = rsv0 + 2 * R;       // 2 x R: w_{j-1}[r_i]    the update reads them after B3)
  double* rr = rsw0 + 2 * R;         // (R + 2) x 8 wave partials (rows, then the two dots)
  double* rcol = rr + 8 * (R + 2);   // R: column j+1 of A^{(j)} at this workgroup's rows
  const int t0 = threadIdx.x, wv = t0 >> 6;
  const int g0 = blockIdx.x, G = a.G, n = a.n;
  if (g0 >= n) return;
  const int lastrow = g0 + G * ((n - 1 - g0) / G);
  double* Wg = a.Wm + (int64_t)g0 * S * R * TT;  // this workgroup's slab
  auto wm = [&](int m, int i, int t) -> double& { return Wg[((int64_t)m * R + i) * TT + t]; };
  double Ar[RL][SR > 0 ? SR : 1];
  uint32_t* abortw = a.flags;

  // Ranges K > klast = (n-1)/512 hold no column and are not launched; klast runs the tail.
  const bool last = K == a.klast;
  const int jend = min(lastrow + 1, n - 1);
  // the 16-row plan runs range 0 as two halves: [0, 256) with the slab slot, [256, 511) with
  // slot 0 in LDS (H); every other plan runs [0, 511)
  constexpr bool SPLIT0 = K == 0 && R == 16;
  const int jb = K == 0 ? (H ? TT / 2 : 0) : TT * K - 1;
  const int je = last ? jend : min(jend, (SPLIT0 && !H) ? TT / 2 : TT * (K + 1) - 1);

  // ---- load the live block -----------------------------------------------------------------
#pragma unroll
  for (int ii = 0; ii < RL; ++ii) {
    const int i = I0 + ii;
    const int r = g0 + G * i;
#pragma unroll
    for (int m = K; m < S; ++m) {
      const int c = t0 + TT * m;
      double v;
      if (K == 0 && !H)
        v = (r < n && c < n) ? a.C[(int64_t)r * a.ldc + c] : 0.0;
      else
        v = wm(m, i, t0);
      if (m < K + SGH) {
        if (H) {
          if (t0 >= TT / 2) Ah[ii * (TT / 2) + t0 - TT / 2] = v;
        } else if (K == 0) {
          wm(m, i, t0) = v;
        }
      } else if (m < K + SGH + SL) {
        Al[((m - K - SGH) * RL + ii) * TT + t0] = v;
      } else {
        Ar[ii][m - K - SGH - SL] = v;
      }
    }
  }
  double vp[S];
  double tau_p = 0.0;
#pragma unroll
  for (int m = 0; m < S; ++m) {
    const int c = t0 + TT * m;
    vp[m] = (jb > 0 && c < n) ? a.V[(int64_t)(jb - 1) * a.ldv + c] : 0.0;
  }
  if (jb > 0) tau_p = a.tau[jb - 1];
  int rk = 0;

  const int xrep = xcc_id() % a.nrep;
  int64_t* trace = (a.trace && (g0 == a.trace_wg || a.trace_wg < 0) && t0 == 0)
                       ? a.trace + (a.trace_wg < 0 ? (int64_t)g0 * n * 8 : 0)
                       : nullptr;
  for (int j = jb; j < je; ++j) {
#ifdef PODS_TRD_DRAIN  // diagnostic variant builds only (tools/lib_variants.sh): the wave's stores done first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if (trace) trace[j * 8 + 0] = (int64_t)__builtin_amdgcn_s_memrealtime();
    // Re-materialise the lane/workgroup indices every column: without this the compiler
    // hoists ~100 loop-invariant addresses and masks out of the column loop and spills.
    int t = t0, g = g0;
    asm volatile("" : "+v"(t));
    asm volatile("" : "+s"(g));
    const int lane = t & 63;
    double* rsv = rsv0 + (j & 1) * R;
    double* rsw = rsw0 + (j & 1) * R;
    // ---- inputs: p_{j-1} (p), column j of A^{(j-1)} (x), p_{j-1}[j] -----------------------
    double p[S], x[S], pj = 0.0;
    int nspin = 0;
    if (j == 0) {
#pragma unroll
      for (int m = 0; m < S; ++m) {
        const int c = t + TT * m;
        p[m] = 0.0;
        x[m] = c < n ? a.C[c] : 0.0;
      }
    } else {
      const __amdgpu_buffer_rsrc_t rp = rsrc8(hbuf(a.pbuf, xrep, (j - 1) & 1, HS), HS);
      const __amdgpu_buffer_rsrc_t rc = rsrc8(hbuf(a.rbuf, xrep, (j - 1) & 1, HS), HS);
      const uint32_t want = (uint32_t)j;
      // Every spin re-reads all of this lane's live granules (simple straight-line code keeps the
      // register allocation flat); the wave leaves when all its lanes saw the tag.  Slots below
      // ML hold only columns < j (slot K-1 reaches j = 512K-1 only in the range's first column):
      // no loads for them; a granule whose column is dead or past n is loaded with its pair but
      // not checked (nothing publishes it any more).
      constexpr int PW = (S % 2 == 0) ? 2 : 1;
      constexpr int ML = (K == 0 ? 0 : K - 1) / PW * PW;
      const int lj = hslot<S>(j);
      for (int spin = 0;; ++spin) {
        bool ok = true;
#pragma unroll
        for (int m = 0; m < ML; ++m) {
          p[m] = 0.0;
          x[m] = 0.0;
        }
#pragma unroll
        for (int m = ML; m < S; m += PW) {
          double q1[PW], q2[PW];
          if constexpr (PW == 2) {
            gld2(rp, t * S + m, q1[0], q1[1]);
            gld2(rc, t * S + m, q2[0], q2[1]);
          } else {
            q1[0] = gld(rp, t * S + m);
            q2[0] = gld(rc, t * S + m);
          }
#pragma unroll
          for (int u = 0; u < PW; ++u) {
            const int c = t + TT * (m + u);
            const bool in = c >= j && c < n;
            ok = ok && (!in || (tag_ok(q1[u], want) && tag_ok(q2[u], want)));
            p[m + u] = in ? untag(q1[u]) : 0.0;
            x[m + u] = in ? untag(q2[u]) : 0.0;
          }
        }
        const double qj = gld(rp, lj);
        ok = ok && tag_ok(qj, want);
        pj = untag(qj);
        nspin = spin;
        if (__all(ok)) break;
        if ((spin & 1023) == 1023) {
          if (ld_flag(abortw) != 0) break;
          if (spin > SPIN_LIMIT) {
            st_flag(abortw, 1u);
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (trace) trace[j * 8 + 1] = (int64_t)__builtin_amdgcn_s_memrealtime() | ((int64_t)nspin << 48);
    // ---- w = tau p ; alpha = -tau/2 (w . v) ; w += alpha v  (dsytd2) -------------------
    double dot = 0.0;
#pragma unroll
    for (int m = 0; m < S; ++m) {
      p[m] = tau_p * p[m];
      dot = __builtin_fma(p[m], vp[m], dot);
    }
    // v_{j-1} at this workgroup's rows, for the lanes that hold them (row r sits in lane r % 512,
    // slot r / 512); with G = 256 workgroups (n > 4080) row g + 256 i is in lane g (i even) or
    // g + 256 (i odd), slot i / 2 -- a register known at compile time, so only those two lanes
    // store and nothing is selected (the general loop picks the slot with 2 S v_cndmasks per row
    // in every lane: ~0.5 us per column at range 0, r6 trace)
    share_rows<R, S, I0>(rsv, vp, g, G, t, n);
    dot = block_sum<TT / 64>(dot, red + 8 * (rk++ & 1));                       // B1
    if (trace) trace[j * 8 + 2] = (int64_t)__builtin_amdgcn_s_memrealtime();
    const double alpha = -0.5 * tau_p * dot;
    // p now holds w_{j-1} (in place)
#pragma unroll
    for (int m = 0; m < S; ++m) p[m] = __builtin_fma(alpha, vp[m], p[m]);
    const double vj = j >= 1 ? 1.0 : 0.0;  // v_{j-1}[j] (the reflector's unit entry)
    const double wj = __builtin_fma(alpha, vj, tau_p * pj);
    // ---- column j of A^{(j)} -------------------------------------------------------------
#pragma unroll
    for (int m = 0; m < S; ++m) {
      const int c = t + TT * m;
      x[m] = (c >= j && c < n) ? __builtin_fma(-p[m], vj, __builtin_fma(-vp[m], wj, x[m])) : 0.0;
    }
    if (t == ((j + 1) & (TT - 1))) bc[(j & 1) * 2] = pick(x, (j + 1) / TT);
    share_rows<R, S, I0>(rsw, p, g, G, t, n);                                      // w_{j-1} likewise
    double ss = 0.0;
#pragma unroll
    for (int m = 0; m < S; ++m) {
      const int c = t + TT * m;
      if (c >= j + 2 && c < n) ss = __builtin_fma(x[m], x[m], ss);
    }
    ss = block_sum<TT / 64>(ss, red + 8 * (rk++ & 1));                          // B2
    if (trace) trace[j * 8 + 3] = (int64_t)__builtin_amdgcn_s_memrealtime();
    // ---- Householder reflector of x = A^{(j)}[j+1:, j] (dlarfg) --------------------------
    const double alpha0 = bc[(j & 1) * 2];
    double tau_j = 0.0, beta = alpha0, scal = 0.0;
    if (ss != 0.0) {
      beta = -copysign(sqrt(__builtin_fma(alpha0, alpha0, ss)), alpha0);
      tau_j = (beta - alpha0) / beta;
      scal = 1.0 / (alpha0 - beta);
    }
    const bool writer = g == j % G;
    if (writer && t == (j & (TT - 1))) a.D[j] = pick(x, j / TT);
#pragma unroll
    for (int m = 0; m < S; ++m) {
      const int c = t + TT * m;
      x[m] = (c == j + 1) ? 1.0 : ((c >= j + 2 && c < n) ? x[m] * scal : 0.0);
    }
    // ---- p_j = A^{(j)} v_j from the stored A^{(j-1)} (dlatrd's correction):
    // ----   p_j = A^{(j-1)} v_j - v_{j-1} (w_{j-1} . v_j) - w_{j-1} (v_{j-1} . v_j)
    // ---- so the hand-off needs only a read of the stored rows; the rank-2 update of step
    // ---- j-1 is applied after the publish, overlapping the next column's hop.
    if (trace) trace[j * 8 + 4] = (int64_t)__builtin_amdgcn_s_memrealtime();
    const __amdgpu_buffer_rsrc_t pw = rsrc8(hbuf(a.pbuf, 0, j & 1, HS), 2 * NREP * HS);
    const __amdgpu_buffer_rsrc_t cw = rsrc8(hbuf(a.rbuf, 0, j & 1, HS), 2 * NREP * HS);
    const uint32_t tag = (uint32_t)(j + 1);
    const bool pubcol = t == ((j + 1) & (TT - 1));
    // rows per reduction group; H (15 rows): groups of 4, the last one padded with a zero row
    constexpr int RH = (SG > 0) ? 2 : ((RL % 4 == 0 || H) ? 4 : ((RL % 2 == 0) ? 2 : 1));
    constexpr int NG = (RL + RH - 1) / RH;
    {
      double dd[2] = {0.0, 0.0};
#pragma unroll
      for (int m = 0; m < S; ++m) {
        dd[0] = __builtin_fma(p[m], x[m], dd[0]);   // w_{j-1} . v_j
        dd[1] = __builtin_fma(vp[m], x[m], dd[1]);  // v_{j-1} . v_j
      }
      const double sd = rows_wave_sum(dd);          // rows 0,1: dd[0]; rows 2,3: dd[1]
      if (lane == 0) rr[R * 8 + wv] = sd;
      if (lane == 32) rr[(R + 1) * 8 + wv] = sd;
    }
    // The lane holding column j+1 also publishes column j+1 of A^{(j)} (stored value minus
    // the pending rank-2 update) for its rows, from the values the symv loop just read.
    // (j+1 always lies in slot K during range K.)
    // Slab slots (L2-resident, SG > 0) are only read here, like the on-chip slots (A^{(j-1)}
    // plus the dlatrd corrections above); their rank-2 update joins the others after the
    // publish, where it overlaps the next column's hop.  (Updating them here mixed stores
    // into the loads, and a pending store makes every load wait a full vmcnt drain: one L2
    // round trip per row group on the critical path.)
    // (Skipping the dead part of slot K -- this wave's columns 512K + 64 wv .. + 63 once all are
    // below j, exact since x and the pending update's multipliers are zero there -- was
    // bit-identical and slower, r4: the wave-uniform branches raised range 0's spills 47 -> 83
    // VGPRs and pods_syev 36.8 -> 39.9 ms; ranges 1-7 only: 37.0 ms.)
    // slab loads run SPF row groups ahead
    constexpr int SPF = K == 0 ? 0 : 3;  // range 0: no registers to spare (depth 2 measured no faster)
    double slab[SG > 0 ? RL : 1][SG > 0 ? SG : 1];
    // slab slots (L2): a wave whose 64 columns of slot m all lie below j holds nothing live
    // there any more (x, p and v_{j-1} are zero on them), so its slab loads and stores go out of
    // the buffer's range (a buffer load then returns 0 and a store is dropped, with no memory
    // access and no branch) -- exact, and range 0 moves half its slab traffic on average
    const __amdgpu_buffer_rsrc_t rwm = __builtin_amdgcn_make_buffer_rsrc(Wg, 0, S * R * TT * 8, 0x00020000);
    // per slot: the lane's byte offset (out of range when dead) in a VGPR, the (slot, row) part
    // as the instruction's scalar offset
    int soff[SG > 0 ? SG : 1];
#pragma unroll
    for (int m = 0; m < (SG > 0 ? SG : 1); ++m) soff[m] = TT * (K + m) + 64 * wv + 63 < j ? 0x40000000 : t * 8;
    auto slab_ld = [&](int m, int i) -> double {
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rwm, soff[m - K], (m * R + i) * TT * 8, 0));
    };
#pragma unroll
    for (int ii = 0; ii < (SG > 0 ? SPF * RH : 0); ++ii)
#pragma unroll
      for (int m = K; m < K + SG; ++m) slab[ii][m - K] = slab_ld(m, I0 + ii);
#pragma unroll
    for (int h = 0; h < NG; ++h) {
#pragma unroll
      for (int ii = (h + SPF) * RH; ii < (SG > 0 ? (h + SPF + 1) * RH : 0); ++ii)
        if (ii < RL)
#pragma unroll
          for (int m = K; m < K + SG; ++m) slab[ii][m - K] = slab_ld(m, I0 + ii);
      double acc[RH], colv[RH];
#pragma unroll
      for (int q = 0; q < RH; ++q) acc[q] = 0.0;
#pragma unroll
      for (int m = K; m < S; ++m) {
#pragma unroll
        for (int q = 0; q < RH; ++q) {
          const int ii = h * RH + q;
          if (ii >= RL) {  // H: the zero row padding the last group
            if (m == K) colv[q] = 0.0;
            continue;
          }
          double val;
          if (m < K + SGH) {
            if constexpr (H) {  // lanes < 256 hold nothing live in slot K (their columns are < j)
              const double hv = Ah[ii * (TT / 2) + (t & (TT / 2 - 1))];
              val = t >= TT / 2 ? hv : 0.0;
            } else {
              val = slab[ii][m - K];
            }
          } else if (m < K + SGH + SL) {
            val = Al[((m - K - SGH) * RL + ii) * TT + t];
          } else {
            val = Ar[ii][m - K - SGH - SL];
          }
          acc[q] = __builtin_fma(val, x[m], acc[q]);
          if (m == K) colv[q] = val;
        }
      }
      if (pubcol) {
#pragma unroll
        for (int q = 0; q < RH; ++q) {
          const int i = I0 + h * RH + q;
          if (i < R) rcol[i] = __builtin_fma(-rsv[i], p[K], __builtin_fma(-rsw[i], vp[K], colv[q]));
        }
      }
      const double sum = rows_wave_sum(acc);
      const int ir = I0 + h * RH + lane / (64 / RH);
      if ((lane & (64 / RH - 1)) == 0 && ir < R) rr[ir * 8 + wv] = sum;
    }
    if (trace) trace[j * 8 + 5] = (int64_t)__builtin_amdgcn_s_memrealtime();
    __syncthreads();                                                               // B3
    if (trace) trace[j * 8 + 6] = (int64_t)__builtin_amdgcn_s_memrealtime();
    // publish p_j and column j+1 for this workgroup's rows, one (row, XCD copy) per thread
    if (t < R * a.nrep) {
      const int i = t % R, rep_ = t / R;
      const int r = g + G * i;
      if (i >= I0 && r >= j + 1 && r < n) {
        double sum = rr[i * 8], d1 = rr[R * 8], d2 = rr[(R + 1) * 8];
#pragma unroll
        for (int q = 1; q < 8; ++q) {
          sum += rr[i * 8 + q];
          d1 += rr[R * 8 + q];
          d2 += rr[(R + 1) * 8 + q];
        }
        gst(pw, rep_ * 2 * HS + hslot<S>(r), __builtin_fma(-rsw[i], d2, __builtin_fma(-rsv[i], d1, sum)), tag);
        gst(cw, rep_ * 2 * HS + hslot<S>(r), rcol[i], tag);
      }
    }
    // the writer's outputs leave after the hand-off so they never delay it
    if (writer) {
      if (t == 0) {
        a.E[j] = beta;
        a.tau[j] = tau_j;
      }
#if defined(PODS_TRD_NOV)  // diagnostic variant builds only (tools/lib_variants.sh): no V stores (wrong vectors)
      if (x[0] == 12345.678) a.V[j] = x[1];
#elif defined(PODS_TRD_VNT)  // diagnostic variant: V through nontemporal stores
#pragma unroll
      for (int m = 0; m < S; ++m) {
        const int c = t + TT * m;
        if (c < n) __builtin_nontemporal_store(x[m], a.V + (int64_t)j * a.ldv + c);
      }
#else
#pragma unroll
      for (int m = 0; m < S; ++m) {
        const int c = t + TT * m;
        if (c < n) st_sc1(a.V + (int64_t)j * a.ldv + c, x[m]);  // sc1: keep V out of L2
      }
#endif
    }
    // ---- rank-2 update of step j-1 on rows >= j+1 (dead rows: zero multipliers, exact
    // ---- no-op arithmetic, so no branch touches the matrix registers) --------------------
#pragma unroll
    for (int h = 0; h < NG; ++h) {
      double vr[RH], wr[RH];
      // The group's multipliers and LDS slot values are read back to back before any use or
      // write (r5): read one by one -- each behind its row's liveness branch, or after the
      // previous element's LDS write -- they compiled to one LDS round trip each, serial.
      double rv[RH], rw[RH];
#pragma unroll
      for (int q = 0; q < RH; ++q) {
        rv[q] = h * RH + q < RL ? rsv[I0 + h * RH + q] : 0.0;
        rw[q] = h * RH + q < RL ? rsw[I0 + h * RH + q] : 0.0;
      }
      double lv[RH][SL > 0 ? SL : 1];
#pragma unroll
      for (int q = 0; q < RH; ++q)
#pragma unroll
        for (int m = 0; m < SL; ++m) lv[q][m] = h * RH + q < RL ? Al[(m * RL + h * RH + q) * TT + t] : 0.0;
      // H: slot K's values of the group (lanes 256..511; the waves of lanes < 256 hold none)
      double hv[RH];
#pragma unroll
      for (int q = 0; q < RH; ++q)
        hv[q] = (H && h * RH + q < RL && wv >= 4) ? Ah[(h * RH + q) * (TT / 2) + (t & (TT / 2 - 1))] : 0.0;
#pragma unroll
      for (int q = 0; q < RH; ++q) {
        const int i = I0 + h * RH + q;
        const int r = g + G * i;
        const bool live = r >= j + 1 && r < n;
        vr[q] = uniform(live ? rv[q] : 0.0);
        wr[q] = uniform(live ? rw[q] : 0.0);
      }
#pragma unroll
      for (int m = K; m < S; ++m) {
#pragma unroll
        for (int q = 0; q < RH; ++q) {
          const int ii = h * RH + q;
          if (ii >= RL) continue;
          if (m < K + SGH && H) {
            hv[q] = __builtin_fma(-vr[q], p[m], __builtin_fma(-wr[q], vp[m], hv[q]));
          } else if (m < K + SGH) {
            const int so = (m * R + I0 + ii) * TT * 8;
            const double ref = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rwm, soff[m - K], so, 0));
            const double nv = __builtin_fma(-vr[q], p[m], __builtin_fma(-wr[q], vp[m], ref));
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rwm, 0, 0, 0)), nv), rwm, soff[m - K], so, 0);
          } else if (m < K + SGH + SL) {
            double& ref = lv[q][m - K - SGH];
            ref = __builtin_fma(-vr[q], p[m], __builtin_fma(-wr[q], vp[m], ref));
          } else {
            double& ref = Ar[ii][m - K - SGH - SL];
            ref = __builtin_fma(-vr[q], p[m], __builtin_fma(-wr[q], vp[m], ref));
          }
        }
      }
#pragma unroll
      for (int q = 0; q < RH; ++q)
        if (h * RH + q < RL) {
#pragma unroll
          for (int m = 0; m < SL; ++m) Al[(m * RL + h * RH + q) * TT + t] = lv[q][m];
          if (H && wv >= 4) Ah[(h * RH + q) * (TT / 2) + (t & (TT / 2 - 1))] = hv[q];
        }
    }
    if (trace) trace[j * 8 + 7] = (int64_t)__builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int m = 0; m < S; ++m) vp[m] = x[m];
    tau_p = tau_j;
  }

  if (!last) {
    // ---- park the live block for the next range ---------------------------------------------
#pragma unroll
    for (int ii = 0; ii < RL; ++ii) {
#pragma unroll
      for (int m = K + SG; m < S; ++m) {
        if (m < K + SGH) {  // H: slot K's live lanes (range 1 no longer reads slot K)
          if (t0 >= TT / 2) wm(m, I0 + ii, t0) = Ah[ii * (TT / 2) + t0 - TT / 2];
        } else if (m < K + SGH + SL) {
          wm(m, I0 + ii, t0) = Al[((m - K - SGH) * RL + ii) * TT + t0];
        } else {
          wm(m, I0 + ii, t0) = Ar[ii][m - K - SGH - SL];
        }
      }
    }
  } else if (lastrow == n - 1 && n > 1) {
    // ---- D[n-1] = A^{(n-1)}[n-1, n-1] (owner of row n-1) ----------------------------------
    // tau_{n-2} = 0 (nothing below row n-1), v_{n-2} = e_{n-1}: d = a - 2 w[n-1]
    const int j = n - 1;
    if (t0 == (j & (TT - 1))) {
      const __amdgpu_buffer_rsrc_t rp = rsrc8(hbuf(a.pbuf, 0, (j - 1) & 1, HS), HS);
      const __amdgpu_buffer_rsrc_t rc = rsrc8(hbuf(a.rbuf, 0, (j - 1) & 1, HS), HS);
      const int lj = hslot<S>(j);
      double pv = 0.0, cv = 0.0;
      bool np = true, nc = true;
      for (int spin = 0; (np || nc) && spin <= SPIN_LIMIT; ++spin) {
        if (np) {
          const double q = gld(rp, lj);
          if (tag_ok(q, (uint32_t)j)) { pv = untag(q); np = false; }
        }
        if (nc) {
          const double q = gld(rc, lj);
          if (tag_ok(q, (uint32_t)j)) { cv = untag(q); nc = false; }
        }
      }
      if (np || nc) st_flag(abortw, 1u);
      const double wv_ = tau_p * pv;
      const double al = -0.5 * tau_p * wv_;
      const double wj = __builtin_fma(al, 1.0, wv_);
      a.D[j] = __builtin_fma(-wj, 1.0, __builtin_fma(-1.0, wj, cv));
    }
  } else if (n == 1 && g0 == 0 && t0 == 0) {
    a.D[0] = a.C[0];
  }
}

// -----------------------------------------------------------------------------------------
// Gershgorin bounds, pivmin and the bisection tolerance of T (one 256-thread workgroup).
// out: {gl, gu, pivmin, atol}
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tri_bounds(const double* __restrict__ D,
                                                    const double* __restrict__ E, int n,
                                                    double* __restrict__ out) {
  __shared__ double s_lo[256], s_hi[256], s_e2[256];
  const int t = threadIdx.x;
  double lo = DBL_MAX, hi = -DBL_MAX, e2m = 0.0;
  for (int i = t; i < n; i += 256) {
    const double el = i > 0 ? fabs(E[i - 1]) : 0.0;
    const double er = i < n - 1 ? fabs(E[i]) : 0.0;
    lo = fmin(lo, D[i] - (el + er));
    hi = fmax(hi, D[i] + (el + er));
    e2m = fmax(e2m, er * er);
  }
  s_lo[t] = lo;
  s_hi[t] = hi;
  s_e2[t] = e2m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      s_lo[t] = fmin(s_lo[t], s_lo[t + o]);
      s_hi[t] = fmax(s_hi[t], s_hi[t + o]);
      s_e2[t] = fmax(s_e2[t], s_e2[t + o]);
    }
    __syncthreads();
  }
  if (t == 0) {
    const double ulp = DBL_EPSILON;
    const double pivmin = DBL_MIN * fmax(1.0, s_e2[0]);
    const double tnorm = fmax(fabs(s_lo[0]), fabs(s_hi[0]));
    // dstebz: widen by FUDGE*TNORM*ULP*N + FUDGE*2*PIVMIN, FUDGE = 2.1
    const double wid = 2.1 * tnorm * ulp * n + 2.1 * 2.0 * pivmin;
    out[0] = s_lo[0] - wid;
    out[1] = s_hi[0] + wid;
    out[2] = pivmin;
    out[3] = 2.0 * ulp * tnorm;
  }
}

// e / q with a refined hardware reciprocal (v_rcp_f64 + one Newton step, ~1 ulp): the
// Sturm count only needs the sign of each pivot, and this keeps the recurrence's critical
// path far shorter than an IEEE division.
__device__ __forceinline__ double fast_div(double e, double q) {
  double r = __builtin_amdgcn_rcp(q);
  r = __builtin_fma(r, __builtin_fma(-q, r, 1.0), r);
  return e * r;
}

// Numbers of eigenvalues of T below NC shifts at once (dlaebz's Sturm count, pivmin-guarded;
// the NC recurrences are independent and interleave).
template <int NC>
__device__ __forceinline__ void sturm_counts(const double2* __restrict__ de, int n,
                                             const double (&sig)[NC], double pivmin, int (&cnt)[NC]) {
  double q[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    q[c] = 1.0;
    cnt[c] = 0;
  }
  for (int i = 0; i < n; ++i) {
    const double2 v = de[i];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      double qc = (v.x - sig[c]) - fast_div(v.y, q[c]);
      if (fabs(qc) < pivmin) qc = -pivmin;
      cnt[c] += qc < 0.0 ? 1 : 0;
      q[c] = qc;
    }
  }
}

// Shared shifts for the first bracket of every eigenvalue: NSH spread uniformly over the
// Gershgorin interval and NSH log-spaced over [2^-56.5, 1] * tnorm, where a POD spectrum
// keeps most of its eigenvalues.  One Sturm count per shift (k_sturm_grid) brackets all n
// eigenvalues at once; k_bisect then refines each from the tighter of its two brackets.
constexpr int NSH = 32768;
__device__ __forceinline__ double grid_shift(int s, double gl, double gu) {
  if (s < NSH) return gl + (gu - gl) * ((double)(s + 1) / (double)(NSH + 1));
  const double tn = fmax(fabs(gl), fabs(gu));
  return tn * exp2(-56.5 * (double)(2 * NSH - 1 - s) / (double)NSH);  // ascending in s
}

// {d_i, e_{i-1}^2} in global memory for tridiagonals too long for LDS (n > 10240)
__global__ void k_de_fill(const double* __restrict__ D, const double* __restrict__ E, int n,
                          double2* __restrict__ deg) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double e = i > 0 ? E[i - 1] : 0.0;
  deg[i] = make_double2(D[i], e * e);
}

// GDE: {d, e^2} read from global memory (n too long for LDS).  A compile-time choice: a
// runtime select between the two would make every Sturm load a flat load (2.17 vs 1.41 ms
// of k_bisect at n = 4096).
template <bool GDE>
__global__ __launch_bounds__(256) void k_sturm_grid(const double* __restrict__ D,
                                                    const double* __restrict__ E, int n,
                                                    const double* __restrict__ bounds,
                                                    int* __restrict__ cnt, const double2* __restrict__ deg) {
  extern __shared__ double2 desh[];
  const double2* de = GDE ? deg : desh;
  if (!GDE) {
    for (int i = threadIdx.x; i < n; i += 256) {
      const double e = i > 0 ? E[i - 1] : 0.0;
      desh[i] = make_double2(D[i], e * e);
    }
  }
  __syncthreads();
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= 2 * NSH) return;
  const double sig[1] = {grid_shift(s, bounds[0], bounds[1])};
  int c[1];
  sturm_counts<1>(de, n, sig, bounds[2], c);
  cnt[s] = c[0];
}

// [lo, hi) from one shift family: the first shift with count >= k+1 and the one before it
// (a binary search on the counts; both ends are tested, so count(lo) <= k < count(hi) holds
// even where rounding makes the counts non-monotone).
__device__ __forceinline__ void grid_bracket(const int* __restrict__ cnt, int base, int k, double gl,
                                             double gu, double& lo, double& hi) {
  int a = 0, b = NSH;
  while (a < b) {
    const int mid = (a + b) >> 1;
    if (cnt[base + mid] >= k + 1)
      b = mid;
    else
      a = mid + 1;
  }
  hi = a < NSH ? grid_shift(base + a, gl, gu) : DBL_MAX;
  lo = a > 0 ? grid_shift(base + a - 1, gl, gu) : -DBL_MAX;
}

constexpr int BL = 16;  // lanes per eigenvalue
constexpr int NCH = 1;  // shifts per lane: 16 shifts per step split the bracket into 17

// Eigenvalue k (ascending) of T by multisection: shift s = c*BL + l (chain c of lane l) sits
// at lo + (s+1) (hi-lo)/(BL*NCH+1).  Output lam_desc[n-1-k].  LDS: n x {d_i, e_{i-1}^2}.
// (The kernel is fp64-issue bound, so fewer shifts per step -- less work per bit -- win.)
template <bool GDE>
__global__ __launch_bounds__(256) void k_bisect(const double* __restrict__ D,
                                                const double* __restrict__ E, int n,
                                                const double* __restrict__ bounds,
                                                double* __restrict__ lam_desc, int k0, int k1,
                                                const int* __restrict__ gcnt, const double2* __restrict__ deg) {
  extern __shared__ double2 desh[];
  const double2* de = GDE ? deg : desh;
  const int t = threadIdx.x, lane = t & 63;
  if (!GDE) {
    for (int i = t; i < n; i += 256) {
      const double e = i > 0 ? E[i - 1] : 0.0;
      desh[i] = make_double2(D[i], e * e);
    }
  }
  __syncthreads();
  const double gl = bounds[0], gu = bounds[1], pivmin = bounds[2], atol = bounds[3];
  const int l = t % BL;
  const int k = k0 + blockIdx.x * (256 / BL) + t / BL;  // ascending index, [k0, k1) this launch
  const bool active = k < k1;
  double lo = gl, hi = gu;
  if (gcnt && active) {
    double lu, hu, ll, hl;
    grid_bracket(gcnt, 0, k, gl, gu, lu, hu);
    grid_bracket(gcnt, NSH, k, gl, gu, ll, hl);
    lo = fmax(gl, lu);
    hi = fmin(gu, hu);
    if (fmax(lo, ll) < fmin(hi, hl)) {
      lo = fmax(lo, ll);
      hi = fmin(hi, hl);
    }
  }
  for (int it = 0; it < 128; ++it) {
    const bool conv = !active || (hi - lo) <= fmax(atol, 2.0 * DBL_EPSILON * fmax(fabs(lo), fabs(hi)));
    if (__all(conv)) break;
    const double step = (hi - lo) * (1.0 / (BL * NCH + 1));
    double sig[NCH];
    int cnt[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) sig[c] = lo + step * (double)(c * BL + l + 1);
    sturm_counts<NCH>(de, n, sig, pivmin, cnt);
    int f = BL * NCH;  // first shift with count >= k+1
#pragma unroll
    for (int c = NCH - 1; c >= 0; --c) {
      const unsigned long long m = __ballot(cnt[c] >= k + 1);
      const uint32_t gm = (uint32_t)((m >> (lane & ~(BL - 1))) & ((1u << BL) - 1));
      if (gm) f = c * BL + __ffs(gm) - 1;
    }
    if (!conv) {
      const double nhi = f < BL * NCH ? lo + step * (double)(f + 1) : hi;
      const double nlo = f > 0 ? lo + step * (double)f : lo;
      lo = nlo;
      hi = nhi;
    }
  }
  if (active && l == 0) lam_desc[n - 1 - k] = 0.5 * (lo + hi);
}

// -----------------------------------------------------------------------------------------
// Eigenvector of T for lam_desc[k] by a twisted factorisation (LAPACK dlar1v's recurrences):
// T - lam I = L+ D+ L+^T (top down) = U- D- U-^T (bottom up); the twist index r minimises
// |gamma_r| = |D+_r + D-_r - (d_r - lam)|, then z_r = 1, z_i = -L+_i z_{i+1} (i < r),
// z_{i+1} = -U-_i z_i (i >= r), normalised.  One workgroup per vector.  The two
// factorisations run concurrently (lane 0 of waves 0 and 1), gamma and its argmin are
// parallel, the multipliers L+_i = e_i / D+_i and U-_i = e_i / D-_{i+1} are formed in parallel
// in place of the pivots, and the two halves of z are again two concurrent chains.
// LDS: d - lam (then z), e, D+ (then L+), D- (then U- shifted by one): 4n doubles + 16.
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_twisted(const double* __restrict__ D,
                                                 const double* __restrict__ E, int n,
                                                 const double* __restrict__ lam_desc,
                                                 const double* __restrict__ bounds,
                                                 double* __restrict__ G, double* __restrict__ Z,
                                                 int ldz) {
  extern __shared__ double sh[];
  double* sa = sh;          // d - lam, later z
  double* se = sh + n;      // e
  double* dp = sh + 2 * n;  // D+, later L+
  double* dm = sh + 3 * n;  // D-, later U- (U-_i at dm[i+1])
  double* scr = sh + 4 * n;  // 16 doubles of reduction scratch
  double* rv = scr;
  double* ri = scr + 4;
  const int k = blockIdx.x, t = threadIdx.x;
  const double lam = lam_desc[k];
  const double pivmin = bounds[2], atol = bounds[3];
  double* g = G + (int64_t)k * n;  // |gamma_i|
  for (int i = t; i < n; i += 256) {
    sa[i] = D[i] - lam;
    se[i] = i < n - 1 ? E[i] : 0.0;
  }
  __syncthreads();
  // (the serial loops read their operands 16 at a time so one LDS latency covers 16 steps)
  constexpr int CH = 16;
  if (t == 0) {  // L+ D+ L+^T, top down
    double dpi = sa[0];
    for (int i0 = 0; i0 < n - 1; i0 += CH) {
      double ev[CH], av[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int i = min(i0 + u, n - 2);
        ev[u] = se[i];
        av[u] = sa[i + 1];
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (i0 + u < n - 1) {
          if (fabs(dpi) < pivmin) dpi = -pivmin;
          dp[i0 + u] = dpi;
          const double li = fast_div(ev[u], dpi);
          dpi = av[u] - li * ev[u];
        }
      }
    }
    if (fabs(dpi) < pivmin) dpi = -pivmin;
    dp[n - 1] = dpi;
  } else if (t == 64) {  // U- D- U-^T, bottom up
    double dmi = sa[n - 1];
    if (fabs(dmi) < pivmin) dmi = -pivmin;
    dm[n - 1] = dmi;
    for (int i0 = n - 2; i0 >= 0; i0 -= CH) {
      double ev[CH], av[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int i = max(i0 - u, 0);
        ev[u] = se[i];
        av[u] = sa[i];
      }
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (i0 - u >= 0) {
          const double ui = fast_div(ev[u], dmi);
          dmi = av[u] - ui * ev[u];
          if (fabs(dmi) < pivmin) dmi = -pivmin;
          dm[i0 - u] = dmi;
        }
      }
    }
  }
  __syncthreads();
  // |gamma| and its argmin (ties: the larger index, as the sequential bottom-up scan)
  {
    double bv = DBL_MAX;
    int bi = -1;
    for (int i = t; i < n; i += 256) {
      const double gi = fabs(dp[i] + dm[i] - sa[i]);
      g[i] = gi;
      if (gi <= bv) {
        bv = gi;
        bi = i;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov < bv || (ov == bv && oi > bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if ((t & 63) == 0) {
      rv[t >> 6] = bv;
      ri[t >> 6] = (double)bi;
    }
    __syncthreads();
    if (t == 0) {
      int best = 0;
      for (int w = 1; w < 4; ++w)
        if (rv[w] < rv[best] || (rv[w] == rv[best] && ri[w] > ri[best])) best = w;
      scr[8] = ri[best];
    }
  }
  // A numerically repeated eigenvalue (T split into blocks, e.g. zero or diagonal blocks):
  // the q-th member of such a cluster twists at the index with the (q+1)-th smallest
  // |gamma|, which lands each member in a different block.
  int q = 0;
  for (int jj = 0; jj < k; ++jj)
    if (fabs(lam_desc[jj] - lam) <= 4.0 * atol) ++q;
  if (q > 0) {
    __syncthreads();
    for (int round = 0; round <= q; ++round) {
      double bv = DBL_MAX;
      int bi = n;
      for (int i = t; i < n; i += 256) {
        const double v = g[i];
        if (v < bv || (v == bv && i < bi)) {
          bv = v;
          bi = i;
        }
      }
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ov < bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      __syncthreads();
      if ((t & 63) == 0) {
        rv[t >> 6] = bv;
        ri[t >> 6] = (double)bi;
      }
      __syncthreads();
      if (t == 0) {
        int best = 0;
        for (int w = 1; w < 4; ++w)
          if (rv[w] < rv[best] || (rv[w] == rv[best] && ri[w] < ri[best])) best = w;
        scr[8] = ri[best];
        const int ib = (int)ri[best];
        if (ib >= 0 && ib < n) g[ib] = DBL_MAX;  // excluded from later rounds
      }
      __syncthreads();
    }
  }
  __syncthreads();
  // (no finite |gamma| -- a NaN input -- leaves the argmin at -1 or n: clamped, so garbage in
  // gives garbage out, never an access outside the vectors)
  const int r = min(max((int)scr[8], 0), n - 1);
  // multipliers in place: L+_i = e_i / D+_i at dp[i], U-_i = e_i / D-_{i+1} at dm[i+1]
  for (int i = t; i < n - 1; i += 256) {
    dp[i] = se[i] / dp[i];
    dm[i + 1] = se[i] / dm[i + 1];
  }
  __syncthreads();
  double* z = sa;
  if (t == 0) {
    z[r] = 1.0;
    double zn1 = 1.0, zn2 = 0.0;  // z[i+1], z[i+2]
    for (int i0 = r - 1; i0 >= 0; i0 -= CH) {
      double lv[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) lv[u] = dp[max(i0 - u, 0)];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int i = i0 - u;
        if (i >= 0) {
          double zi = -lv[u] * zn1;
          // a zero component: use row i+1 of (T - lam I) z = 0 instead (dlar1v)
          if (zn1 == 0.0 && se[i] != 0.0 && i + 2 < n) zi = -(se[i + 1] / se[i]) * zn2;
          z[i] = zi;
          zn2 = zn1;
          zn1 = zi;
        }
      }
    }
  } else if (t == 64) {
    double zi = 1.0, zp = 0.0;  // z[i], z[i-1]
    for (int i0 = r; i0 < n - 1; i0 += CH) {
      double uv[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) uv[u] = dm[min(i0 + u, n - 2) + 1];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int i = i0 + u;
        if (i < n - 1) {
          double zn = -uv[u] * zi;
          if (zi == 0.0 && se[i] != 0.0 && i >= 1) zn = -(se[i - 1] / se[i]) * zp;
          z[i + 1] = zn;
          zp = zi;
          zi = zn;
        }
      }
    }
  }
  __syncthreads();
  // unit 2-norm
  double ss = 0.0;
  for (int i = t; i < n; i += 256) ss = __builtin_fma(z[i], z[i], ss);
  ss = wave_sum(ss);
  if ((t & 63) == 0) scr[t >> 6] = ss;
  __syncthreads();
  const double inv = 1.0 / sqrt((scr[0] + scr[1]) + (scr[2] + scr[3]));
  for (int i = t; i < n; i += 256) Z[(int64_t)i * ldz + k] = z[i] * inv;
}

// Modified Gram-Schmidt of the nvec vectors inside clusters |lam_i - lam_k| <= 1e-3 ||T||
// (dstein ORTOL), in descending order, then re-normalise.  One workgroup.
__global__ __launch_bounds__(256) void k_orth(const double* __restrict__ lam_desc,
                                              const double* __restrict__ bounds, int n, int nvec,
                                              double* __restrict__ Z, int ldz) {
  __shared__ double red[2][4];
  const int t = threadIdx.x;
  const double tnorm = fmax(fabs(bounds[0]), fabs(bounds[1]));
  int rk = 0;
  auto dot = [&](int a, int b) {
    double d = 0.0;
    for (int i = t; i < n; i += 256) d = __builtin_fma(Z[(int64_t)i * ldz + a], Z[(int64_t)i * ldz + b], d);
    d = wave_sum(d);
    double* rb = red[rk++ & 1];
    if ((t & 63) == 0) rb[t >> 6] = d;
    __syncthreads();
    return rb[0] + rb[1] + rb[2] + rb[3];
  };
  auto project_out = [&](int k) {  // MGS of column k against its cluster's earlier columns
    bool touched = false;
    for (int jj = 0; jj < k; ++jj) {
      if (fabs(lam_desc[jj] - lam_desc[k]) > 1e-3 * tnorm) continue;
      const double d = dot(jj, k);
      for (int i = t; i < n; i += 256)
        Z[(int64_t)i * ldz + k] = __builtin_fma(-d, Z[(int64_t)i * ldz + jj], Z[(int64_t)i * ldz + k]);
      __syncthreads();
      touched = true;
    }
    return touched;
  };
  auto clustered = [&](int k) {
    for (int jj = 0; jj < k; ++jj)
      if (fabs(lam_desc[jj] - lam_desc[k]) <= 1e-3 * tnorm) return true;
    return false;
  };
  for (int k = 1; k < nvec; ++k) {
    if (!clustered(k)) continue;
    const double s0 = dot(k, k);
    project_out(k);
    double s = dot(k, k);
    // "twice is enough" (Kahan-Parlett): a projection that removed more than half of the
    // squared norm leaves a vector whose orthogonality error grows like 1/sqrt(s / s0); a second
    // pass restores it to rounding level
    if (s < 0.5 * s0 && s >= 1e-16) {
      project_out(k);
      s = dot(k, k);
    }
    // A vector that (nearly) lies in the span of the cluster's earlier ones -- identical
    // inverse-iteration results inside a degenerate cluster, e.g. a zero or diagonal block --
    // is replaced by a unit vector orthogonalised against them (dstein's restart, as a
    // deterministic choice), so the columns stay orthonormal instead of turning into NaN.
    for (int attempt = 0; s < 1e-16 && attempt < n; ++attempt) {
      const int p = (int)(((int64_t)k * 7919 + attempt * 104729) % n);
      for (int i = t; i < n; i += 256) Z[(int64_t)i * ldz + k] = i == p ? 1.0 : 0.0;
      __syncthreads();
      project_out(k);
      project_out(k);
      s = dot(k, k);
    }
    const double inv = 1.0 / sqrt(s);
    for (int i = t; i < n; i += 256) Z[(int64_t)i * ldz + k] = Z[(int64_t)i * ldz + k] * inv;
    __syncthreads();
  }
}

// -----------------------------------------------------------------------------------------
// Back-transformation.  Reflector j (0..n-2): H_j = I - tau_j v_j v_j^T, v_j = row j of V
// (zeros at c <= j, 1 at c = j+1).  Block b holds reflectors [64b, 64b+nb); its compact-WY
// factor T_b (dlarft 'F','C') makes H_{64b} ... H_{64b+nb-1} = I - V_b T_b V_b^T.
// -----------------------------------------------------------------------------------------
constexpr int WB = 64;

typedef double bt_f64x4 __attribute__((ext_vector_type(4)));

// T_b of block b (one workgroup per block).  Gram matrix G = V_b V_b^T on fp64 MFMA
// (wave w: rows 16w..16w+15 x all 64 columns, 4 v_mfma_f64_16x16x4 accumulators), V_b staged
// through LDS 64 columns at a time with the next chunk's loads in flight; then the dlarft
// recurrence T[0:i, i] = -tau_i T[0:i, 0:i] G[0:i, i], T[i][i] = tau_i.
__global__ __launch_bounds__(256) void k_larft(const double* __restrict__ V, int64_t ldv,
                                               const double* __restrict__ tau, int n,
                                               double* __restrict__ Tg) {
  __shared__ double vs[WB][WB + 1];
  __shared__ double gm[WB][WB + 1];
  __shared__ double tm[WB][WB + 1];
  __shared__ double tmp[WB];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int j0 = b * WB;
  const int nb = min(WB, n - 1 - j0);
  bt_f64x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = bt_f64x4{0.0, 0.0, 0.0, 0.0};
  double st[16];
  auto load = [&](int cb) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u, p = e >> 6, cc = e & 63, c = cb + cc;
      st[u] = (p < nb && c < n) ? V[(int64_t)(j0 + p) * ldv + c] : 0.0;
    }
  };
  const int cstart = j0 + 1;  // V_b is zero left of column j0 + 1
  load(cstart);
  for (int cb = cstart; cb < n; cb += WB) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = t + 256 * u;
      vs[e >> 6][e & 63] = st[u];
    }
    __syncthreads();
    if (cb + WB < n) load(cb + WB);
#pragma unroll
    for (int kk = 0; kk < WB; kk += 4) {
      const double a = vs[16 * w + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double bq = vs[16 * q + (lane & 15)][kk + (lane >> 4)];
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bq, acc[q], 0, 0, 0);
      }
    }
  }
  // C/D layout: col = lane & 15, row = (lane >> 4) + 4 r
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) gm[16 * w + (lane >> 4) + 4 * r][16 * q + (lane & 15)] = acc[q][r];
  for (int e = t; e < WB * WB; e += 256) tm[e / WB][e % WB] = 0.0;
  __syncthreads();
  for (int i = 0; i < nb; ++i) {
    const double ti = tau[j0 + i];
    if (t == 0) tm[i][i] = ti;
    if (t < i) tmp[t] = -ti * gm[t][i];
    __syncthreads();
    if (t < i) {
      double s = 0.0;
      for (int q = t; q < i; ++q) s = __builtin_fma(tm[t][q], tmp[q], s);
      tm[t][i] = s;
    }
    __syncthreads();
  }
  for (int e = t; e < WB * WB; e += 256) Tg[(int64_t)b * WB * WB + e] = tm[e / WB][e % WB];
}

// ---- 16-byte {value, tag} granules for the back-transformation's hand-offs: no value bits
// ---- are borrowed, the tag is the block iteration + 1 (the buffers are zeroed per call).
typedef int bt_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc16(const double* base, int64_t count) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), 0, (int)(count * 16), 0x00020000);
}
__device__ __forceinline__ void gst16(__amdgpu_buffer_rsrc_t r, int idx, double v, uint32_t tag) {
  const long long b = __double_as_longlong(v);
  bt_v4i q;
  q.x = (int)(b & 0xffffffffll);
  q.y = (int)(b >> 32);
  q.z = (int)tag;
  q.w = 0;
  __builtin_amdgcn_raw_buffer_store_b128(q, r, idx * 16, 0, 16u);
}
__device__ __forceinline__ bool gld16(__amdgpu_buffer_rsrc_t r, int idx, uint32_t tag, double& v) {
  const bt_v4i q = __builtin_amdgcn_raw_buffer_load_b128(r, idx * 16, 0, (1u << 31) | 16u);
  v = __hiloint2double(q.y, q.x);
  return (uint32_t)q.z == tag;
}

// One persistent launch for Z <- Q_0 Q_1 ... Q_{nblk-1} Z (blocks applied last to first).
// Workgroup g owns rows [g*CR, g*CR + CR) of Z in LDS.  Per block: every workgroup with rows
// below the block's first reflector forms its partial V_b Z (64 x nvec) and publishes it; the
// workgroup owning vector k (k mod G) sums the partials in workgroup order, multiplies by T_b
// and publishes column k of W2 = T_b V_b Z; every active workgroup then applies
// Z -= V_b^T W2 to its rows.  Two hand-offs per block instead of three kernel boundaries.
template <int CR>
__global__ __launch_bounds__(256, 1) void k_bt_fused(const double* __restrict__ V, int64_t ldv,
                                                     const double* __restrict__ Tg, int n, int nvec,
                                                     int nblk, double* __restrict__ Z, int ldz,
                                                     double* part, double* w2g, uint32_t* abortw) {
  extern __shared__ double sm[];
  const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
  const int c0 = g * CR;
  const int rows = min(CR, n - c0);
  const int ldvt = CR + 1;
  double* zs = sm;                  // CR x nvec
  double* vt = zs + CR * nvec;      // 64 x (CR + 1): V_b restricted to this workgroup's rows
  double* wr = vt + 64 * ldvt;      // 64 x nvec: W2
  double* wk = wr + 64 * nvec;      // 4 x 64: reducer partial sums
  double* tl = wk + 256;            // 64 x 65: T_b (reducer workgroups)
  for (int e = t; e < CR * nvec; e += 256) {
    const int c = e / nvec, k = e - c * nvec;
    zs[e] = c < rows ? Z[(int64_t)(c0 + c) * ldz + k] : 0.0;
  }
  const int PW = 64 * nvec;  // granules per workgroup partial
  const __amdgpu_buffer_rsrc_t rp = rsrc16(part, (int64_t)2 * G * PW);
  const __amdgpu_buffer_rsrc_t rw = rsrc16(w2g, (int64_t)2 * PW);
  bool bad = false;
  for (int it = 0; it < nblk && !bad; ++it) {
    const int b = nblk - 1 - it, j0 = 64 * b, nb = min(64, n - 1 - j0);
    const int gmin = (j0 + 1) / CR;
    const uint32_t tag = (uint32_t)(it + 1);
    const int par = it & 1;
    const bool active = g >= gmin;
    __syncthreads();  // the previous block's apply is done with vt and wr
    if (g < nvec) {  // T_b for the reducer (all loads in flight together)
      double tv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) tv[u] = Tg[(int64_t)b * 64 * 64 + t + 256 * u];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int e = t + 256 * u;
        tl[(e >> 6) * 65 + (e & 63)] = tv[u];
      }
    }
    if (active) {
      double vv[CR / 4];
#pragma unroll
      for (int u = 0; u < CR / 4; ++u) {
        const int e = t + 256 * u, p = e / CR, c = e - p * CR;
        vv[u] = (p < nb && c < rows) ? V[(int64_t)(j0 + p) * ldv + c0 + c] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < CR / 4; ++u) {
        const int e = t + 256 * u, p = e / CR, c = e - p * CR;
        vt[p * ldvt + c] = vv[u];
      }
      __syncthreads();
      for (int o = t; o < PW; o += 256) {
        const int p = o / nvec, k = o - p * nvec;
        double s = 0.0;
#pragma unroll 16
        for (int c = 0; c < CR; ++c) s = __builtin_fma(vt[p * ldvt + c], zs[c * nvec + k], s);
        gst16(rp, (par * G + g) * PW + o, s, tag);
      }
    }
    // ---- reduction + T_b: vector k by workgroup k mod G, 4 threads per row p ------------------
    for (int k = g; k < nvec; k += G) {
      const int p = t & 63, qd = t >> 6;  // quarter qd sums workgroups gmin + qd, +4, +8, ...
      double s = 0.0;
      for (int gg0 = gmin + qd; gg0 < G && !bad; gg0 += 64) {
        double v[16];
        for (int spin = 0;; ++spin) {
          bool ok = true;
#pragma unroll
          for (int u = 0; u < 16; ++u) {
            const int gg = gg0 + 4 * u;
            v[u] = 0.0;
            if (gg < G) ok = gld16(rp, (par * G + gg) * PW + p * nvec + k, tag, v[u]) && ok;
          }
          if (ok) break;
          if (spin > SPIN_LIMIT || __hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bad = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
      }
      wk[qd * 64 + p] = s;
      __syncthreads();
      if (t < 64) {
        const double wsum = ((wk[p] + wk[64 + p]) + wk[128 + p]) + wk[192 + p];
        wk[p] = wsum;
      }
      __syncthreads();
      if (t < 64) {
        const double* T = tl + p * 65;
        double w = 0.0;
        for (int q = p; q < 64; ++q) w = __builtin_fma(T[q], wk[q], w);
        gst16(rw, par * PW + p * nvec + k, w, tag);
      }
      __syncthreads();
    }
    bad = __syncthreads_or(bad);
    if (!active || bad) continue;
    // ---- apply: Z -= V_b^T W2 on this workgroup's rows --------------------------------------
    for (int o0 = 0; o0 < PW; o0 += 256 * 8) {  // up to 8 granules per lane in flight
      double v[8];
      for (int spin = 0;; ++spin) {
        bool ok = true;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int o = o0 + t + 256 * u;
          v[u] = 0.0;
          if (o < PW) ok = gld16(rw, par * PW + o, tag, v[u]) && ok;
        }
        if (ok) break;
        if (spin > SPIN_LIMIT || __hip_atomic_load(abortw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          __hip_atomic_store(abortw, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bad = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = o0 + t + 256 * u;
        if (o < PW) wr[o] = v[u];
      }
    }
    bad = __syncthreads_or(bad);
    for (int o = t; o < rows * nvec; o += 256) {
      const int c = o / nvec, k = o - c * nvec;
      double s = 0.0;
      for (int p = 0; p < 64; ++p) s = __builtin_fma(vt[p * ldvt + c], wr[p * nvec + k], s);
      zs[o] -= s;
    }
  }
  __syncthreads();
  for (int e = t; e < rows * nvec; e += 256) {
    const int c = e / nvec, k = e - c * nvec;
    Z[(int64_t)(c0 + c) * ldz + k] = zs[e];
  }
}

template <int R, int S, int K, int SG, int SL, int H = 0>
static hipError_t launch_trd_t(const TrdArgs& a, hipStream_t st) {
  constexpr int I0 = H ? 1 : ((2 * K < R) ? 2 * K : R);
  const size_t lds = ((size_t)SL * (R - I0) * TT + (size_t)H * (R - I0) * (TT / 2) + 16 + 4 + 4 * R + 8 * (R + 2) + R) *
                     sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_trd<R, S, K, SG, SL, H>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = check_persistent(reinterpret_cast<const void*>(&k_trd<R, S, K, SG, SL, H>), TT, lds, a.G, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_trd<R, S, K, SG, SL, H>), dim3(a.G), dim3(TT), lds, st, a);
  return hipGetLastError();
}

}  // namespace eig

bool persistent_grid_fits(int blocks_per_cu, int cus, int64_t grid) {
  return blocks_per_cu > 0 && cus > 0 && grid <= (int64_t)blocks_per_cu * cus;
}

// CUs a stream may use: the popcount of its CU mask (a stream made by
// hipExtStreamCreateWithCUMask), else the device's CU count
int stream_cus(hipStream_t st) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  if (!st) return cus;
  uint32_t m[16] = {};
  int n = 0;
  if (hipExtStreamGetCUMask(st, 16, m) == hipSuccess)
    for (int i = 0; i < 16; ++i) n += __builtin_popcount(m[i]);
  return (n > 0 && n < cus) ? n : cus;
}

hipError_t check_persistent(const void* fn, int block, size_t lds, int64_t grid, hipStream_t st) {
  struct Key {
    const void* fn;
    int block;
    size_t lds;
    int dev;
    int per, cus;
  };
  static std::mutex mu;
  static std::vector<Key> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  int per = -1, cus = 0;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const Key& k : cache)
      if (k.fn == fn && k.block == block && k.lds == lds && k.dev == dev) {
        per = k.per;
        cus = k.cus;
      }
  }
  if (per < 0) {
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, block, lds);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(mu);
    cache.push_back(Key{fn, block, lds, dev, per, cus});
  }
  if (st) cus = std::min(cus, stream_cus(st));
  return persistent_grid_fits(per, cus, grid) ? hipSuccess : hipErrorCooperativeLaunchTooLarge;
}

// Tridiagonalisation plan: rows per workgroup R (G = ceil(n/R) <= 256 workgroups),
// S = ceil(n/512) column slots per lane.
int trd_plan(int n, int* R, int* G, int64_t* slab_doubles) {
  int r = 0;
  if (n <= 256) r = 1;
  else if (n <= 512) r = 2;
  else if (n <= 1024) r = 4;
  else if (n <= 2048) r = 8;
  else if (n <= 4096) r = 16;
  else return -1;
  const int s = r == 16 ? 8 : (r == 8 ? 4 : (r == 4 ? 2 : 1));
  *R = r;
  *G = (n + r - 1) / r;
  *slab_doubles = (int64_t)(*G) * s * r * eig::TT;
  return 0;
}

// One launch per column range (k_trd header).  Storage split per range {SG, SL}: 16 rows
// x 8 slots = 128 doubles/lane at range 0 do not fit VGPRs + LDS next to the vectors, so
// one slot stays in the (L2-resident) slab there; later ranges hold everything on chip.
// Range 1 (14 rows x 7 slots) keeps all of it in VGPRs + LDS even though the compiler then
// spills ~100 VGPRs of loop-invariant state: 5.43 ms against 6.25 ms with a slab slot,
// whose mixed load/store traffic serialises every row group on a full vmcnt drain (r4, with
// the slab through buffer ops and its dead columns skipped: 6.44 against 5.49 ms, spills
// 104 -> 48; range 0 gained from the same change, 8.07 -> 7.62 ms).
hipError_t launch_trd(const TrdArgs& a, int R, hipStream_t st) { return launch_trd_ranges(a, R, 0, 7, st); }

// Column ranges kb..ke (inclusive, clipped to klast) of the tridiagonalisation: each range is
// its own launch and leaves the live block parked in a.Wm, so a caller may run the ranges of
// one matrix in separate calls (with other work on the stream between them) as long as the
// workspace of TrdArgs is left alone in between.
// LDS slots of ranges 2-5 of the 16-row plan (variant builds: -DPODS_TRD_SL3=...).  r6: range 3
// with none (204 VGPRs, no spill) instead of one -- pods_syev 31.09 -> 30.83 ms, the C3 step
// 69.02 -> 68.78 ms; range 2 with 3 slots and ranges 4-5 with one measured slower
// (profiles/r6/trd_range_slots_ab.log)
#ifndef PODS_TRD_SL2
#define PODS_TRD_SL2 2
#endif
#ifndef PODS_TRD_SL3
#define PODS_TRD_SL3 0
#endif
#ifndef PODS_TRD_SL4
#define PODS_TRD_SL4 0
#endif
#ifndef PODS_TRD_SL5
#define PODS_TRD_SL5 0
#endif
hipError_t launch_trd_ranges(const TrdArgs& a, int R, int kb, int ke, hipStream_t st) {
  using namespace eig;
  hipError_t e = hipSuccess;
  if (a.klast != (a.n - 1) / TT) return hipErrorInvalidValue;
#define PODS_TRD(RR, SS, KK, SGG, SLL) \
  if (e == hipSuccess && KK <= a.klast && KK >= kb && KK <= ke) e = launch_trd_t<RR, SS, KK, SGG, SLL>(a, st)
  switch (R) {
    case 1: PODS_TRD(1, 1, 0, 0, 0); break;
    case 2: PODS_TRD(2, 1, 0, 0, 0); break;
    case 4:
      PODS_TRD(4, 2, 0, 0, 0);
      PODS_TRD(4, 2, 1, 0, 0);
      break;
    case 8:
      PODS_TRD(8, 4, 0, 0, 0);
      PODS_TRD(8, 4, 1, 0, 0);
      PODS_TRD(8, 4, 2, 0, 0);
      PODS_TRD(8, 4, 3, 0, 0);
      break;
    case 16:
      // range 0 in two launches: columns [0, 256) with slot 0 in the L2 slab, [256, 511) with
      // the live half of slot 0 in LDS (r6)
      PODS_TRD(16, 8, 0, 1, 2);
      if (e == hipSuccess && 0 <= a.klast && kb <= 0 && 0 <= ke) e = launch_trd_t<16, 8, 0, 0, 2, 1>(a, st);
      PODS_TRD(16, 8, 1, 0, 2);
      PODS_TRD(16, 8, 2, 0, PODS_TRD_SL2);
      PODS_TRD(16, 8, 3, 0, PODS_TRD_SL3);
      PODS_TRD(16, 8, 4, 0, PODS_TRD_SL4);
      PODS_TRD(16, 8, 5, 0, PODS_TRD_SL5);
      PODS_TRD(16, 8, 6, 0, 0);
      PODS_TRD(16, 8, 7, 0, 0);
      break;
    default: return hipErrorInvalidValue;
  }
#undef PODS_TRD
  return e;
}

hipError_t launch_tri_bounds(const double* D, const double* E, int n, double* bounds, hipStream_t st) {
  hipLaunchKernelGGL(eig::k_tri_bounds, dim3(1), dim3(256), 0, st, D, E, n, bounds);
  return hipGetLastError();
}

// Eigenvalues with ascending indices [k0, k1) (written to lam_desc[n-1-k]); bounds from
// launch_tri_bounds.
hipError_t launch_tri_bisect(const double* D, const double* E, int n, const double* bounds,
                             double* lam_desc, int k0, int k1, int* grid_cnt, hipStream_t st, double2* deg) {
  if (k1 <= k0) return hipSuccess;
  size_t lds = (size_t)n * sizeof(double2);
  if (lds > 160 * 1024) {
    if (!deg) return hipErrorInvalidValue;  // the caller must supply the global {d, e^2} array
    hipLaunchKernelGGL(eig::k_de_fill, dim3((n + 255) / 256), dim3(256), 0, st, D, E, n, deg);
    lds = 0;
  } else {
    deg = nullptr;
  }
  const bool gde = deg != nullptr;
  if (grid_cnt) {
    const void* kg = gde ? reinterpret_cast<const void*>(&eig::k_sturm_grid<true>)
                         : reinterpret_cast<const void*>(&eig::k_sturm_grid<false>);
    hipError_t e = hipFuncSetAttribute(kg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (gde)
      hipLaunchKernelGGL(eig::k_sturm_grid<true>, dim3(2 * eig::NSH / 256), dim3(256), lds, st, D, E, n, bounds,
                         grid_cnt, deg);
    else
      hipLaunchKernelGGL(eig::k_sturm_grid<false>, dim3(2 * eig::NSH / 256), dim3(256), lds, st, D, E, n, bounds,
                         grid_cnt, deg);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const void* kb = gde ? reinterpret_cast<const void*>(&eig::k_bisect<true>)
                       : reinterpret_cast<const void*>(&eig::k_bisect<false>);
  hipError_t e = hipFuncSetAttribute(kb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  const int per = 256 / eig::BL;
  if (gde)
    hipLaunchKernelGGL(eig::k_bisect<true>, dim3((k1 - k0 + per - 1) / per), dim3(256), lds, st, D, E, n,
                       bounds, lam_desc, k0, k1, grid_cnt, deg);
  else
    hipLaunchKernelGGL(eig::k_bisect<false>, dim3((k1 - k0 + per - 1) / per), dim3(256), lds, st, D, E, n,
                       bounds, lam_desc, k0, k1, grid_cnt, deg);
  return hipGetLastError();
}

size_t tri_grid_bytes() { return (size_t)2 * eig::NSH * sizeof(int); }

hipError_t launch_tri_eigvals(const double* D, const double* E, int n, double* bounds,
                              double* lam_desc, int* grid_cnt, hipStream_t st, double2* deg) {
  hipError_t e = launch_tri_bounds(D, E, n, bounds, st);
  if (e != hipSuccess) return e;
  return launch_tri_bisect(D, E, n, bounds, lam_desc, 0, n, grid_cnt, st, deg);
}

hipError_t launch_tri_eigvecs(const double* D, const double* E, int n, const double* lam_desc,
                              const double* bounds, int nvec, double* X, double* Z, hipStream_t st) {
  const size_t lds = ((size_t)n * 4 + 16) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&eig::k_twisted),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(eig::k_twisted, dim3(nvec), dim3(256), lds, st, D, E, n, lam_desc, bounds, X, Z,
                     nvec);
  hipLaunchKernelGGL(eig::k_orth, dim3(1), dim3(256), 0, st, lam_desc, bounds, n, nvec, Z, nvec);
  return hipGetLastError();
}

hipError_t launch_orth(const double* lam_desc, const double* bounds, int n, int nvec, double* Z, int ldz,
                       hipStream_t st) {
  hipLaunchKernelGGL(eig::k_orth, dim3(1), dim3(256), 0, st, lam_desc, bounds, n, nvec, Z, ldz);
  return hipGetLastError();
}

hipError_t launch_back_transform(const double* V, int64_t ldv, const double* tau, int n, int nvec,
                                 double* Tg, double* part, double* W2, uint32_t* abortw, double* Z,
                                 hipStream_t st, bool skip_larft) {
  const int nref = n - 1;
  if (nref <= 0 || nvec <= 0) return hipSuccess;
  const int nblk = (nref + eig::WB - 1) / eig::WB;
  if (!skip_larft) hipLaunchKernelGGL(eig::k_larft, dim3(nblk), dim3(256), 0, st, V, ldv, tau, n, Tg);
  int CR = 0, G = 0;
  bt_plan(n, nvec, &CR, &G);
  hipError_t e = hipMemsetAsync(part, 0, bt_part_bytes(n, nvec), st);
  if (e == hipSuccess) e = hipMemsetAsync(W2, 0, bt_w2_bytes(nvec), st);
  if (e != hipSuccess) return e;
  const size_t lds = ((size_t)CR * nvec + 64 * (CR + 1) + 64 * nvec + 256 + 64 * 65) * sizeof(double);
  const void* fn = CR == 16 ? reinterpret_cast<const void*>(&eig::k_bt_fused<16>)
                 : CR == 32 ? reinterpret_cast<const void*>(&eig::k_bt_fused<32>)
                            : reinterpret_cast<const void*>(&eig::k_bt_fused<64>);
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = check_persistent(fn, 256, lds, G, st);
  if (e != hipSuccess) return e;
  if (CR == 16)
    hipLaunchKernelGGL(eig::k_bt_fused<16>, dim3(G), dim3(256), lds, st, V, ldv, (const double*)Tg, n,
                       nvec, nblk, Z, nvec, part, W2, abortw);
  else if (CR == 32)
    hipLaunchKernelGGL(eig::k_bt_fused<32>, dim3(G), dim3(256), lds, st, V, ldv, (const double*)Tg, n,
                       nvec, nblk, Z, nvec, part, W2, abortw);
  else
    hipLaunchKernelGGL(eig::k_bt_fused<64>, dim3(G), dim3(256), lds, st, V, ldv, (const double*)Tg, n,
                       nvec, nblk, Z, nvec, part, W2, abortw);
  return hipGetLastError();
}

hipError_t launch_larft(const double* V, int64_t ldv, const double* tau, int n, double* Tg, hipStream_t st) {
  const int nref = n - 1;
  if (nref <= 0) return hipSuccess;
  const int nblk = (nref + eig::WB - 1) / eig::WB;
  hipLaunchKernelGGL(eig::k_larft, dim3(nblk), dim3(256), 0, st, V, ldv, tau, n, Tg);
  return hipGetLastError();
}

// rows of Z per workgroup (16, 32 or 64) and workgroups (<= 64) of the back-transformation
void bt_plan(int n, int nvec, int* CR, int* G) {
  (void)nvec;
  const int cr = n <= 1024 ? 16 : (n <= 2048 ? 32 : 64);
  *CR = cr;
  *G = (n + cr - 1) / cr;
}
size_t bt_part_bytes(int n, int nvec) {
  int CR = 0, G = 0;
  bt_plan(n, nvec, &CR, &G);
  return (size_t)2 * G * 64 * nvec * 16;
}
size_t bt_w2_bytes(int nvec) { return (size_t)2 * 64 * nvec * 16; }

}  // namespace pods

// gfx950 kernels of the digital-filter + PODFS hot path.
//
// Numerics contract (compiled with -ffp-contract=off):
//   * k_mt_*          reproduce numpy's legacy MT19937 stream bit-for-bit
//   * k_filter_x/yz   reproduce scipy.signal.convolve(method='direct') x->y->z order and
//                     the adapt1d / adapt2prf expressions bit-for-bit
//   * k_mean          reproduces np.mean's pairwise order bit-for-bit
//   * k_syrk / k_spatial_modes use fp64 FMA (MFMA) -- tolerance-level parity
//   * the DFT (podsgen_dft.hip) uses the host's twiddle table, bit-exact
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "podsgen_kernels.h"

namespace pods {

// Snapshot matrix layout ("K-tiled"): element (snapshot i, row r of the reference A) lives at
// AT[((r / 16) * ns + i) * 16 + r % 16].  A K-tile of 16 rows of A for a panel of snapshots
// i0..i0+n is then one contiguous block (SYRK operand = one 16 KB chunk per 128 snapshots).
__device__ __forceinline__ int64_t at_off(int64_t r, int64_t i, int ns) {
  return (((r >> 4) * ns + i) << 4) + (r & 15);
}

// -----------------------------------------------------------------------------------------
// MT19937
// -----------------------------------------------------------------------------------------
static constexpr int MTN = 624;
static constexpr uint32_t MT_A = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return c ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// One full twist of an LDS state by a 256-thread workgroup (three dependency phases:
// [0,227) reads old words, [227,454) and [454,623) read words written one phase earlier).
__device__ void twist_block256(uint32_t* st) {
  const int t = threadIdx.x;
  uint32_t v = 0;
  if (t < 227) v = mt_mix(st[t], st[t + 1], st[t + 397]);
  __syncthreads();
  if (t < 227) st[t] = v;
  __syncthreads();
  if (t < 227) v = mt_mix(st[227 + t], st[228 + t], st[t]);
  __syncthreads();
  if (t < 227) st[227 + t] = v;
  __syncthreads();
  if (t < 169) v = mt_mix(st[454 + t], st[455 + t], st[227 + t]);
  __syncthreads();
  if (t < 169) st[454 + t] = v;
  __syncthreads();
  if (t == 0) st[623] = mt_mix(st[623], st[0], st[396]);
  __syncthreads();
}

// The same twist by one wavefront (64 lanes): read everything of a phase, then write.
__device__ void twist_wave(uint32_t* st, int lane) {
  uint32_t v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = lane + 64 * r;
    if (i < 227) v[r] = mt_mix(st[i], st[i + 1], st[i + 397]);
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = lane + 64 * r;
    if (i < 227) st[i] = v[r];
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 227 + lane + 64 * r;
    if (i < 454) v[r] = mt_mix(st[i], st[i + 1], st[i - 227]);
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 227 + lane + 64 * r;
    if (i < 454) st[i] = v[r];
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int i = 454 + lane + 64 * r;
    if (i < 623) v[r] = mt_mix(st[i], st[i + 1], st[i - 227]);
  }
  wave_sync();
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int i = 454 + lane + 64 * r;
    if (i < 623) st[i] = v[r];
  }
  wave_sync();
  if (lane == 0) st[623] = mt_mix(st[623], st[0], st[396]);
  wave_sync();
}

// Jump-ahead: dst = g(F) src by block Horner over 32 blocks of 624 coefficients,
//   acc <- twist(acc) ^ sum_r c_{624q+r} window_r(x),  x = (src, twist(src)),
// with the coefficients taken three at a time (a sliding-window table): for each 3-bit
// pattern p, Y_p[k] = XOR_{i in p} x[k + i] is built once per job, so the three windows of
// coefficients r, r+1, r+2 cost ONE LDS read (Y_p[r + w]) instead of one per set bit (a
// per-bit version took 1.19 against 0.89 ms at C3).  Pattern 0 is a row of zeros, so every
// group reads unconditionally and the 24 reads of an 8-group chunk are independent.  XOR is
// exact and order-free.  LDS 47 KB: three workgroups per CU.
__global__ __launch_bounds__(256) void k_mt_jump3(const uint32_t* __restrict__ src_base,
                                                  const int* __restrict__ src_idx,
                                                  const uint32_t* __restrict__ polys,
                                                  const int* __restrict__ poly_idx,
                                                  uint32_t* __restrict__ dst_base,
                                                  const int* __restrict__ dst_idx, int njobs) {
  constexpr int YS = 2 * MTN;  // row stride of the pattern table (indices r + w <= 1246)
  __shared__ uint32_t x[2 * MTN];
  __shared__ uint32_t Y[8 * YS];
  __shared__ uint32_t acc[MTN];
  __shared__ uint32_t g[MTN];
  const int job = blockIdx.x;
  if (job >= njobs) return;
  const uint32_t* s = src_base + (size_t)src_idx[job] * MTN;
  const uint32_t* gsrc = polys + (size_t)poly_idx[job] * MTN;
  for (int i = threadIdx.x; i < MTN; i += 256) {
    const uint32_t v = s[i];
    x[i] = v;
    x[MTN + i] = v;
    acc[i] = 0u;
    g[i] = gsrc[i];
  }
  __syncthreads();
  twist_block256(x + MTN);
  // Y_p[k] for k < 2N (entries past x's end read as zero; they are never used)
  for (int k = threadIdx.x; k < YS; k += 256) {
    const uint32_t a = x[k];
    const uint32_t b = k + 1 < YS ? x[k + 1] : 0u;
    const uint32_t c = k + 2 < YS ? x[k + 2] : 0u;
    Y[0 * YS + k] = 0u;
    Y[1 * YS + k] = a;
    Y[2 * YS + k] = b;
    Y[3 * YS + k] = a ^ b;
    Y[4 * YS + k] = c;
    Y[5 * YS + k] = a ^ c;
    Y[6 * YS + k] = b ^ c;
    Y[7 * YS + k] = a ^ b ^ c;
  }
  __syncthreads();
  const int w0 = threadIdx.x, w1 = threadIdx.x + 256, w2 = threadIdx.x + 512;
  const bool has2 = w2 < MTN;
  const int w2c = has2 ? w2 : w0;  // a valid address for the lanes past the state
  for (int q = 31; q >= 0; --q) {
    if (q != 31) twist_block256(acc);
    uint32_t v0 = 0, v1 = 0, v2 = 0;
    // 26 chunks of 24 coefficients (8 groups of 3) cover r in [0, 624)
    for (int rb = 0; rb < MTN; rb += 24) {
      const int off = q * MTN + rb;
      const int wi = off >> 5, sh = off & 31;
      uint32_t bits = g[wi] >> sh;
      if (sh && wi + 1 < MTN) bits |= g[wi + 1] << (32 - sh);
      bits = __builtin_amdgcn_readfirstlane(bits);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t* Yp = Y + ((bits >> (3 * u)) & 7u) * YS + rb + 3 * u;
        v0 ^= Yp[w0];
        v1 ^= Yp[w1];
        v2 ^= Yp[w2c];
      }
    }
    acc[w0] ^= v0;
    acc[w1] ^= v1;
    if (has2) acc[w2] ^= v2;
    __syncthreads();
  }
  uint32_t* d = dst_base + (size_t)dst_idx[job] * MTN;
  for (int i = threadIdx.x; i < MTN; i += 256) d[i] = acc[i];
}

// Substream generator: one wavefront per substream g, Bs blocks of 624 words from state
// mt^(g*Bs).  Double D of the stream (2 words) -> uniform(low, low+range), written to the
// slab buffer when its padded row lies in [rlo, rhi) of its plane.
__global__ __launch_bounds__(256) void k_mt_generate(const uint32_t* __restrict__ states, int G,
                                                     int64_t Bs, int64_t ntot, int64_t S, int Kp,
                                                     int rlo, int rhi, int64_t Sl, double low,
                                                     double range, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t mts[4][MTN];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = blockIdx.x * 4 + wave;
  if (g >= G) return;
  uint32_t* mt = mts[wave];
  const uint32_t* src = states + (size_t)g * MTN;
  for (int i = lane; i < MTN; i += 64) mt[i] = src[i];
  wave_sync();
  const int64_t D0 = (int64_t)g * Bs * 312;
  // per-lane position of double D0 + lane: plane q, padded row, column -- advanced
  // incrementally (one 64-bit division per substream instead of one per double)
  const int rows_pp = (int)(S / Kp);
  int64_t q = (D0 + lane) / S;
  int o = (int)((D0 + lane) - q * S);
  int row = o / Kp, col = o - (o / Kp) * Kp;
  for (int64_t b = 0; b < Bs; ++b) {
    const int64_t Db = D0 + b * 312;
    if (Db >= ntot) break;
    twist_wave(mt, lane);
    int64_t qq = q;
    int rr = row, cc = col;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int d = lane + 64 * r;
      if (d < 312 && Db + d < ntot) {
        const uint2 w = reinterpret_cast<const uint2*>(mt)[d];
        const uint32_t a = mt_temper(w.x) >> 5, bb = mt_temper(w.y) >> 6;
        const double u = ((double)a * 67108864.0 + (double)bb) / 9007199254740992.0;
        const double val = low + range * u;
        if (rr >= rlo && rr < rhi) out[qq * Sl + (int64_t)(rr - rlo) * Kp + cc] = val;
      }
      cc += 64;
      while (cc >= Kp) {
        cc -= Kp;
        if (++rr == rows_pp) {
          rr = 0;
          ++qq;
        }
      }
    }
    wave_sync();
    col += 312;
    while (col >= Kp) {
      col -= Kp;
      if (++row == rows_pp) {
        row = 0;
        ++q;
      }
    }
  }
}

// One twist cur -> nxt by 227 threads with ONE barrier after it (instead of one per phase):
// thread t produces nxt[t], nxt[227+t] and nxt[454+t] (t < 169) in a register chain -- each
// later phase reads exactly the word the same thread made one phase earlier -- and thread 0
// also nxt[623] = mix(cur[623], nxt[0], nxt[396]), recomputing nxt[169] and nxt[396] (made
// by thread 169) from cur.  Same words as the in-place sequential twist.
__device__ __forceinline__ void twist_chain(const uint32_t* __restrict__ cur, uint32_t* __restrict__ nxt, int t) {
  if (t >= 227) return;
  const uint32_t a = mt_mix(cur[t], cur[t + 1], cur[t + 397]);
  nxt[t] = a;
  const uint32_t b = mt_mix(cur[227 + t], cur[228 + t], a);
  nxt[227 + t] = b;
  if (t < 169) nxt[454 + t] = mt_mix(cur[454 + t], cur[455 + t], b);
  if (t == 0) {
    const uint32_t n169 = mt_mix(cur[169], cur[170], cur[566]);
    const uint32_t n396 = mt_mix(cur[396], cur[397], n169);
    nxt[623] = mt_mix(cur[623], a, n396);
  }
}

// Whole-plane generator (one GPU: the slab holds every row, so double D of the stream goes to
// out[D]).  One 256-thread workgroup per substream; the state is double-buffered in LDS, so
// the twist producing block b (cur -> nxt, twist_chain) and the tempering + 16-B stores of
// block b-1 (reading cur) run side by side: one barrier per 624-word block, four waves per
// substream to hide the LDS and store latency.
__global__ __launch_bounds__(256) void k_mt_generate_full(const uint32_t* __restrict__ states, int G,
                                                          int64_t Bs, int64_t ntot, double low,
                                                          double range, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[2][MTN];
  const int t = threadIdx.x;
  // (a grid smaller than G would take the substreams in turn; spreading the generation over
  // 64-256 workgroups beside the SYRK measured 46-77 ms against 2.4: each substream is a
  // latency-bound twist chain, so the substreams must run side by side)
  for (int g = blockIdx.x; g < G; g += gridDim.x) {
  __syncthreads();  // the previous substream's last tempering read buf
  for (int i = t; i < MTN; i += 256) buf[0][i] = states[(size_t)g * MTN + i];
  __syncthreads();
  const int64_t D0 = (int64_t)g * Bs * 312;
  int64_t nb = (ntot - D0 + 311) / 312;
  nb = nb < Bs ? nb : Bs;
  // iteration b: nxt = twist(cur) = state of block b (if b < nb); temper cur = block b-1 (b >= 1)
  for (int64_t b = 0; b <= nb; ++b) {
    const uint32_t* cur = buf[b & 1];
    uint32_t* nxt = buf[(b + 1) & 1];
    const bool tw = b < nb;
    if (tw) twist_chain(cur, nxt, t);
    if (b >= 1 && t < 156) {
      const uint4 w = reinterpret_cast<const uint4*>(cur)[t];
      const uint32_t a0 = mt_temper(w.x) >> 5, b0 = mt_temper(w.y) >> 6;
      const uint32_t a1 = mt_temper(w.z) >> 5, b1 = mt_temper(w.w) >> 6;
      const double u0 = ((double)a0 * 67108864.0 + (double)b0) / 9007199254740992.0;
      const double u1 = ((double)a1 * 67108864.0 + (double)b1) / 9007199254740992.0;
      const int64_t D = D0 + (b - 1) * 312 + 2 * t;
      if (D + 1 < ntot)
        *reinterpret_cast<double2*>(out + D) = make_double2(low + range * u0, low + range * u1);
      else if (D < ntot)
        out[D] = low + range * u0;
    }
    if (!tw) break;
    __syncthreads();  // nxt complete; cur (tempered above) becomes the next nxt
  }
  }
}

// Row-slab generator (multi-GPU: this rank's rows [rlo, rhi) of every padded plane, the
// 2nfy halo included).  Same structure as k_mt_generate_full; every substream still twists
// through all of its blocks (the stream is sequential), but blocks with no double in the
// slab skip the tempering, conversion and stores -- at 8 ranks that is ~85% of them.
// Double D of the stream: plane q = D / S, offset o = D % S, row o / Kp; it goes to
// out[q * Sl + o - rlo * Kp] when rlo <= row < rhi.  Needs S >= 312 (a block spans at most
// two planes).
__global__ __launch_bounds__(256) void k_mt_generate_slab(const uint32_t* __restrict__ states, int G,
                                                          int64_t Bs, int64_t ntot, int64_t S, int Kp,
                                                          int rlo, int rhi, int64_t Sl, double low,
                                                          double range, double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[2][MTN];
  const int t = threadIdx.x;
  for (int g = blockIdx.x; g < G; g += gridDim.x) {
  __syncthreads();
  for (int i = t; i < MTN; i += 256) buf[0][i] = states[(size_t)g * MTN + i];
  __syncthreads();
  const int64_t D0 = (int64_t)g * Bs * 312;
  int64_t nb = (ntot - D0 + 311) / 312;
  nb = nb < Bs ? nb : Bs;
  const int64_t olo = (int64_t)rlo * Kp, ohi = (int64_t)rhi * Kp;  // slab offsets within a plane
  // plane and offset of the current block's first double, advanced by 312 per block
  int64_t q0 = D0 / S, o0 = D0 - (D0 / S) * S;
  for (int64_t b = 0; b <= nb; ++b) {
    const uint32_t* cur = buf[b & 1];
    uint32_t* nxt = buf[(b + 1) & 1];
    const bool tw = b < nb;
    if (tw) twist_chain(cur, nxt, t);
    if (b >= 1) {
      // block b-1 spans offsets [o0, o0 + 312) of plane q0 (wrapping into plane q0 + 1)
      const int64_t e0 = o0 + 311;
      const bool any = (o0 < ohi && e0 >= olo) || (e0 >= S && e0 - S >= olo);
      if (any && t < 156) {
        const uint4 w = reinterpret_cast<const uint4*>(cur)[t];
        const uint32_t a0 = mt_temper(w.x) >> 5, b0 = mt_temper(w.y) >> 6;
        const uint32_t a1 = mt_temper(w.z) >> 5, b1 = mt_temper(w.w) >> 6;
        const double u0 = ((double)a0 * 67108864.0 + (double)b0) / 9007199254740992.0;
        const double u1 = ((double)a1 * 67108864.0 + (double)b1) / 9007199254740992.0;
        const int64_t Db = D0 + (b - 1) * 312 + 2 * t;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          int64_t q = q0, o = o0 + 2 * t + h;
          if (o >= S) {
            o -= S;
            ++q;
          }
          if (Db + h < ntot && o >= olo && o < ohi) out[q * Sl + o - olo] = low + range * (h ? u1 : u0);
        }
      }
      o0 += 312;
      if (o0 >= S) {
        o0 -= S;
        ++q0;
      }
    }
    if (!tw) break;
    __syncthreads();  // nxt complete; cur (tempered above) becomes the next nxt
  }
  }
}

// Chains of the stream for the multi-GPU state exchange (r5; pods_df_set_exchange).  Chain c
// starts from the 624-word state st0 + c * 624 (the state before the twist that makes its first
// block b0[c]) and runs nb[c] blocks, with the double-buffered LDS twist of k_mt_generate_slab.
//   RECORD (an owner rank's own substreams): before the twist of block b, the state is copied
//     to rec_out + 624 * slot for every record (b, slot) of the chain (rec_first[c] ..
//     rec_first[c+1], sorted by block) -- the start state of another rank's row segment;
//   STORE (a rank's own row segments, one chain per plane): the doubles of the chain's blocks
//     whose padded row lies in [rlo, rhi) of their plane go to out[q Sl + o - rlo Kp], exactly
//     as in k_mt_generate_slab (bit for bit the same doubles).
// So no rank twists the whole stream: each twists its 1/N share once and the ~12 K segment
// starts of every rank (2.5 KB each) travel in one all_to_all.
template <bool RECORD, bool STORE>
__global__ __launch_bounds__(256) void k_mt_chains(const uint32_t* __restrict__ st0, const int64_t* __restrict__ b0,
                                                   const int* __restrict__ nbk, int nchains,
                                                   const int64_t* __restrict__ rec_block,
                                                   const int* __restrict__ rec_slot, const int* __restrict__ rec_first,
                                                   uint32_t* __restrict__ rec_out, int64_t ntot, int64_t S, int Kp,
                                                   int rlo, int rhi, int64_t Sl, double low, double range,
                                                   double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[2][MTN];
  const int t = threadIdx.x;
  for (int c = blockIdx.x; c < nchains; c += gridDim.x) {
    __syncthreads();  // the previous chain's last tempering / record read buf
    for (int i = t; i < MTN; i += 256) buf[0][i] = st0[(size_t)c * MTN + i];
    __syncthreads();
    const int64_t bb = b0[c];
    const int64_t nb = nbk[c];
    const int64_t D0 = bb * 312;
    const int64_t olo = (int64_t)rlo * Kp, ohi = (int64_t)rhi * Kp;
    int64_t q0 = STORE ? D0 / S : 0, o0 = STORE ? D0 - (D0 / S) * S : 0;
    int ri = RECORD ? rec_first[c] : 0;
    const int re = RECORD ? rec_first[c + 1] : 0;
    for (int64_t b = 0; b <= nb; ++b) {
      const uint32_t* cur = buf[b & 1];
      uint32_t* nxt = buf[(b + 1) & 1];
      const bool tw = b < nb;
      if constexpr (RECORD) {
        // cur is the state before block bb + b's twist
        while (ri < re && rec_block[ri] == bb + b) {
          uint32_t* dst = rec_out + (size_t)rec_slot[ri] * MTN;
          for (int i = t; i < MTN; i += 256) dst[i] = cur[i];
          ++ri;
        }
      }
      if (tw) twist_chain(cur, nxt, t);
      if constexpr (STORE) {
        if (b >= 1) {
          const int64_t e0 = o0 + 311;
          const bool any = (o0 < ohi && e0 >= olo) || (e0 >= S && e0 - S >= olo);
          if (any && t < 156) {
            const uint4 w = reinterpret_cast<const uint4*>(cur)[t];
            const uint32_t a0 = mt_temper(w.x) >> 5, c0 = mt_temper(w.y) >> 6;
            const uint32_t a1 = mt_temper(w.z) >> 5, c1 = mt_temper(w.w) >> 6;
            const double u0 = ((double)a0 * 67108864.0 + (double)c0) / 9007199254740992.0;
            const double u1 = ((double)a1 * 67108864.0 + (double)c1) / 9007199254740992.0;
            const int64_t Db = D0 + (b - 1) * 312 + 2 * t;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              int64_t q = q0, o = o0 + 2 * t + h;
              if (o >= S) {
                o -= S;
                ++q;
              }
              if (Db + h < ntot && o >= olo && o < ohi) out[q * Sl + o - olo] = low + range * (h ? u1 : u0);
            }
          }
          o0 += 312;
          if (o0 >= S) {
            o0 -= S;
            ++q0;
          }
        }
      }
      if (!tw) break;
      __syncthreads();  // nxt complete; cur (tempered / recorded above) becomes the next nxt
    }
  }
}

hipError_t launch_mt_chains(int mode, const uint32_t* st0, const int64_t* b0, const int* nb, int nchains,
                            const int64_t* rec_block, const int* rec_slot, const int* rec_first, uint32_t* rec_out,
                            int64_t ntot, int64_t S, int Kp, int rlo, int rhi, int64_t Sl, double low, double range,
                            double* out, hipStream_t st) {
  if (nchains <= 0) return hipSuccess;
  if (mode == 0)
    hipLaunchKernelGGL((k_mt_chains<true, false>), dim3(nchains), dim3(256), 0, st, st0, b0, nb, nchains, rec_block,
                       rec_slot, rec_first, rec_out, ntot, S, Kp, rlo, rhi, Sl, low, range, out);
  else
    hipLaunchKernelGGL((k_mt_chains<false, true>), dim3(nchains), dim3(256), 0, st, st0, b0, nb, nchains, rec_block,
                       rec_slot, rec_first, rec_out, ntot, S, Kp, rlo, rhi, Sl, low, range, out);
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// separable filter
// -----------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t stream_plane(int c, int p, int NX) {
  return p < NX ? (int64_t)c * NX + p : (int64_t)3 * NX + 3 * (int64_t)(p - NX) + c;
}

// x pass: t1[c][i][pt] = sum_a x[c][plane i+a][pt] * bx[NX-1-a], a ascending, acc from 0.
// One thread per (component, padded slab point), sliding register window over the steps.
template <int NX>
__global__ __launch_bounds__(256) void k_filter_x(const double* __restrict__ R,
                                                  const double* __restrict__ bx, int ns,
                                                  int64_t Sl, int steps_per_chunk,
                                                  double* __restrict__ T1) {
  const int64_t pt = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (pt >= Sl) return;
  const int i0 = blockIdx.z * steps_per_chunk;
  const int i1 = min(ns, i0 + steps_per_chunk);
  if (i0 >= i1) return;
  double b[NX];
#pragma unroll
  for (int a = 0; a < NX; ++a) b[a] = bx[NX - 1 - a];
  double w[NX];
#pragma unroll
  for (int a = 0; a < NX - 1; ++a) w[a] = R[stream_plane(c, i0 + a, NX) * Sl + pt];
  for (int i = i0; i < i1; ++i) {
    w[NX - 1] = R[stream_plane(c, i + NX - 1, NX) * Sl + pt];
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < NX; ++a) acc = acc + w[a] * b[a];
    T1[((int64_t)c * ns + i) * Sl + pt] = acc;
#pragma unroll
    for (int a = 0; a < NX - 1; ++a) w[a] = w[a + 1];
  }
}

// The same x pass on two adjacent points per thread (16-B loads and stores; Sl even, so every
// plane starts 16-B aligned).  Per point the arithmetic is identical to k_filter_x.  The plane
// that enters the window at step i is loaded PD steps ahead (a register queue), so each wave
// keeps PD loads in flight instead of waiting for one load per step (the compiler issued the
// step's load and then drained vmcnt(0) before its last tap).
template <int NX, int PD, bool NT = false>
__global__ __launch_bounds__(256) void k_filter_x2(const double* __restrict__ R,
                                                   const double* __restrict__ bx, int ns,
                                                   int64_t Sl, int steps_per_chunk,
                                                   double* __restrict__ T1, int nbx, int ncomp, int nch,
                                                   int s0, int s1) {
  // virtual blocks (point block, component, step chunk), one per workgroup
  const int nvb = nbx * ncomp * nch;
  for (int vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
  const int bxi = vb % nbx, c = (vb / nbx) % ncomp, bz = vb / (ncomp * nbx);
  const int64_t pp = (int64_t)bxi * 256 + threadIdx.x;  // point pair
  if (2 * pp >= Sl) continue;
  const int i0 = s0 + bz * steps_per_chunk;  // steps [s0, s1) of the ns (a chunk of the generation)
  const int i1 = min(s1, i0 + steps_per_chunk);
  if (i0 >= i1) continue;
  double b[NX];
#pragma unroll
  for (int a = 0; a < NX; ++a) b[a] = bx[NX - 1 - a];
  const int64_t Sl2 = Sl >> 1;
  const double2* R2 = reinterpret_cast<const double2*>(R);
  double2* T2 = reinterpret_cast<double2*>(T1);
  double2 w[NX];
  // NT (A/B): nontemporal plane loads and T1 stores (each byte is touched once here)
  typedef double f64x2_nt __attribute__((ext_vector_type(2)));
  auto ldR = [&](int64_t idx) -> double2 {
    if constexpr (NT) {
      const f64x2_nt v = __builtin_nontemporal_load(reinterpret_cast<const f64x2_nt*>(R2 + idx));
      return make_double2(v.x, v.y);
    } else {
      return R2[idx];
    }
  };
#pragma unroll
  for (int a = 0; a < NX - 1; ++a) w[a] = ldR(stream_plane(c, i0 + a, NX) * Sl2 + pp);
  // pf[d] = the plane entering the window at step i + d (planes up to i1 + NX - 2 exist)
  double2 pf[PD];
#pragma unroll
  for (int d = 0; d < PD; ++d)
    pf[d] = i0 + d < i1 ? ldR(stream_plane(c, i0 + d + NX - 1, NX) * Sl2 + pp) : make_double2(0.0, 0.0);
  for (int i = i0; i < i1; ++i) {
    w[NX - 1] = pf[0];
#pragma unroll
    for (int d = 0; d < PD - 1; ++d) pf[d] = pf[d + 1];
    if (i + PD < i1) pf[PD - 1] = ldR(stream_plane(c, i + PD + NX - 1, NX) * Sl2 + pp);
    double ax = 0.0, ay = 0.0;
#pragma unroll
    for (int a = 0; a < NX; ++a) {
      ax = ax + w[a].x * b[a];
      ay = ay + w[a].y * b[a];
    }
    if constexpr (NT)
      __builtin_nontemporal_store((f64x2_nt){ax, ay}, reinterpret_cast<f64x2_nt*>(T2 + ((int64_t)c * ns + i) * Sl2 + pp));
    else T2[((int64_t)c * ns + i) * Sl2 + pp] = make_double2(ax, ay);
#pragma unroll
    for (int a = 0; a < NX - 1; ++a) w[a] = w[a + 1];
  }
  }
}

// y + z passes, Lund transform, rotation, snapshot store.
// Block = (tile of TJ output rows, step i), 512 threads.  Per component: the y pass streams
// YR-row groups of one padded column through registers (b ascending, the scipy order) into
// LDS t2; the z pass gives each thread 16 consecutive outputs of one row from a register
// window of 16+NZ-1 t2 values (cc ascending).  t2 rows are padded by one double per 16 so the
// window reads are LDS-bank-conflict-free.  The three components' results stay in registers
// for the Lund transform (digitalfilters.py:174-176 / :227-229) and the rotation, and each
// thread stores its 16 consecutive snapshot rows as one 128-B line (K-tiled layout).
// lund_sj: 0 when the profile does not vary with j (the 1-D profiles of adapt1d): the table
// (9 rows of K) is staged in LDS per block.  Otherwise (2-D profiles) it is in the chunk-major
// layout of lund_chunk_index (built once by pods_df_configure).
__device__ __forceinline__ int kpad(int k) { return k + (k >> 4); }

// NZC: compile-time z width (0: runtime NZ <= 25, the generic instance)
template <int TJ, int NY, int NZC, int NT>
__global__ __launch_bounds__(NT) void k_filter_yz(
    const double* __restrict__ T1, const double* __restrict__ by, const double* __restrict__ bz,
    int NZr, int ns, int jl, int K, int Kp, int64_t Sl, int ncomp,
    const double* __restrict__ lund, int64_t lund_sj, int lund_mode, const double* __restrict__ rot,
    int rotate, double* __restrict__ AT, int nsb, int KB, int s0, int s1) {
  extern __shared__ __attribute__((aligned(16))) double t2[];  // TJ x ldt
  constexpr int YR = TJ < 16 ? TJ : 16;  // rows per y-pass item
  constexpr int NZMAX = NZC > 0 ? NZC : 25;
  const int NZ = NZC > 0 ? NZC : NZr;
  constexpr int WIN = 16 + NZMAX - 1;
  // (An XCD-aware renumbering of the blocks, so the row tiles of one step group share an L2,
  // cut the HBM traffic 18.4 -> 14.5 GB at C3 at the same time and made C4 ~4 ms slower.)
  int tile_x = blockIdx.x, group_y = blockIdx.y, tile_z = blockIdx.z;
  if (lund_sj != 0) {
    // j-varying Lund table (2-D profiles): the blocks of one (row, column) tile run their step
    // groups back to back on ONE XCD (dispatch deals consecutive blocks round-robin over the 8
    // XCDs), so the tile's 295 KB of Lund parameters stay in that XCD's L2
    const int ntx = gridDim.x, ngy = gridDim.y;
    const int total = ntx * ngy * gridDim.z;
    const int b = blockIdx.x + ntx * (blockIdx.y + ngy * blockIdx.z);
    const int xcd = b & 7, qq = total >> 3, rr = total & 7;
    const int logical = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
    const int tile = logical / ngy;
    group_y = logical - tile * ngy;
    tile_x = tile % ntx;
    tile_z = tile / ntx;
  }
  // column tile: outputs [k0, k0 + Kt) of the K axis from padded columns [k0, k0 + Kpt)
  // (KB = K: one tile; wider inlets are cut into 256-column tiles, so every shape runs the
  // 16-row x 256-thread configuration with a z halo of (NZ - 1) / KB)
  const int k0 = tile_z * KB;
  const int Kt = min(KB, K - k0);
  const int Kpt = Kt + NZ - 1;
  const int ldt = kpad(KB + NZ - 1 + 16) + 1;
  const int jt = tile_x * TJ;
  const int tid0 = threadIdx.x;
  const int rows = min(TJ, jl - jt);
  const int64_t Pl = (int64_t)jl * K;
  const int kch = (Kt + 15) >> 4;      // 16-wide output chunks per row
  const int zitems = TJ * kch;         // <= NT (host guarantees)
  double byr[NY];
#pragma unroll
  for (int b = 0; b < NY; ++b) byr[b] = by[NY - 1 - b];
  double bzr[NZMAX];
#pragma unroll
  for (int cc = 0; cc < NZMAX; ++cc) bzr[cc] = cc < NZ ? bz[NZ - 1 - cc] : 0.0;
  // A Lund table that does not vary along j (lund_sj == 0) is staged once per block in LDS
  // (9 rows of K, padded like t2) and read conflict-free by the 16-wide output chunks.
  const bool lsh = lund_sj == 0 && lund_mode >= 0;
  const int ldl = kpad(KB) + 1;
  double* lt = t2 + (size_t)TJ * ldt;
  if (lsh) {
    const int ne = lund_mode == 1 ? 9 : 7;
    for (int e = 0; e < ne; ++e)
      for (int k = tid0; k < Kt; k += NT) lt[e * ldl + kpad(k)] = lund[(int64_t)e * Pl + k0 + k];
  }
  // NSB consecutive steps per block: each thread's stores for one snapshot-row group then
  // land on consecutive 128-B lines of the K-tiled layout (steps are contiguous there)
  const int ib = s0 + group_y * nsb;  // steps [s0, s1) of the ns
  const int ie = min(s1, ib + nsb);
#pragma clang loop unroll(disable)
  for (int i = ib; i < ie; ++i) {
    // the Lund table pointer is re-materialised per step: otherwise the (step-invariant)
    // parameter loads are hoisted out of the loop and spill
    int zero = 0;
    asm volatile("" : "+s"(zero));
    const double* lund_i = lund + zero;
    const double* T1i = T1 + zero;
    const double* roti = rot + zero;
    int tid = tid0;
    asm volatile("" : "+v"(tid));
    const int zr = tid / kch, zk0 = (tid - (tid / kch) * kch) * 16;
    const bool zact = tid < zitems && zr < rows;
    double res[3][16];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      // ncomp is 3 (generator) or 1 (pods_filter_block): the unrolled body is guarded
      if (c < ncomp) {
      const double* src = T1i + ((int64_t)c * ns + i) * Sl + (int64_t)jt * Kp + k0;
      // main items: (column, YR-row group) for the first cmain columns, one per thread;
      // the remaining halo columns as single-output mini items spread over all threads
      // (2*Kp items on NT threads would leave a few threads a second full item)
      constexpr int GRP = TJ / YR;
      const int cmain = min(Kpt, NT / GRP);
      for (int it = tid; it < GRP * cmain; it += NT) {
        const int grp = it / cmain, col = it - grp * cmain;
        const int r0 = grp * YR;
        if (r0 >= rows) continue;
        // all rows of the column first (clamped to the tile, so every load is in bounds and
        // they issue back to back), then the taps
        double v[YR + NY - 1];
        const int rmax = rows + NY - 2 - r0;
#pragma unroll
        for (int r = 0; r < YR + NY - 1; ++r)
          v[r] = src[(int64_t)(r0 + min(r, rmax)) * Kp + col];
        double acc[YR];
#pragma unroll
        for (int jj = 0; jj < YR; ++jj) acc[jj] = 0.0;
#pragma unroll
        for (int r = 0; r < YR + NY - 1; ++r) {
#pragma unroll
          for (int jj = 0; jj < YR; ++jj) {
            const int b = r - jj;
            if (b >= 0 && b < NY) acc[jj] = acc[jj] + v[r] * byr[b];
          }
        }
#pragma unroll
        for (int jj = 0; jj < YR; ++jj)
          if (r0 + jj < rows) t2[(r0 + jj) * ldt + kpad(col)] = acc[jj];
      }
      for (int it = tid; it < (Kpt - cmain) * TJ; it += NT) {
        const int col = cmain + it / TJ, jj = it - (it / TJ) * TJ;
        if (jj >= rows) continue;
        double v[NY];
#pragma unroll
        for (int b = 0; b < NY; ++b) v[b] = src[(int64_t)(jj + b) * Kp + col];
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < NY; ++b) acc = acc + v[b] * byr[b];
        t2[jj * ldt + kpad(col)] = acc;
      }
      __syncthreads();
      if (zact) {
        const double* rowp = t2 + zr * ldt;
        double w[WIN];
#pragma unroll
        for (int e = 0; e < WIN; ++e) w[e] = (e < 16 + NZ - 1) ? rowp[kpad(zk0 + e)] : 0.0;
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          double acc = 0.0;
#pragma unroll
          for (int cc = 0; cc < NZMAX; ++cc)
            if (cc < NZ) acc = acc + w[kk + cc] * bzr[cc];
          res[c][kk] = acc;
        }
      }
      __syncthreads();
      }
    }
    if (zact) {
    double R9[9];
    if (rotate) {
#pragma unroll
      for (int e = 0; e < 9; ++e) R9[e] = roti[e];
    }
    const int j = jt + zr;
    const int64_t p0 = (int64_t)j * K + k0 + zk0;
    // j-varying table: chunk-major layout (lund_chunk_index), one coalesced 16-B load per
    // (parameter, output pair)
    const int QC = (K + 15) >> 4;
    const double2* L2 = reinterpret_cast<const double2*>(lund_i) + (int64_t)j * 9 * 8 * QC + ((k0 + zk0) >> 4);
    // the Lund transform / rotation overwrite res in place
    double (&out)[3][16] = res;
    double2 pp[9];
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (lund_mode < 0) continue;
      double prm[9];
      if (lsh) {
        const double* L = lt + kpad(zk0 + kk);
#pragma unroll
        for (int e = 0; e < 9; ++e) prm[e] = (e < 7 || lund_mode == 1) ? L[e * ldl] : 0.0;
      } else {
        if ((kk & 1) == 0) {
#pragma unroll
          for (int e = 0; e < 9; ++e)
            pp[e] = (e < 7 || lund_mode == 1) ? L2[((int64_t)e * 8 + (kk >> 1)) * QC] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) prm[e] = (kk & 1) ? pp[e].y : pp[e].x;
      }
      const double xu = res[0][kk], xv = res[1][kk], xw = res[2][kk];
      const double a00 = prm[0], a10 = prm[1], a11 = prm[2];
      const double a20 = prm[3], a21 = prm[4], a22 = prm[5];
      // digitalfilters.py:174-176 (adapt1d) / :227-229 (adapt2prf), left to right, zero terms kept
      double u = ((a00 * xu + 0.0 * xv) + 0.0 * xw) + prm[6];
      double v = (a10 * xu + a11 * xv) + 0.0 * xw;
      double ww = (a20 * xu + a21 * xv) + a22 * xw;
      if (lund_mode == 1) {
        v = v + prm[7];
        ww = ww + prm[8];
      }
      if (rotate) {  // rotate_velocity :1119-1131: numpy R.dot(V) -> OpenBLAS dgemv, whose
                     // 3-term row dot is fma(R2, w, fma(R0, u, R1*v)) (pinned by golden rot case)
        const double ur = __builtin_fma(R9[2], ww, __builtin_fma(R9[0], u, R9[1] * v));
        const double vr = __builtin_fma(R9[5], ww, __builtin_fma(R9[3], u, R9[4] * v));
        const double wr = __builtin_fma(R9[8], ww, __builtin_fma(R9[6], u, R9[7] * v));
        u = ur;
        v = vr;
        ww = wr;
      }
      out[0][kk] = u;
      out[1][kk] = v;
      out[2][kk] = ww;
    }
    const int nk = min(16, Kt - zk0);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c >= ncomp) break;
      const int64_t r0 = c * Pl + p0;
      if (nk == 16 && (r0 & 15) == 0) {
        // one full 128-B line of the K-tiled layout
        double2* dst = reinterpret_cast<double2*>(AT + at_off(r0, i, ns));
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = make_double2(out[c][2 * e], out[c][2 * e + 1]);
      } else {
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
          if (kk < nk) AT[at_off(r0 + kk, i, ns)] = out[c][kk];
      }
    }
    }
  }
}

// Stand-alone Lund transform + rotation on one step's (yu, yv, yw) fields (the operator API
// adapt1d / adapt2prf / rotate_velocity called on their own); same expressions as k_filter_yz.
__global__ void k_lund_apply(double* __restrict__ yu, double* __restrict__ yv, double* __restrict__ yw,
                             int64_t P, const double* __restrict__ lund, int lund_mode,
                             const double* __restrict__ rot, int rotate) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  double u = yu[p], v = yv[p], w = yw[p];
  if (lund_mode >= 0) {
    const double xu = u, xv = v, xw = w;
    const double a00 = lund[0 * P + p], a10 = lund[1 * P + p], a11 = lund[2 * P + p];
    const double a20 = lund[3 * P + p], a21 = lund[4 * P + p], a22 = lund[5 * P + p];
    u = ((a00 * xu + 0.0 * xv) + 0.0 * xw) + lund[6 * P + p];
    v = (a10 * xu + a11 * xv) + 0.0 * xw;
    w = (a20 * xu + a21 * xv) + a22 * xw;
    if (lund_mode == 1) {
      v = v + lund[7 * P + p];
      w = w + lund[8 * P + p];
    }
  }
  if (rotate) {
    const double ur = __builtin_fma(rot[2], w, __builtin_fma(rot[0], u, rot[1] * v));
    const double vr = __builtin_fma(rot[5], w, __builtin_fma(rot[3], u, rot[4] * v));
    const double wr = __builtin_fma(rot[8], w, __builtin_fma(rot[6], u, rot[7] * v));
    u = ur;
    v = vr;
    w = wr;
  }
  yu[p] = u;
  yv[p] = v;
  yw[p] = w;
}

hipError_t launch_lund_apply(double* yu, double* yv, double* yw, int64_t P, const double* lund,
                             int lund_mode, const double* rot, int rotate, hipStream_t st) {
  hipLaunchKernelGGL(k_lund_apply, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, yu, yv, yw, P, lund,
                     lund_mode, rot, rotate);
  return hipGetLastError();
}

// -----------------------------------------------------------------------------------------
// mean over snapshots: numpy pairwise program (leaf = (start,len), add = (-1, 0))
// -----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mean(const double* __restrict__ AT, int64_t rowlen,
                                              int ns, const int* __restrict__ prog, int nprog,
                                              double* __restrict__ mean,
                                              unsigned long long* __restrict__ devmax) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool valid = r < rowlen;
  // devmax: the largest |fl(a - mean)| (the int8 correlation's scale, podsgen_corr_i8.hip) from
  // the row's extremes -- rounding is monotonic, so fl(max - mean) bounds every fl(a - mean)
  double mx = -__builtin_huge_val(), mn = __builtin_huge_val(), dev = 0.0;
  if (valid) {
    double stk[40];
    int sp = 0;
    for (int op = 0; op < nprog; ++op) {
      const int s = prog[2 * op], n = prog[2 * op + 1];
      if (s < 0) {
        const double bsum = stk[--sp];
        stk[sp - 1] = stk[sp - 1] + bsum;
        continue;
      }
      const double* a = AT + at_off(r, s, ns);  // consecutive snapshots are 16 doubles apart
      auto ld = [&](int64_t k) -> double {
        const double x = a[k];
        mx = fmax(mx, x);
        mn = fmin(mn, x);
        return x;
      };
      double res;
      if (n < 8) {
        res = 0.0;
        for (int i = 0; i < n; ++i) res = res + ld((int64_t)i * 16);
      } else {
        double r0 = ld(0), r1 = ld(16), r2 = ld(32), r3 = ld(48);
        double r4 = ld(64), r5 = ld(80), r6 = ld(96), r7 = ld(112);
        int i = 8;
        // two iterations' 16 loads in flight per wave (the adds keep numpy's order)
#pragma unroll 2
        for (; i < n - (n % 8); i += 8) {
          const int64_t b = (int64_t)i * 16;
          r0 = r0 + ld(b);
          r1 = r1 + ld(b + 16);
          r2 = r2 + ld(b + 32);
          r3 = r3 + ld(b + 48);
          r4 = r4 + ld(b + 64);
          r5 = r5 + ld(b + 80);
          r6 = r6 + ld(b + 96);
          r7 = r7 + ld(b + 112);
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < n; ++i) res = res + ld((int64_t)i * 16);
      }
      stk[sp++] = res;
    }
    const double mu = (0.0 + stk[0]) / (double)ns;
    mean[r] = mu;
    dev = fmax(mx - mu, mu - mn);
  }
  if (devmax) {
    unsigned long long u = (unsigned long long)__double_as_longlong(dev > 0.0 ? dev : 0.0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long v = __shfl_xor(u, o);
      u = v > u ? v : u;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(devmax, u);
  }
}

// The same mean with the leaves spread over threads (r5): k_mean walks a row's whole program in
// one thread (3 waves per SIMD at C3, each a chain of 256 dependent load groups plus a scratch
// stack: latency-bound at ~5.3 TB/s).  Here a 256-thread block takes 16 rows; thread (row rl,
// lane lg) sums leaves lg, lg + 16, ... of its row with k_mean's exact leaf arithmetic into LDS,
// and one thread per row then replays the program over those leaf sums (stack in LDS) -- the
// same additions in the same order, so the mean is bit-identical.  The leaves (start, length)
// follow the program in prog (upload_mean_program); nleaf <= 256.
template <int LN>
__global__ __launch_bounds__(16 * LN) void k_mean_leaves(const double* __restrict__ AT, int64_t rowlen, int ns,
                                                     const int* __restrict__ prog, int nprog, int nleaf,
                                                     double* __restrict__ mean,
                                                     unsigned long long* __restrict__ devmax) {
  extern __shared__ __attribute__((aligned(16))) double ml[];
  double* vals = ml;                        // [16][nleaf]
  double* mxs = ml + 16 * nleaf;            // [16][LN]
  double* mns = mxs + 16 * LN;              // [16][LN]
  double* stk = mns + 16 * LN;              // [16][32]
  const int rl = threadIdx.x & 15, lg = threadIdx.x >> 4;
  const int64_t r = (int64_t)blockIdx.x * 16 + rl;
  const bool valid = r < rowlen;
  const int* leaves = prog + 2 * nprog;
  double mx = -__builtin_huge_val(), mn = __builtin_huge_val();
  if (valid) {
    for (int lf = lg; lf < nleaf; lf += LN) {
      const int s = leaves[2 * lf], n = leaves[2 * lf + 1];
      const double* a = AT + at_off(r, s, ns);
      auto ld = [&](int64_t k) -> double {
        const double x = a[k];
        mx = fmax(mx, x);
        mn = fmin(mn, x);
        return x;
      };
      double res;
      if (n < 8) {
        res = 0.0;
        for (int i = 0; i < n; ++i) res = res + ld((int64_t)i * 16);
      } else {
        double r0 = ld(0), r1 = ld(16), r2 = ld(32), r3 = ld(48);
        double r4 = ld(64), r5 = ld(80), r6 = ld(96), r7 = ld(112);
        int i = 8;
#pragma unroll 2
        for (; i < n - (n % 8); i += 8) {
          const int64_t b = (int64_t)i * 16;
          r0 = r0 + ld(b);
          r1 = r1 + ld(b + 16);
          r2 = r2 + ld(b + 32);
          r3 = r3 + ld(b + 48);
          r4 = r4 + ld(b + 64);
          r5 = r5 + ld(b + 80);
          r6 = r6 + ld(b + 96);
          r7 = r7 + ld(b + 112);
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < n; ++i) res = res + ld((int64_t)i * 16);
      }
      vals[rl * nleaf + lf] = res;
    }
  }
  mxs[rl * LN + lg] = mx;
  mns[rl * LN + lg] = mn;
  __syncthreads();
  double dev = 0.0;
  if (lg == 0 && valid) {
    double* st = stk + rl * 32;
    int sp = 0, k = 0;
    for (int op = 0; op < nprog; ++op) {
      if (prog[2 * op] < 0) {
        const double bsum = st[--sp];
        st[sp - 1] = st[sp - 1] + bsum;
      } else {
        st[sp++] = vals[rl * nleaf + k++];
      }
    }
    const double mu = (0.0 + st[0]) / (double)ns;
    mean[r] = mu;
    for (int q = 0; q < LN; ++q) {
      mx = fmax(mx, mxs[rl * LN + q]);
      mn = fmin(mn, mns[rl * LN + q]);
    }
    dev = fmax(mx - mu, mu - mn);
  }
  if (devmax && threadIdx.x < 64) {  // the 16 row threads are lanes 0-15 of wave 0
    unsigned long long u = (unsigned long long)__double_as_longlong(dev > 0.0 ? dev : 0.0);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long v = __shfl_xor(u, o);
      u = v > u ? v : u;
    }
    if (threadIdx.x == 0) atomicMax(devmax, u);
  }
}

// main() :1492-1495 (A[:, j] = A[:, j] - mean_field) in place on the K-tiled snapshot matrix:
// element f of AT belongs to row r = (f / (16 ns)) * 16 + f % 16.  Two doubles per thread.
// The subtraction is the one the SYRK and the spatial-mode kernels would otherwise repeat
// per fragment read, so their results are unchanged bit for bit.
__global__ __launch_bounds__(256) void k_center(double* __restrict__ AT, int64_t npairs, int ns,
                                                const double* __restrict__ mean) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= npairs) return;
  const int64_t f = 2 * q;
  const int64_t r = (f / ((int64_t)ns << 4)) * 16 + (f & 15);
  double2* p = reinterpret_cast<double2*>(AT) + q;
  const double2 v = *p;
  *p = make_double2(v.x - mean[r], v.y - mean[r + 1]);
}

// -----------------------------------------------------------------------------------------
// correlation SYRK on fp64 MFMA (v_mfma_f64_16x16x4_f64)
// C[i][j] = sum_r (A_T[i][r]-m[r]) (A_T[j][r]-m[r]), lower-triangle tiles, mirrored.
// -----------------------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void glds16(const void* src, uint32_t lds_byte_addr) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)lds_byte_addr,
                                   16, 0, 0);
}


// Split-K SYRK: one 128 x 128 tile of the lower triangle per 256-thread workgroup, TWO
// workgroups per CU.  Operands are streamed by LDS-DMA (global_load_lds_dwordx4) into a
// 2-stage ring (66.5 KB per workgroup); counted vmcnt + raw s_barrier keep the next K-tile in
// flight across the barrier.  The two workgroups' K-tile barriers are independent, so one keeps
// the fp64 MFMA pipe fed while the other waits at its barrier (one 512-thread 256 x 128
// workgroup per CU stalled all 8 waves at every barrier: 53.0 against 50.8 ms at C3).  The
// K-tiled A makes each (panel, K-tile) operand one contiguous block; rows are XOR-swizzled on
// the SOURCE address (double2 slot j of row R holds logical slot j ^ ((R>>1)&7)) so the MFMA
// fragment reads are bank-conflict free.  CENTRED = 1: A was centred in place (k_center), so
// the fragments go to the MFMAs as read; CENTRED = 0 subtracts the mean slot at fragment read
// (57.0 against 52.9 ms).  4 waves as 2 x 2, each 64 x 64 = 4 x 4 blocks of
// v_mfma_f64_16x16x4_f64.  Partial tiles go to slab `split`; k_syrk_reduce sums the slabs in
// split order (deterministic).
template <int KT_, int NST_>
struct SyrkCfg {
  static constexpr int BM = 128, BN = 128, KT = KT_, NST = NST_, NW = 4;
  static constexpr int XB = BM * KT * 8;            // X panel bytes per stage
  static constexpr int YB = BN * KT * 8;            // Y panel bytes per stage
  static constexpr int MBYTES = NW * KT * 8;        // mean slice (CENTRED = 0)
  static constexpr int STAGE = XB + YB + MBYTES;
  static constexpr int XP = XB / 1024 / NW;         // 1 KB LDS-DMA instructions per wave
  static constexpr int YP = YB / 1024 / NW;
  static constexpr int SLOTS = KT / 2;              // 16-B slots per row
  static constexpr int RPI = 64 / SLOTS;            // rows per 1 KB instruction
  static constexpr int SWZ = SLOTS - 1;             // swizzle mask
  static constexpr int RSH = KT == 16 ? 1 : 2;      // row bits that pick the swizzle
};

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int CENTRED, int KT, int NST, int OCC>
__global__ __launch_bounds__(256, OCC) void k_syrk_g128(const double* __restrict__ AT, int ns,
                                                        int64_t Kdim, const double* __restrict__ mean,
                                                        const int4* __restrict__ items, int nitems,
                                                        int64_t ksplit, double* __restrict__ work,
                                                        int64_t ldc, int64_t slab) {
  using Cf = SyrkCfg<KT, NST>;
  constexpr int XB = Cf::XB, YB = Cf::YB, STAGE = Cf::STAGE, XP = Cf::XP, YP = Cf::YP;
  constexpr int SLOTS = Cf::SLOTS, RPI = Cf::RPI, SWZ = Cf::SWZ, RSH = Cf::RSH;
  constexpr int Q = XP + YP + (CENTRED ? 0 : 1);    // DMA instructions per wave per K-tile
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int b = blockIdx.x;
  const int xcd = b & 7, qq = nitems >> 3, rr = nitems & 7;
  const int logical = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (b >> 3);
  const int4 it = items[logical];
  const int bi = it.x, bj = it.y, sp = it.z;
  const int i0 = bi * Cf::BM, j0 = bj * Cf::BN;
  const int64_t kt0 = (int64_t)sp * (ksplit / KT);
  const int64_t kt1 = min(Kdim, (int64_t)(sp + 1) * ksplit) / KT;
  const int nt = (int)(kt1 - kt0);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
  const int lrow = lane / SLOTS, lslot = lane % SLOTS;
  // K-tiled A: a K-tile of KT rows of one snapshot is KT contiguous doubles inside its 16-row
  // group (KT = 8: the half `hk` of the group)
  int64_t xsrc[XP], ysrc[YP];
#pragma unroll
  for (int q = 0; q < XP; ++q) {
    const int R = (wave * XP + q) * RPI + lrow;
    xsrc[q] = ((int64_t)min(i0 + R, ns - 1) << 4) + ((lslot ^ ((R >> RSH) & SWZ)) << 1);
  }
#pragma unroll
  for (int q = 0; q < YP; ++q) {
    const int R = (wave * YP + q) * RPI + lrow;
    ysrc[q] = ((int64_t)min(j0 + R, ns - 1) << 4) + ((lslot ^ ((R >> RSH) & SWZ)) << 1);
  }
  const int64_t blk = (int64_t)ns << 4;
  auto issue = [&](int t) {
    const int64_t kt = kt0 + t;
    const uint32_t base = lds0 + (uint32_t)((t % NST) * STAGE);
    const double* g = AT + ((kt * KT) >> 4) * blk + ((kt * KT) & 15);
#pragma unroll
    for (int q = 0; q < XP; ++q) glds16(g + xsrc[q], base + (wave * XP + q) * 1024);
#pragma unroll
    for (int q = 0; q < YP; ++q) glds16(g + ysrc[q], base + XB + (wave * YP + q) * 1024);
    if (!CENTRED && lane < KT / 2) glds16(mean + kt * KT + (lane << 1), base + XB + YB + wave * KT * 8);
  };
  f64x4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = (f64x4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (t < nt) issue(t);
  const int fr = lane & 15, fk = lane >> 4, fs = (fr >> RSH) & SWZ;
  const int xrow = (wr * 64 + fr) * KT, yrow = (wc * 64 + fr) * KT;
  for (int t = 0; t < nt; ++t) {
    // K-tile t landed (K-tiles t+1 .. t+NST-2 may still be in flight); after the barrier every
    // wave has also finished reading stage (t-1) % NST, which K-tile t+NST-1 now overwrites
    if (t + NST - 2 < nt) wait_vmcnt<Q * (NST - 2)>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (t + NST - 1 < nt) issue(t + NST - 1);
    const char* st = smem + (t % NST) * STAGE;
    const double* Xs = reinterpret_cast<const double*>(st);
    const double* Ys = reinterpret_cast<const double*>(st + XB);
    const double* Ms = reinterpret_cast<const double*>(st + XB + YB + wave * KT * 8);
#pragma unroll
    for (int kk = 0; kk < KT; kk += 4) {
      const int k = kk + fk;
      const int koff = ((((k >> 1) ^ fs)) << 1) + (k & 1);
      const double mk = CENTRED ? 0.0 : Ms[k];
      double a[4], bv[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = CENTRED ? Xs[xrow + koff + m * 16 * KT] : Xs[xrow + koff + m * 16 * KT] - mk;
#pragma unroll
      for (int n = 0; n < 4; ++n) bv[n] = CENTRED ? Ys[yrow + koff + n * 16 * KT] : Ys[yrow + koff + n * 16 * KT] - mk;
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], bv[n], acc[m][n], 0, 0, 0);
    }
  }
  double* dst = work + (int64_t)sp * slab;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int gi = i0 + wr * 64 + m * 16 + fk + 4 * reg;
        const int gj = j0 + wc * 64 + n * 16 + fr;
        if (gi < ns && gj <= gi) dst[(int64_t)gi * ldc + gj] = acc[m][n][reg];
      }
}

// C[i][j] = (sum_s part_s[max][min]) [/ ns], splits summed in order.
// Sum of the split-K slabs (split order: v = ((p0 + p1) + p2) + ...) over 64x64 tiles of the
// lower triangle; each tile is written to C and, through LDS, transposed into the upper
// triangle, so every global access is row-contiguous.
__global__ __launch_bounds__(256) void k_syrk_reduce(const double* __restrict__ part, int nsplit,
                                                     int64_t slab, int ns, int64_t ldc,
                                                     double* __restrict__ C, int divide) {
  __shared__ double tile[64][65];
  // linear lower-triangle tile index -> (ti >= tj)
  const int L = blockIdx.x;
  int ti = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
  while ((ti + 1) * (ti + 2) / 2 <= L) ++ti;
  while (ti * (ti + 1) / 2 > L) --ti;
  const int tj = L - ti * (ti + 1) / 2;
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  const double dn = (double)ns;
  // the thread's 16 rows advance through the slabs together: 16 independent loads per slab
  // keep the memory pipe full (a per-element chain over the slabs would be latency bound)
  double v[16];
  int64_t off[16];
  bool ok[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int r = r0 + 4 * q;
    const int i = ti * 64 + r, j = tj * 64 + c;
    ok[q] = i < ns && j < ns && (ti > tj || c <= r);
    off[q] = ok[q] ? (int64_t)i * ldc + j : 0;
    v[q] = ok[q] ? part[off[q]] : 0.0;
  }
  for (int sp = 1; sp < nsplit; ++sp) {
    const double* ps = part + (int64_t)sp * slab;
    double t[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) t[q] = ok[q] ? ps[off[q]] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) v[q] = v[q] + t[q];
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    if (ok[q]) {
      if (divide) v[q] = v[q] / dn;
      C[off[q]] = v[q];
    }
    tile[r0 + 4 * q][c] = ok[q] ? v[q] : 0.0;
  }
  __syncthreads();
#pragma unroll 4
  for (int r = r0; r < 64; r += 4) {
    // upper element (tj*64 + r, ti*64 + c) = lower element (ti*64 + c, tj*64 + r)
    const int i = tj * 64 + r, j = ti * 64 + c;
    const bool ok = i < ns && j < ns && (ti > tj || r < c);
    if (ok) C[(int64_t)i * ldc + j] = tile[c][r];
  }
}

// 1/lambda (np.ones(nm)/energy, PODFS.py:1331): IEEE division, as numpy's
__global__ void k_recip(const double* __restrict__ x, int n, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = 1.0 / x[i];
}

hipError_t launch_recip(const double* x, int n, double* y, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_recip, dim3((n + 255) / 256), dim3(256), 0, st, x, n, y);
  return hipGetLastError();
}

__global__ void k_divide(double* __restrict__ x, int64_t n, double d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] / d;
}

// -----------------------------------------------------------------------------------------
// temporal modes: descending reorder + PODFS.py:1323-1325 scaling
// -----------------------------------------------------------------------------------------
// Python's builtin sum(T[:, j]**2) is one sequential chain (PODFS.py:1324): the squares are
// formed in parallel into LDS (coalescing the strided column), then lane 0 runs the chain with
// its LDS reads issued eight ahead.  One workgroup per column.
constexpr int TMAG_MAX = 8192;
__global__ __launch_bounds__(256) void k_temporal_mag(const double* __restrict__ V, int64_t v_rs,
                                                      int64_t v_cs, int ns, int ncols,
                                                      double* __restrict__ mag) {
  __shared__ __attribute__((aligned(16))) double sq[TMAG_MAX];
  const int j = blockIdx.x;
  if (j >= ncols) return;
  const double* col = V + (int64_t)(ns - 1 - j) * v_cs;
  for (int i0 = 0; i0 < ns; i0 += TMAG_MAX) {
    const int n = min(TMAG_MAX, ns - i0);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 256) {
      const double x = col[(int64_t)(i0 + i) * v_rs];
      sq[i] = x * x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = i0 == 0 ? 0.0 : mag[j];
      int i = 0;
      for (; i + 8 <= n; i += 8) {
        const double2 a = *reinterpret_cast<const double2*>(sq + i);
        const double2 b = *reinterpret_cast<const double2*>(sq + i + 2);
        const double2 c = *reinterpret_cast<const double2*>(sq + i + 4);
        const double2 d = *reinterpret_cast<const double2*>(sq + i + 6);
        s = s + a.x; s = s + a.y; s = s + b.x; s = s + b.y;
        s = s + c.x; s = s + c.y; s = s + d.x; s = s + d.y;
      }
      for (; i < n; ++i) s = s + sq[i];
      mag[j] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) mag[j] = mag[j] / (double)ns;
}

__global__ void k_temporal_scale(const double* __restrict__ V, int64_t v_rs, int64_t v_cs, int ns,
                                 int ncols, int nvalid, const double* __restrict__ lam,
                                 const double* __restrict__ mag, double* __restrict__ T) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= ncols) return;
  double x = V[(int64_t)i * v_rs + (int64_t)(ns - 1 - j) * v_cs];
  if (j < nvalid) x = x * sqrt(lam[j] / mag[j]);
  T[(int64_t)i * ncols + j] = x;
}

// -----------------------------------------------------------------------------------------
// spatial modes Phi[r][m] = ((sum_i (A_T[i][r]-m_r) T[i][m]) * (1/lambda_m)) / ns
// (PODFS.py:1330-1333).  Each thread owns two adjacent rows (one 16-B load per snapshot from
// the K-tiled layout), the snapshot axis is split into KS chunks (blockIdx.y) so the launch
// holds enough loads in flight to stream A at HBM rate, and the loads run one 8-snapshot
// group ahead of the FMAs.  T is staged through LDS (broadcast reads).  KS > 1 writes
// partial sums part[ks][r][m] that k_spatial_reduce folds in a fixed order.
// -----------------------------------------------------------------------------------------
// r6: 4 snapshots per load group (142 VGPRs, 3 waves per SIMD) instead of 8 (210, 2 waves): 1.28 vs
// 1.31 ms for pods_spatial_modes at C3, Phi bit-identical; 128- or 256-snapshot T chunks, 16 per
// group, 3 waves forced at 8, and the next chunk's first group loaded across the chunk barriers
// measured equal or slower (profiles/r6/spatial_variants_ab.log; variant builds: -DPODS_SPATIAL_*)
#ifndef PODS_SPATIAL_U
#define PODS_SPATIAL_U 4
#endif
#ifndef PODS_SPATIAL_CH
#define PODS_SPATIAL_CH 64
#endif
#ifndef PODS_SPATIAL_WPE
#define PODS_SPATIAL_WPE 1
#endif
template <int NMB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PODS_SPATIAL_WPE))) void k_spatial_modes(const double* __restrict__ AT, int64_t rowlen,
                                                       int ns, const double* __restrict__ mean,
                                                       const double* __restrict__ T, int ldT, int col0,
                                                       int nm, const double* __restrict__ inv_lam,
                                                       double* __restrict__ phi, int ldphi, int chunk,
                                                       double* __restrict__ part) {
  constexpr int CH = PODS_SPATIAL_CH, U = PODS_SPATIAL_U;
  __shared__ __attribute__((aligned(16))) double Ts[CH][NMB];
  const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  const int64_t rowpad = (rowlen + 15) & ~(int64_t)15;
  const bool valid = r < rowpad;
  const double m0 = r < rowlen ? mean[r] : 0.0;
  const double m1 = r + 1 < rowlen ? mean[r + 1] : 0.0;
  const int i0 = blockIdx.y * chunk;
  const int i1 = min(ns, i0 + chunk);
  double acc0[NMB], acc1[NMB];
#pragma unroll
  for (int m = 0; m < NMB; ++m) acc0[m] = acc1[m] = 0.0;
  const double* base = AT + (valid ? at_off(r, 0, ns) : 0);
  for (int c0 = i0; c0 < i1; c0 += CH) {
    const int lim = min(CH, i1 - c0);
    __syncthreads();
    for (int e = threadIdx.x; e < CH * NMB; e += 256) {
      const int ii = e / NMB, m = e % NMB;
      Ts[ii][m] = (ii < lim && m < nm) ? T[(int64_t)(c0 + ii) * ldT + col0 + m] : 0.0;
    }
    __syncthreads();
    if (!valid) continue;
    const double2* src = reinterpret_cast<const double2*>(base + (int64_t)c0 * 16);
    double2 cur[U], nxt[U];
    // The loads past lim re-read the chunk's last snapshot and are zeroed where they are used
    // (r5), and the groups alternate between two register sets within one loop iteration: with
    // the substitution at the load the compiler sank each prefetch load into its own branch,
    // and with a loop-carried prefetch its wait counts lost their order at the loop head -- in
    // both cases each group waited for its loads right after issuing them
    auto load = [&](double2 (&v)[U], int g0) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = src[min(g0 + u, lim - 1) * 8];
      __builtin_amdgcn_sched_barrier(0);  // issued here, not sunk next to their uses
    };
    auto group = [&](const double2 (&v)[U], int g0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = g0 + u < lim;  // zero past lim: Ts rows are 0 too
        const double a0 = in ? v[u].x - m0 : 0.0, a1 = in ? v[u].y - m1 : 0.0;
        const double* tr = Ts[(g0 + u) & (CH - 1)];
#pragma unroll
        for (int m = 0; m < NMB; m += 2) {
          const double2 tv = *reinterpret_cast<const double2*>(tr + m);
          acc0[m] = __builtin_fma(a0, tv.x, acc0[m]);
          acc1[m] = __builtin_fma(a1, tv.x, acc1[m]);
          acc0[m + 1] = __builtin_fma(a0, tv.y, acc0[m + 1]);
          acc1[m + 1] = __builtin_fma(a1, tv.y, acc1[m + 1]);
        }
      }
    };
    load(cur, 0);
    for (int g = 0; g < lim; g += 2 * U) {
      load(nxt, g + U);
      group(cur, g);
      load(cur, g + 2 * U);
      group(nxt, g + U);
    }
  }
  if (part) {
    if (!valid) return;
    double* pp = part + ((int64_t)blockIdx.y * rowpad + r) * NMB;
#pragma unroll
    for (int m = 0; m < NMB; m += 2) {
      *reinterpret_cast<double2*>(pp + m) = make_double2(acc0[m], acc0[m + 1]);
      *reinterpret_cast<double2*>(pp + NMB + m) = make_double2(acc1[m], acc1[m + 1]);
    }
    return;
  }
  // Phi rows leave through LDS, a quarter of the block (128 rows) at a time, so the stores of
  // the block's (512 rows x nm) region are contiguous (a thread's own 2 x nm values would be
  // scattered 8-B stores, 2 nm * 8 B apart from lane to lane)
  __shared__ double ph[128 * NMB];
  const double dn = (double)ns;
  const int64_t rb0 = (int64_t)blockIdx.x * 512;
  for (int h = 0; h < 4; ++h) {
    __syncthreads();
    if ((threadIdx.x >> 6) == h) {
      const int lr = 2 * (threadIdx.x & 63);
#pragma unroll
      for (int m = 0; m < NMB; ++m) {
        if (m < nm) {
          ph[lr * NMB + m] = (acc0[m] * inv_lam[col0 + m]) / dn;
          ph[(lr + 1) * NMB + m] = (acc1[m] * inv_lam[col0 + m]) / dn;
        }
      }
    }
    __syncthreads();
    const int64_t r0 = rb0 + 128 * h;
    const int nr = (int)(rowlen - r0 < 128 ? rowlen - r0 : 128);
    for (int e = threadIdx.x; e < nr * nm; e += 256) {
      const int lr = e / nm, m = e - lr * nm;
      phi[(r0 + lr) * ldphi + col0 + m] = ph[lr * NMB + m];
    }
  }
}

__global__ __launch_bounds__(256) void k_spatial_reduce(const double* __restrict__ part, int ks, int nmb,
                                                        int64_t rowlen, int col0, int nm,
                                                        const double* __restrict__ inv_lam, int ns,
                                                        double* __restrict__ phi, int ldphi) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = e / nm;
  const int m = (int)(e - r * nm);
  if (r >= rowlen) return;
  const int64_t rowpad = (rowlen + 15) & ~(int64_t)15;
  double s = 0.0;
  for (int k = 0; k < ks; ++k) s += part[((int64_t)k * rowpad + r) * nmb + m];
  phi[r * ldphi + col0 + m] = (s * inv_lam[col0 + m]) / (double)ns;
}

// -----------------------------------------------------------------------------------------
// launchers
// -----------------------------------------------------------------------------------------
hipError_t launch_mt_jump(const uint32_t* src, const int* src_idx, const uint32_t* polys,
                          const int* poly_idx, uint32_t* dst, const int* dst_idx, int njobs,
                          hipStream_t st) {
  if (njobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mt_jump3, dim3(njobs), dim3(256), 0, st, src, src_idx, polys, poly_idx, dst,
                     dst_idx, njobs);
  return hipGetLastError();
}

hipError_t launch_mt_generate(const uint32_t* states, int G, int64_t Bs, int64_t ntot, int64_t S,
                              int Kp, int rlo, int rhi, int64_t Sl, double low, double range,
                              double* out, hipStream_t st, int per_cu) {
  if (G <= 0) return hipSuccess;
  const int gw = G;
  // per_cu > 0: pad the whole-plane generator's LDS so that at most per_cu of its workgroups
  // share a CU (beside the late tridiagonalisation ranges, which must always find room)
  size_t pad = 0;
  if (per_cu > 0) {
    const size_t want = (160 * 1024) / (per_cu + 1) + 1024, have = 2 * MTN * sizeof(uint32_t);
    pad = want > have ? want - have : 0;
  }
  if (rlo == 0 && (int64_t)rhi * Kp == S && Sl == S && ((uintptr_t)out & 15) == 0 && Bs % 2 == 0) {
    // whole planes: out[D] for stream double D (even block starts keep the 16-B stores aligned)
    if (pad) {
      hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mt_generate_full),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_mt_generate_full, dim3(gw), dim3(256), pad, st, states, G, Bs, ntot, low, range, out);
    return hipGetLastError();
  }
  if (S >= 312) {
    hipLaunchKernelGGL(k_mt_generate_slab, dim3(gw), dim3(256), 0, st, states, G, Bs, ntot, S, Kp, rlo, rhi,
                       Sl, low, range, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_mt_generate, dim3((G + 3) / 4), dim3(256), 0, st, states, G, Bs, ntot, S, Kp,
                     rlo, rhi, Sl, low, range, out);
  return hipGetLastError();
}

template <int NX>
static hipError_t launch_fx(const double* R, const double* bx, int ns, int64_t Sl, int ncomp,
                            int chunk, double* T1, hipStream_t st, int s0, int s1, int max_grid) {
  if (Sl % 2 == 0 && ((uintptr_t)R & 15) == 0 && ((uintptr_t)T1 & 15) == 0) {
    const int nsr = s1 - s0;  // steps of this launch
    // point pairs: half the threads, so twice the step chunks keep the same parallelism
    // with PD loads in flight per wave, about four resident workgroups per CU suffice: step
    // chunks so the grid is one round of ~1024 workgroups (a partial second round of a
    // longer grid left most CUs idle at the end)
    (void)chunk;
    const int64_t bx_ = (Sl / 2 + 255) / 256;
    const int64_t want = 1024;
    const int64_t nch0 = std::max<int64_t>(1, std::min<int64_t>(nsr, want / std::max<int64_t>(1, bx_ * ncomp)));
    const int chunk2 = (int)((nsr + nch0 - 1) / nch0);
    const int nch = (nsr + chunk2 - 1) / chunk2;
    const int64_t nvb = bx_ * ncomp * nch;
    const int64_t grid = max_grid > 0 ? std::min<int64_t>(nvb, max_grid) : nvb;  // grid-stride over nvb
    // nontemporal plane loads / T1 stores: 8.15 vs 8.22 ms of main-stream generation at C3
    // (bench A/B, r4)
    hipLaunchKernelGGL((k_filter_x2<NX, 8, true>), dim3((unsigned)grid), dim3(256), 0, st, R, bx, ns, Sl, chunk2,
                       T1, (int)bx_, ncomp, nch, s0, s1);
    return hipGetLastError();
  }
  if (s0 != 0 || s1 != ns) return hipErrorInvalidValue;  // step ranges: the point-pair kernel only
  const int nch = (ns + chunk - 1) / chunk;
  dim3 grid((unsigned)((Sl + 255) / 256), (unsigned)ncomp, (unsigned)nch);
  hipLaunchKernelGGL(k_filter_x<NX>, grid, dim3(256), 0, st, R, bx, ns, Sl, chunk, T1);
  return hipGetLastError();
}

hipError_t launch_filter_x(int NX, const double* R, const double* bx, int ns, int64_t Sl, int ncomp,
                           int chunk, double* T1, hipStream_t st, int s0, int s1, int max_grid) {
  if (s1 < 0) s1 = ns;
  switch (NX) {
#define PODS_FX(n) \
  case n:          \
    return launch_fx<n>(R, bx, ns, Sl, ncomp, chunk, T1, st, s0, s1, max_grid);
    PODS_FX(1) PODS_FX(3) PODS_FX(5) PODS_FX(7) PODS_FX(9) PODS_FX(11) PODS_FX(13) PODS_FX(15)
    PODS_FX(17) PODS_FX(19) PODS_FX(21) PODS_FX(23) PODS_FX(25) PODS_FX(27) PODS_FX(29)
    PODS_FX(31) PODS_FX(33) PODS_FX(35) PODS_FX(37) PODS_FX(39) PODS_FX(41) PODS_FX(43)
    PODS_FX(45) PODS_FX(47) PODS_FX(49)
#undef PODS_FX
    default:
      return hipErrorInvalidValue;
  }
}

// y/z tile: 16 rows x 256 threads, 256-column tiles of K (one tile when K <= 256): two
// workgroups per CU (LDS ~58 KB each), so one block's loads overlap the other's filter
// arithmetic.  Measured alternatives at C3: a 32-row x 512-thread tile (smaller y halo, 97 KB of
// LDS, one block per CU) 12.2 against 11.2 ms of generation.  Wider inlets (C4, C5) used to
// take taller-than-wide tiles of the whole row (16 x 512 at K = 512, 8 x 512 at K = 1024:
// a 2.5x y halo on the T1 reads); they now run this same tile over 256-column slices.
constexpr int YZ_TJ = 16, YZ_NT = 256, YZ_KB = 256;

template <int NY, int NZC>
static hipError_t launch_fyz_t(const double* T1, const double* by, const double* bz, int NZ, int ns,
                               int jl, int K, int Kp, int64_t Sl, int ncomp, const double* lund,
                               int64_t lund_sj, int lund_mode, const double* rot, int rotate,
                               double* AT, hipStream_t st, int s0, int s1) {
  constexpr int TJ = YZ_TJ, NT = YZ_NT;
  const int nsr = s1 - s0;
  const int KB = std::min(K, YZ_KB);
  const int ldt = (KB + NZ - 1 + 16) + ((KB + NZ - 1 + 16) >> 4) + 1;
  const int ldl = KB + (KB >> 4) + 1;
  const size_t lds = ((size_t)TJ * ldt + (lund_sj == 0 ? 9 * (size_t)ldl : 0)) * sizeof(double);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_filter_yz<TJ, NY, NZC, NT>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  // enough blocks to fill the chip twice over, at most 16 steps each
  const int tiles = (jl + TJ - 1) / TJ;
  const int ktiles = (K + KB - 1) / KB;
  const int nsb = (int)std::max<int64_t>(1, std::min<int64_t>(16, (int64_t)tiles * ktiles * nsr / 512));
  const dim3 grid((unsigned)tiles, (unsigned)((nsr + nsb - 1) / nsb), (unsigned)ktiles);
  hipLaunchKernelGGL((k_filter_yz<TJ, NY, NZC, NT>), grid, dim3(NT), lds, st, T1, by, bz, NZ, ns, jl, K,
                     Kp, Sl, ncomp, lund, lund_sj, lund_mode, rot, rotate, AT, nsb, KB, s0, s1);
  return hipGetLastError();
}

template <int NY>
static hipError_t launch_fyz(const double* T1, const double* by, const double* bz, int NZ, int ns,
                             int jl, int K, int Kp, int64_t Sl, int ncomp, const double* lund,
                             int64_t lund_sj, int lund_mode, const double* rot, int rotate,
                             double* AT, hipStream_t st, int s0, int s1) {
  if (NZ > 25) return hipErrorInvalidValue;
  if (NZ == NY)  // isotropic y/z widths: the z taps are compile-time too
    return launch_fyz_t<NY, NY>(T1, by, bz, NZ, ns, jl, K, Kp, Sl, ncomp, lund, lund_sj, lund_mode, rot,
                                rotate, AT, st, s0, s1);
  return launch_fyz_t<NY, 0>(T1, by, bz, NZ, ns, jl, K, Kp, Sl, ncomp, lund, lund_sj, lund_mode, rot, rotate,
                             AT, st, s0, s1);
}

hipError_t launch_filter_yz(int NY, const double* T1, const double* by, const double* bz, int NZ,
                            int ns, int jl, int K, int Kp, int64_t Sl, int ncomp,
                            const double* lund, int64_t lund_sj, int lund_mode, const double* rot,
                            int rotate, double* AT, hipStream_t st, int s0, int s1) {
  if (s1 < 0) s1 = ns;
  switch (NY) {
#define PODS_FYZ(n) \
  case n:           \
    return launch_fyz<n>(T1, by, bz, NZ, ns, jl, K, Kp, Sl, ncomp, lund, lund_sj, lund_mode, rot, rotate, AT, st, \
                         s0, s1);
    PODS_FYZ(1) PODS_FYZ(3) PODS_FYZ(5) PODS_FYZ(7) PODS_FYZ(9) PODS_FYZ(11) PODS_FYZ(13)
    PODS_FYZ(15) PODS_FYZ(17) PODS_FYZ(19) PODS_FYZ(21) PODS_FYZ(23) PODS_FYZ(25)
#undef PODS_FYZ
    default:
      return hipErrorInvalidValue;
  }
}

int filter_yz_max_K(int Kp) {
  (void)Kp;
  return 4096;  // 256-column tiles (the y/z kernel has no K limit; tested to K = 1024)
}

hipError_t launch_mean(const double* AT, int64_t rowlen, int ns, const int* prog, int nprog,
                       double* mean, hipStream_t st, double* devmax, int nleaf) {
  if (devmax) {
    const hipError_t e = hipMemsetAsync(devmax, 0, sizeof(double), st);
    if (e != hipSuccess) return e;
  }
  // default (r5): the leaves spread over threads when there are at least 2 (and <= 256); else one
  // thread per row (k_mean)
  if (nleaf >= 2 && nleaf <= 256) {
    // 16 leaf lanes per row (1.12-1.14 ms at C3; 32 lanes in 512-thread blocks 1.20, one thread
    // per row 1.23: profiles/r5/mean_ab.log)
    constexpr int LN = 16;
    const size_t lds = ((size_t)16 * nleaf + 2 * 16 * LN + 16 * 32) * sizeof(double);
    hipLaunchKernelGGL(k_mean_leaves<LN>, dim3((unsigned)((rowlen + 15) / 16)), dim3(16 * LN), lds, st, AT, rowlen,
                       ns, prog, nprog, nleaf, mean, reinterpret_cast<unsigned long long*>(devmax));
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_mean, dim3((unsigned)((rowlen + 255) / 256)), dim3(256), 0, st, AT, rowlen, ns,
                     prog, nprog, mean, reinterpret_cast<unsigned long long*>(devmax));
  return hipGetLastError();
}

hipError_t launch_center(double* AT, int64_t rowpad, int ns, const double* mean, hipStream_t st) {
  const int64_t npairs = rowpad * (int64_t)ns / 2;  // rowpad is a multiple of 16
  hipLaunchKernelGGL(k_center, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, st, AT, npairs, ns, mean);
  return hipGetLastError();
}

// Number of K splits for the 128 x 128 lower-triangle tiles on 512 concurrent workgroups
// (two per CU): ~8+ rounds, chosen to minimise the partial last round, >= 64 K-tiles of 16
// per item.
// SYRK configuration: K-tile 16, 2-stage ring, two workgroups per CU.  Measured at C3 against
// it (r3, tools/syrk_probe.py, same data): K-tile 8 with a 4-stage ring (prefetch distance 24
// instead of 16) 50.7 vs 48.8 ms, K-tile 8 / 3 stages / three workgroups per CU 49.5 ms,
// K-tile 8 / 3 stages / two per CU 49.8 ms -- the shorter K-tiles' extra barriers cost more
// than the deeper prefetch gains.  r4 (tools/syrk_ab.py, one call, 12 runs each): s_setprio(1)
// around each K-tile's MFMA cluster 49.28 vs 48.84 ms; no workgroup barrier at all -- every wave
// LDS-DMAs its own 64 X and 64 Y rows into a private ring (K-tile 8) and waits on its own
// vmcnt only -- 50.13 ms with 2 stages (two workgroups per CU; the L2 -> LDS traffic doubles)
// and 58.28 ms with 3 (one workgroup per CU).
#ifndef PODS_SYRK_KT  // compile-time overrides for A/B builds (tools/lib_variants.sh)
#define PODS_SYRK_KT 16
#define PODS_SYRK_NST 2
#define PODS_SYRK_OCC 2
#endif
constexpr int SYRK_KT = PODS_SYRK_KT, SYRK_NST = PODS_SYRK_NST, SYRK_OCC = PODS_SYRK_OCC;

int syrk_plan(int ns, int64_t Kdim, int64_t* ksplit) {
  constexpr int KT = 16;
  const int nb = (ns + 127) / 128;
  const int tiles = nb * (nb + 1) / 2, slots = 256 * SYRK_OCC;
  const int64_t kts = Kdim / KT;
  const int64_t maxsplit = std::max<int64_t>(1, kts / 64);
  int64_t best = 1;
  double best_cost = 1e300;
  for (int64_t s = 1; s <= std::min<int64_t>(maxsplit, 32); ++s) {
    const int64_t items = (int64_t)tiles * s;
    const double rounds = std::ceil((double)items / slots);
    // time ~ rounds * (work per item) + small per-split reduce cost
    const double cost = rounds / (double)s + 0.002 * s;
    if (cost < best_cost - 1e-12) {
      best_cost = cost;
      best = s;
    }
  }
  int64_t ks = (kts + best - 1) / best * KT;
  const int64_t nsplit = (Kdim + ks - 1) / ks;
  *ksplit = ks;
  return (int)std::max<int64_t>(1, nsplit);
}

hipError_t launch_syrk(const double* AT, int ns, int64_t Kdim, const double* mean, const int* items, int nitems,
                       int nsplit, int64_t ksplit, double* C, int64_t ldc, int divide, double* work, int centred,
                       hipStream_t st) {
  const int64_t slab = (int64_t)ns * ldc;
  auto launch = [&](auto kern, int lds) -> hipError_t {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(nitems), dim3(256), lds, st, AT, ns, Kdim, mean,
                       reinterpret_cast<const int4*>(items), nitems, ksplit, work, ldc, slab);
    return hipGetLastError();
  };
  constexpr int lds = SYRK_NST * SyrkCfg<SYRK_KT, SYRK_NST>::STAGE;
  hipError_t le = centred ? launch(k_syrk_g128<1, SYRK_KT, SYRK_NST, SYRK_OCC>, lds)
                          : launch(k_syrk_g128<0, SYRK_KT, SYRK_NST, SYRK_OCC>, lds);
  if (le != hipSuccess) return le;
  hipLaunchKernelGGL(k_syrk_reduce, dim3(((ns + 63) / 64) * ((ns + 63) / 64 + 1) / 2), dim3(256), 0, st, work,
                     nsplit, slab, ns, ldc, C, divide);
  return hipGetLastError();
}

hipError_t launch_divide(double* x, int64_t n, double d, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_divide, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, d);
  return hipGetLastError();
}

hipError_t launch_temporal(const double* V, int64_t v_rs, int64_t v_cs, int ns, int ncols,
                           int nvalid, const double* lam, double* mag, double* T, hipStream_t st) {
  hipLaunchKernelGGL(k_temporal_mag, dim3(ncols), dim3(256), 0, st, V, v_rs, v_cs, ns, ncols, mag);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_temporal_scale, dim3((ncols + 255) / 256, ns), dim3(256), 0, st, V, v_rs, v_cs,
                     ns, ncols, nvalid, lam, mag, T);
  return hipGetLastError();
}

int spatial_split(int64_t rowlen, int ns) {
  const int64_t blocks = ((rowlen + 15) / 16 * 16 / 2 + 255) / 256;
  int ks = 1;
  while (blocks * ks < 1536 && ks < 16 && ns / (ks * 2) >= 64) ks *= 2;
  return ks;
}

size_t spatial_work_bytes(int64_t rowlen, int ns) {
  const int ks = spatial_split(rowlen, ns);
  return ks > 1 ? (size_t)ks * ((rowlen + 15) / 16 * 16) * 32 * sizeof(double) : 0;
}

hipError_t launch_spatial(const double* AT, int64_t rowlen, int ns, const double* mean,
                          const double* T, int ldT, int nm, const double* inv_lam, double* phi,
                          double* work, hipStream_t st) {
  const int64_t rowpad = (rowlen + 15) / 16 * 16;
  const int ks = work ? spatial_split(rowlen, ns) : 1;
  const int chunk = ((ns + ks - 1) / ks + 7) / 8 * 8;
  const dim3 grid((unsigned)((rowpad / 2 + 255) / 256), (unsigned)ks);
  double* part = ks > 1 ? work : nullptr;
  for (int col0 = 0; col0 < nm; col0 += 32) {
    const int nb = nm - col0 < 32 ? nm - col0 : 32;
    const int nmb = nb <= 8 ? 8 : nb <= 16 ? 16 : nb <= 20 ? 20 : 32;
    if (nmb == 8)
      hipLaunchKernelGGL(k_spatial_modes<8>, grid, dim3(256), 0, st, AT, rowlen, ns, mean, T, ldT, col0,
                         nb, inv_lam, phi, nm, chunk, part);
    else if (nmb == 16)
      hipLaunchKernelGGL(k_spatial_modes<16>, grid, dim3(256), 0, st, AT, rowlen, ns, mean, T, ldT, col0,
                         nb, inv_lam, phi, nm, chunk, part);
    else if (nmb == 20)
      hipLaunchKernelGGL(k_spatial_modes<20>, grid, dim3(256), 0, st, AT, rowlen, ns, mean, T, ldT, col0,
                         nb, inv_lam, phi, nm, chunk, part);
    else
      hipLaunchKernelGGL(k_spatial_modes<32>, grid, dim3(256), 0, st, AT, rowlen, ns, mean, T, ldT, col0,
                         nb, inv_lam, phi, nm, chunk, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (part) {
      const int64_t tot = rowlen * nb;
      hipLaunchKernelGGL(k_spatial_reduce, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, part, ks,
                         nmb, rowlen, col0, nb, inv_lam, ns, phi, nm);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}


}  // namespace pods

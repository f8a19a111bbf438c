// Fourier-coefficient ranking and energy count on the device (PODFS.py:1575-1593).
//
// For mode i the reference forms cmod = abs(c[:, i]) (float32), orders the coefficients
// with sorted(zip(cmod, n), reverse=True) -- descending |c|, ties to the larger n -- and
// keeps the leading ones until a float64 running sum of cmod (Python 2 / numpy-1.x
// promotion) reaches float64(sum_f32(cmod)) * et.  Bit-exactness contract:
//   * |c| is numpy's complex64 absolute value (the SIMD loop of numpy >= 1.22:
//     larger * sqrt(fma(smaller/larger, smaller/larger, 1)), all float32) -- checked
//     against np.abs on the host in tests/test_gpu_parity.py;
//   * the float32 total replays numpy's pairwise summation program (the same program
//     k_mean uses, in float32);
//   * the running sum is sequential float64 in rank order.
// One 1024-thread workgroup per mode: keys (|c| bits << 32 | n) are bitonic-sorted in LDS.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "podsgen_kernels.h"

namespace pods {

// numpy's float32 complex absolute value.  The quotient and the square root are formed in
// float64 and rounded once to float32: with 53 >= 2*24 + 2 bits, that double rounding is
// innocuous for division and square root (Figueroa), i.e. equal to the correctly rounded
// float32 operations numpy's SIMD loop performs.
__device__ __forceinline__ float np_cabsf(float re, float im) {
  const float a = fabsf(re), b = fabsf(im);
  const float larger = fmaxf(a, b), smaller = fminf(b, a);
  if (isinf(larger)) return larger;
  const float ratio = (larger == 0.0f || isinf(smaller)) ? 0.0f : (float)((double)smaller / (double)larger);
  const float h2 = __builtin_fmaf(ratio, ratio, 1.0f);
  const float h = (float)__builtin_sqrt((double)h2);
  return h * larger;
}

constexpr int RANK_THREADS = 1024;

__global__ __launch_bounds__(RANK_THREADS) void k_rank(const float2* __restrict__ c, int ns, int nm,
                                                       int n2, double et, const int* __restrict__ prog,
                                                       int nprog, int32_t* __restrict__ c_ind,
                                                       int64_t* __restrict__ c_count) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];  // n2
  __shared__ float cm_sum;
  const int mode = blockIdx.x;
  const int t = threadIdx.x;
  for (int n = t; n < n2; n += RANK_THREADS) {
    unsigned long long k = 0ull;
    if (n < ns) {
      const float2 v = c[(int64_t)n * nm + mode];
      const float m = np_cabsf(v.x, v.y);
      k = ((unsigned long long)__float_as_uint(m) << 32) | (unsigned)n;
    }
    keys[n] = k;
  }
  __syncthreads();
  // numpy pairwise float32 sum of cmod in index order (one lane; 8-way ILP inside blocks)
  if (t == 0) {
    float stk[40];
    int sp = 0;
    for (int op = 0; op < nprog; ++op) {
      const int s = prog[2 * op], n = prog[2 * op + 1];
      if (s < 0) {
        const float b = stk[--sp];
        stk[sp - 1] = stk[sp - 1] + b;
        continue;
      }
      auto at = [&](int i) { return __uint_as_float((unsigned)(keys[s + i] >> 32)); };
      float res;
      if (n < 8) {
        res = 0.0f;
        for (int i = 0; i < n; ++i) res = res + at(i);
      } else {
        float r0 = at(0), r1 = at(1), r2 = at(2), r3 = at(3);
        float r4 = at(4), r5 = at(5), r6 = at(6), r7 = at(7);
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
          r0 = r0 + at(i);
          r1 = r1 + at(i + 1);
          r2 = r2 + at(i + 2);
          r3 = r3 + at(i + 3);
          r4 = r4 + at(i + 4);
          r5 = r5 + at(i + 5);
          r6 = r6 + at(i + 6);
          r7 = r7 + at(i + 7);
        }
        res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (; i < n; ++i) res = res + at(i);
      }
      stk[sp++] = res;
    }
    cm_sum = 0.0f + stk[0];
  }
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int p = t; p < n2 / 2; p += RANK_THREADS) {
        const int lo = 2 * p - (p & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const unsigned long long a = keys[lo], b = keys[hi];
        if ((a < b) == desc) {
          keys[lo] = b;
          keys[hi] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int n = t; n < ns; n += RANK_THREADS) c_ind[(int64_t)mode * ns + n] = (int32_t)(keys[n] & 0xffffffffull);
  if (t == 0) {
    const double target = (double)cm_sum * et;
    int64_t count = 0;
    if (target > 0.0) {
      double e = 0.0;
      count = -1;  // unreachable target (et > 1): the host raises like the reference's IndexError
      for (int k = 0; k < ns; ++k) {
        e = e + (double)__uint_as_float((unsigned)(keys[k] >> 32));
        if (e >= target) {
          count = k + 1;
          break;
        }
      }
    }
    c_count[mode] = count;
  }
}

int rank_max_ns() { return 16384; }

hipError_t launch_rank(const float* c, int ns, int nm, double et, const int* prog, int nprog,
                       int32_t* c_ind, int64_t* c_count, hipStream_t st) {
  if (ns <= 0 || nm <= 0) return hipSuccess;
  if (ns > rank_max_ns()) return hipErrorInvalidValue;
  int n2 = 2;
  while (n2 < ns) n2 <<= 1;
  const size_t lds = (size_t)n2 * sizeof(unsigned long long);
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rank),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_rank, dim3(nm), dim3(RANK_THREADS), lds, st, reinterpret_cast<const float2*>(c), ns,
                     nm, n2, et, prog, nprog, c_ind, c_count);
  return hipGetLastError();
}

}  // namespace pods

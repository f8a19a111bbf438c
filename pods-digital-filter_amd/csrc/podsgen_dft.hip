// Shifted direct DFT of the temporal modes (PODFS.py:1562-1571), bit-exact:
//
//   c[n, i] = (y * np.exp(-1j*2*k*np.pi*time/period)).sum() / ns,   k = n - ns//2,
//
// stored complex64.  The exponentials are NOT evaluated on the device: libm's sin/cos
// (glibc's, through numpy's complex exp) and OCML's differ in the last bit for a few
// arguments, and one flipped bit can reorder two coefficients of equal float32 modulus in the
// ranking (PODFS.py:1581).  The host evaluates the reference expression itself once per
// (ns, time axis) -- podsgen.host.dft_twiddles -- and uploads the table W[q][m] = (cos, sin);
// rows q < nk hold k = q, and for even ns row nk holds k = -ns/2 (n = 0).  Rows for k < 0
// are not stored: np.exp of the negated argument is the exact conjugate (checked on the host
// for every table, tests/test_host_cpu.py), so c[h - k] = conj(c[h + k]).
//
// Summation order: numpy's pairwise complex sum (cpairwise_program in podsgen_api.cpp):
// leaves of <= 64 complex values, each summed with numpy's 4-accumulator unrolled loop, then
// combined in the program's postfix order.  A workgroup owns one table row (one k) and a
// chunk of modes: its threads sum the (leaf, mode) pairs in parallel into LDS, then one
// thread per mode replays the combine program.  The complex product is numpy's
// (y + 0j)(c + js) = (y c - 0 s, y s + 0 c) and the division by ns is numpy's complex / real
// (multiplication by 1/ns), compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "podsgen_ext.h"

namespace pods {
namespace {

constexpr int DFT_LDS_PAIRS = 4096;  // (leaf, mode) partial sums per workgroup: 64 KB
constexpr int DFT_STACK = 32;

__global__ __launch_bounds__(256) void k_dft_tab(const double* __restrict__ T, int ldT, int nm, int ns,
                                                 const double2* __restrict__ W, const int* __restrict__ prog,
                                                 int nprog, const int* __restrict__ leaves, int nleaf, int mc,
                                                 int nk, double inv_n, float2* __restrict__ cout) {
  __shared__ double2 part[DFT_LDS_PAIRS];
  const int q = blockIdx.x;
  const int m0 = blockIdx.y * mc;
  const int nmc = min(mc, nm - m0);
  const double2* Wr = W + (int64_t)q * ns;
  const int items = nleaf * nmc;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int lf = it / nmc, md = it - lf * nmc;
    const int s = leaves[2 * lf], n = leaves[2 * lf + 1];
    const double* y = T + m0 + md;
    double rr, ri;
    if (n < 4) {
      rr = -0.0;
      ri = -0.0;
      for (int m = s; m < s + n; ++m) {
        const double2 w = Wr[m];
        const double yv = y[(int64_t)m * ldT];
        rr = rr + (yv * w.x - 0.0 * w.y);
        ri = ri + (yv * w.y + 0.0 * w.x);
      }
    } else {
      double r[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double2 w = Wr[s + e];
        const double yv = y[(int64_t)(s + e) * ldT];
        r[2 * e] = yv * w.x - 0.0 * w.y;
        r[2 * e + 1] = yv * w.y + 0.0 * w.x;
      }
      int i = 4;
      for (; i < n - (n % 4); i += 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double2 w = Wr[s + i + e];
          const double yv = y[(int64_t)(s + i + e) * ldT];
          r[2 * e] = r[2 * e] + (yv * w.x - 0.0 * w.y);
          r[2 * e + 1] = r[2 * e + 1] + (yv * w.y + 0.0 * w.x);
        }
      }
      rr = (r[0] + r[2]) + (r[4] + r[6]);
      ri = (r[1] + r[3]) + (r[5] + r[7]);
      for (; i < n; ++i) {
        const double2 w = Wr[s + i];
        const double yv = y[(int64_t)(s + i) * ldT];
        rr = rr + (yv * w.x - 0.0 * w.y);
        ri = ri + (yv * w.y + 0.0 * w.x);
      }
    }
    part[lf * nmc + md] = make_double2(rr, ri);
  }
  __syncthreads();
  const int md = threadIdx.x;
  if (md >= nmc) return;
  double sr[DFT_STACK], si[DFT_STACK];
  int sp = 0, lf = 0;
  for (int op = 0; op < nprog; ++op) {
    if (prog[2 * op] < 0) {
      --sp;
      sr[sp - 1] = sr[sp - 1] + sr[sp];
      si[sp - 1] = si[sp - 1] + si[sp];
    } else {
      const double2 v = part[lf * nmc + md];
      ++lf;
      sr[sp] = v.x;
      si[sp] = v.y;
      ++sp;
    }
  }
  const double cr = (0.0 + sr[0]) * inv_n;
  const double ci = (0.0 + si[0]) * inv_n;
  const float2 val = make_float2((float)cr, (float)ci);
  const int h = ns / 2, mode = m0 + md;
  if (q < nk) {
    const int k = q;
    cout[(int64_t)(h + k) * nm + mode] = val;
    if (k > 0 && h - k >= 0) cout[(int64_t)(h - k) * nm + mode] = make_float2(val.x, -val.y);
  } else {
    cout[mode] = val;  // n = 0, k = -ns/2
  }
}

}  // namespace

int dft_table_rows(int ns) {
  const int h = ns / 2;
  const int nk = (ns % 2 == 0) ? h : h + 1;  // k = 0..nk-1
  return nk + ((ns % 2 == 0) ? 1 : 0);
}

hipError_t launch_dft_tab(const double* T, int ldT, int nm, int ns, const double2* W, const int* prog, int nprog,
                          const int* leaves, int nleaf, double inv_n, float2* c, hipStream_t st) {
  if (nleaf <= 0 || nleaf > DFT_LDS_PAIRS) return hipErrorInvalidValue;
  const int h = ns / 2;
  const int nk = (ns % 2 == 0) ? h : h + 1;
  const int rows = dft_table_rows(ns);
  const int mc = std::max(1, std::min(nm, std::min(256, DFT_LDS_PAIRS / nleaf)));
  const int ny = (nm + mc - 1) / mc;
  hipLaunchKernelGGL(k_dft_tab, dim3((unsigned)rows, (unsigned)ny), dim3(256), 0, st, T, ldT, nm, ns, W, prog,
                     nprog, leaves, nleaf, mc, nk, inv_n, c);
  return hipGetLastError();
}

}  // namespace pods

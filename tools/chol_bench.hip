// Microbenchmark of one-wave 64x64 Cholesky + triangular inverse variants (k_chol_inv
// candidates): time per launch over 200 back-to-back launches.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/chol_bench.hip -o tools/chol_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int MODE>
__global__ __launch_bounds__(64) void chol(const double* __restrict__ G, double* __restrict__ Rinv) {
  __shared__ double col[64];
  __shared__ double Ls[64][64];
  __shared__ double Xs[64][65];
  __shared__ double dinv[64];
  const int i = threadIdx.x;
  double gr[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) gr[k] = 0.5 * (G[i * 64 + k] + G[k * 64 + i]);
  if (MODE == 0) {  // loads + stores only
#pragma unroll
    for (int k = 0; k < 64; ++k) Rinv[k * 64 + i] = gr[k];
    return;
  }
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double d = __shfl(gr[j], j);
    const double ljj = d > 0.0 ? sqrt(d) : __builtin_nan("");
    const double lij = i == j ? ljj : gr[j] / ljj;
    gr[j] = i >= j ? lij : 0.0;
    col[i] = i > j ? lij : 0.0;
    if (i == j) dinv[j] = 1.0 / ljj;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = j + 1; k < 64; ++k) gr[k] = fma(-lij, col[k], gr[k]);
    __builtin_amdgcn_wave_barrier();
  }
  if (MODE == 1) {
#pragma unroll
    for (int k = 0; k < 64; ++k) Rinv[k * 64 + i] = gr[k];
    return;
  }
#pragma unroll
  for (int k = 0; k < 64; ++k) Ls[i][k] = gr[k];
  const int c = i;
  for (int t = 0; t < 64; ++t) Xs[t][c] = t == c ? 1.0 : 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int t = 63; t >= 0; --t) {
    const double xt = Xs[t][c] * dinv[t];
    Xs[t][c] = xt;
#pragma unroll 8
    for (int k = 0; k < t; ++k) Xs[k][c] = fma(-Ls[t][k], xt, Xs[k][c]);
  }
  for (int t = 0; t < 64; ++t) Rinv[t * 64 + c] = Xs[t][c];
}

// chol3: readlane pivots and one reciprocal per step (instead of ds_bpermute and two divisions)
__global__ __launch_bounds__(64) void chol3(const double* __restrict__ G, double* __restrict__ Rinv) {
  __shared__ double col[2][64];
  __shared__ double Ls[64][64];
  __shared__ double Xs[64][65];
  __shared__ double dinv[64];
  const int i = threadIdx.x;
  double gr[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) gr[k] = 0.5 * (G[i * 64 + k] + G[k * 64 + i]);
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(gr[j]), j);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(gr[j]), j);
    const double d = __hiloint2double(hi, lo);
    const double ljj = d > 0.0 ? sqrt(d) : __builtin_nan("");
    const double r = 1.0 / ljj;
    const double lij = i == j ? ljj : gr[j] * r;
    gr[j] = i >= j ? lij : 0.0;
    col[j & 1][i] = lij;
    if (i == 0) dinv[j] = r;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = j + 1; k < 64; ++k) gr[k] = fma(-lij, col[j & 1][k], gr[k]);
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int k = 0; k < 64; ++k) Ls[i][k] = gr[k];
  const int c = i;
  for (int t = 0; t < 64; ++t) Xs[t][c] = t == c ? 1.0 : 0.0;
  for (int t = 63; t >= 0; --t) {
    const double xt = Xs[t][c] * dinv[t];
    Xs[t][c] = xt;
#pragma unroll 8
    for (int k = 0; k < t; ++k) Xs[k][c] = fma(-Ls[t][k], xt, Xs[k][c]);
  }
  for (int t = 0; t < 64; ++t) Rinv[t * 64 + c] = Xs[t][c];
}


// chol4: factorisation and the inverse fused.  Step j forms column j of L (broadcast through
// LDS), updates the trailing rows of G (lane i: row i) and, with the SAME column, the forward
// substitution for Z = L^{-1} (lane c: column c of Z, s_k -= L_kj z_j for k > j); z_j is final
// at step j and parked in LDS (Zs[c][j] = Z[j][c] = R^{-1}[c][j]... transposed once at the end).
__global__ __launch_bounds__(64) void chol4(const double* __restrict__ G, double* __restrict__ Rinv) {
  __shared__ double col[2][64];
  __shared__ double Zs[64][65];
  const int i = threadIdx.x;
  double gr[64], sv[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    gr[k] = 0.5 * (G[i * 64 + k] + G[k * 64 + i]);
    sv[k] = k == i ? 1.0 : 0.0;
  }
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(gr[j]), j);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(gr[j]), j);
    const double d = __hiloint2double(hi, lo);
    const double ljj = d > 0.0 ? sqrt(d) : __builtin_nan("");
    const double r = 1.0 / ljj;
    const double lij = gr[j] * r;          // lanes i > j: L[i][j]
    const double zj = sv[j] * r;           // Z[j][c] (lane c)
    Zs[i][j] = zj;
    col[j & 1][i] = lij;
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
  // Rinv[t][c] = Z[c][t]: lane c writes column c from row c of... Zs[c'][t] = Z[t][c']
  // -> Rinv[t][c] = Z[c][t] = Zs[t][c]
#pragma unroll
  for (int t = 0; t < 64; ++t) Rinv[t * 64 + i] = Zs[t][i];
}

int main() {
  const int m = 64;
  std::vector<double> h(m * m);
  // G = Y^T Y + shift for a random-ish Y: SPD
  for (int a = 0; a < m; ++a)
    for (int b = 0; b < m; ++b) h[a * m + b] = (a == b ? 70.0 : 0.0) + 1.0 / (1.0 + a + b);
  double *G, *R;
  CK(hipMalloc(&G, m * m * 8));
  CK(hipMalloc(&R, m * m * 8));
  CK(hipMemcpy(G, h.data(), m * m * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](auto kern, const char* name) -> int {
    for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, G, R);
    CK(hipEventRecord(e0));
    for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, G, R);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<double> r(m * m);
    CK(hipMemcpy(r.data(), R, m * m * 8, hipMemcpyDeviceToHost));
    printf("%-28s %8.2f us/launch  R[0]=%.6f R[63*64+63]=%.6f\n", name, ms * 1e3 / 200, r[0], r[63 * 64 + 63]);
    return 0;
  };
  run(chol<0>, "loads+stores");
  run(chol<1>, "factorisation");
  run(chol<2>, "factorisation+inverse");
  run(chol3, "readlane+inverse");
  run(chol4, "fused factorisation+inverse");
  return 0;
}

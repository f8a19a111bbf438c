// Launchers added after the first kernel files (kept apart from podsgen_kernels.h so that
// a change here rebuilds only its users).  All enqueue on `st`.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pods {

// ---- bit-exact shifted DFT from a host twiddle table (podsgen_dft.hip) ----------------
// rows of the table W (ns doubles2 each): k = 0..nk-1, plus k = -ns/2 for even ns
int dft_table_rows(int ns);
// leaves: nleaf x {start, count} in the order cpairwise_program's leaves appear in prog
hipError_t launch_dft_tab(const double* T, int ldT, int nm, int ns, const double2* W, const int* prog, int nprog,
                          const int* leaves, int nleaf, double inv_n, float2* c, hipStream_t st);

// snapshots [i0, i1) of the K-tiled snapshot matrix as (i1-i0) x rowlen rows (podsgen_pack.hip)
hipError_t launch_gather_snapshots(const double* AT, int ns, int64_t rowlen, int i0, int i1, double* out,
                                   hipStream_t st);

// out = alpha (C Y) + beta Y + gamma Z on fp64 MFMA from the tiled copy Ct of C (launch_tile_c:
// cheb_tiled_doubles(n) doubles, 64 x 64 tiles, each contiguous); Y/Z/out n x 64 row-major, out
// distinct from Y and Z (podsgen_subspace.hip); part: cheb_splits(n) x n x 64 doubles of
// split-K partials (unused when cheb_splits(n) == 1)
int cheb_splits(int n);
size_t cheb_tiled_doubles(int n);
hipError_t launch_tile_c(const double* C, int64_t ldc, int n, double* Ct, hipStream_t st);
hipError_t launch_cheb_step(const double* Ct, int n, const double* Y, const double* Z, int m, double alpha,
                            double beta, double gamma, double* part, double* out, hipStream_t st);

// small dense pieces of the subspace iteration, m = 64 (podsgen_subspace.hip):
// G = Y^T Z (64 x 64) through gram_slices(n) row-slice partials in part (summed in order);
// Rinv = L^{-T} for G = L L^T (X = Y Rinv orthonormalises Y when G = Y^T Y);
// out = Y M for an m x m M (m a multiple of 16).  Outputs distinct from inputs.
int gram_slices(int n);
hipError_t launch_gram(const double* Y, const double* Z, int n, double* part, double* G, hipStream_t st);
hipError_t launch_chol_inv(const double* G, double* Rinv, hipStream_t st);
// out = Y M, or Z - Y M when Z is not null
hipError_t launch_right_mul(const double* Y, const double* M, const double* Z, int n, int m, double* out,
                            hipStream_t st);

}  // namespace pods

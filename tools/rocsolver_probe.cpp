// Eigensolver landscape at n: sytrd, sterf, syevd, syevdx(top 20), syevj, syevdj.
// hipcc -O2 tools/rocsolver_probe.cpp -lrocsolver -lrocblas -o /tmp/rsp
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 4096;
  std::vector<double> h((size_t)n * n);
  std::mt19937_64 g(1); std::normal_distribution<double> N;
  // C = B B^T / n with B n x (n+n/2): SPD with one decaying spectrum
  int m = n + n / 2; std::vector<double> B((size_t)n * m);
  for (auto& x : B) x = N(g);
  rocblas_handle hdl; rocblas_create_handle(&hdl);
  double *dB, *dC, *dA, *D, *E, *tau, *W, *Z; int* info; int* nev; double* resid; int* nsw;
  hipMalloc(&dB, B.size() * 8); hipMalloc(&dC, (size_t)n * n * 8); hipMalloc(&dA, (size_t)n * n * 8);
  hipMalloc(&D, n * 8); hipMalloc(&E, n * 8); hipMalloc(&tau, n * 8); hipMalloc(&W, n * 8);
  hipMalloc(&Z, (size_t)n * 32 * 8); hipMalloc(&info, 4); hipMalloc(&nev, 4); hipMalloc(&resid, 8); hipMalloc(&nsw, 4);
  hipMemcpy(dB, B.data(), B.size() * 8, hipMemcpyHostToDevice);
  double one = 1.0 / n, zero = 0;
  rocblas_dgemm(hdl, rocblas_operation_none, rocblas_operation_transpose, n, n, m, &one, dB, n, dB, n, &zero, dC, n);
  hipDeviceSynchronize();
  auto reset = [&] { hipMemcpy(dA, dC, (size_t)n * n * 8, hipMemcpyDeviceToDevice); hipDeviceSynchronize(); };
  auto T = [&](const char* name, auto fn) {
    for (int r = 0; r < 2; ++r) {
      reset(); double t = now(); fn(); hipDeviceSynchronize(); t = now() - t;
      if (r == 1) printf("%-28s n=%d %9.2f ms\n", name, n, t * 1e3);
    }
    fflush(stdout);
  };
  T("sytrd", [&] { rocsolver_dsytrd(hdl, rocblas_fill_lower, n, dA, n, D, E, tau); });
  T("sytrd+sterf", [&] { rocsolver_dsytrd(hdl, rocblas_fill_lower, n, dA, n, D, E, tau); rocsolver_dsterf(hdl, n, D, E, info); });
  T("syevd (V)", [&] { rocsolver_dsyevd(hdl, rocblas_evect_original, rocblas_fill_lower, n, dA, n, D, E, info); });
  T("syevd (N)", [&] { rocsolver_dsyevd(hdl, rocblas_evect_none, rocblas_fill_lower, n, dA, n, D, E, info); });
  T("syevdx top20 (V)", [&] { rocsolver_dsyevdx(hdl, rocblas_evect_original, rocblas_erange_index, rocblas_fill_lower, n, dA, n, 0, 0, n - 19, n, nev, W, Z, n, info); });
  T("syevj (V)", [&] { rocsolver_dsyevj(hdl, rocblas_esort_ascending, rocblas_evect_original, rocblas_fill_lower, n, dA, n, 1e-14, resid, 30, nsw, W, info); });
  T("syevdj (V)", [&] { rocsolver_dsyevdj(hdl, rocblas_evect_original, rocblas_fill_lower, n, dA, n, W, info); });
  int hs; hipMemcpy(&hs, nsw, 4, hipMemcpyDeviceToHost); printf("syevj sweeps %d\n", hs);
  return 0;
}

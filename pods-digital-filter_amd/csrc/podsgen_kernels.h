// Launchers of the gfx950 kernels (podsgen_kernels.hip).  All enqueue on `st`.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace pods {

// Persistent (spin-waiting) grids hand data between workgroups, so every workgroup must be
// resident at once.  check_persistent asks the occupancy API (cached per kernel and LDS size)
// and returns hipErrorCooperativeLaunchTooLarge when grid > blocks per CU x CUs, before launch.
bool persistent_grid_fits(int blocks_per_cu, int cus, int64_t grid);
// st: the stream the grid goes to -- a stream created with a CU mask (hipExtStreamCreateWithCUMask)
// offers only its masked CUs (stream_cus)
hipError_t check_persistent(const void* fn, int block, size_t lds, int64_t grid, hipStream_t st = nullptr);
int stream_cus(hipStream_t st);

hipError_t launch_mt_jump(const uint32_t* src, const int* src_idx, const uint32_t* polys,
                          const int* poly_idx, uint32_t* dst, const int* dst_idx, int njobs,
                          hipStream_t st);
hipError_t launch_mt_generate(const uint32_t* states, int G, int64_t Bs, int64_t ntot, int64_t S,
                              int Kp, int rlo, int rhi, int64_t Sl, double low, double range,
                              double* out, hipStream_t st, int per_cu = 0);
// the multi-GPU state exchange's chains (mode 0: record segment start states, 1: store segments)
hipError_t launch_mt_chains(int mode, const uint32_t* st0, const int64_t* b0, const int* nb, int nchains,
                            const int64_t* rec_block, const int* rec_slot, const int* rec_first, uint32_t* rec_out,
                            int64_t ntot, int64_t S, int Kp, int rlo, int rhi, int64_t Sl, double low, double range,
                            double* out, hipStream_t st);
// max_grid > 0: at most that many workgroups (each then takes several virtual blocks): the x pass
// beside the eigensolver's tail keeps to a few waves per CU
hipError_t launch_filter_x(int NX, const double* R, const double* bx, int ns, int64_t Sl, int ncomp,
                           int chunk, double* T1, hipStream_t st, int s0 = 0, int s1 = -1, int max_grid = 0);
// lund_sj: 0 = one row of 9 x K parameters for every j (plain layout lund[e * Pl + k]);
// otherwise the table is j-varying and in the chunk-major layout below
inline int64_t lund_chunk_index(int64_t j, int e, int k, int K) {
  const int QC = (K + 15) / 16, q = k / 16, kk = k % 16;
  return ((((j * 9 + e) * 8 + kk / 2) * QC + q) * 2) + (kk & 1);
}
inline int64_t lund_chunk_size(int64_t jl, int K) { return jl * 9 * 16 * (int64_t)((K + 15) / 16); }
hipError_t launch_filter_yz(int NY, const double* T1, const double* by, const double* bz, int NZ,
                            int ns, int jl, int K, int Kp, int64_t Sl, int ncomp,
                            const double* lund, int64_t lund_sj, int lund_mode, const double* rot,
                            int rotate, double* AT, hipStream_t st, int s0 = 0, int s1 = -1);
int filter_yz_max_K(int Kp);
hipError_t launch_lund_apply(double* yu, double* yv, double* yw, int64_t P, const double* lund,
                             int lund_mode, const double* rot, int rotate, hipStream_t st);
// devmax (nullable): also max |fl(a - mean)| over the matrix, as a double (zeroed here)
hipError_t launch_mean(const double* AT, int64_t rowlen, int ns, const int* prog, int nprog,
                       double* mean, hipStream_t st, double* devmax = nullptr, int nleaf = 0);
// The correlation by exact int8-MFMA modular products + CRT (podsgen_corr_i8.hip).
struct CorrI8Plan {
  int bbits;       // scaled elements are integers with |a'| <= 2^bbits
  int nlaunch;     // residue + SYRK launches (K chunks of the residue buffer)
  int nsplit;      // K splits per launch
  int kcs;         // 64-row K chunks per split
  int64_t chunks;  // K chunks per launch (nsplit * kcs)
  int64_t nkc;     // K chunks of the matrix
  int nitems;      // work items per modulus per launch
  int64_t r_bytes; // residue buffer
  int64_t p_bytes; // per-modulus partial buffer
};
int corr_i8_nmod();
int corr_i8_plan(int ns, int64_t rowlen, int64_t rowpad, int64_t budget_bytes, CorrI8Plan* out, int force_split = 0);
std::vector<int> corr_i8_items(int ns, const CorrI8Plan& p);
hipError_t launch_absdev(const double* AT, int ns, int64_t rowlen, int64_t rowpad, const double* mean,
                         double* devmax, hipStream_t st);
hipError_t launch_corr_i8(const double* AT, int ns, int64_t rowlen, int64_t rowpad, const double* mean,
                          const double* devmax, const CorrI8Plan& p, const int* items, int8_t* R, uint8_t* P,
                          double* C, int64_t ldc, int divide, hipStream_t st, hipEvent_t syrk_begin,
                          hipEvent_t syrk_end, const int* xitems, int per_xcd, unsigned* pace_ctr);
// the persistent SYRK's per-XCD item table from the grid-order one (per_xcd: items per XCD)
std::vector<int> corr_i8_xcd_items(const std::vector<int>& items, int nitems, int* per_xcd);
// slack past the residue buffer's end (allocation padding)
constexpr int64_t CORR_I8_RPAD = 1 << 16;
// Split-K SYRK (k_syrk_g128 + k_syrk_reduce).  Plan: returns the number of K splits (work
// slabs of ns*ns doubles).
int syrk_plan(int ns, int64_t Kdim, int64_t* ksplit);
// items: nitems x int4 {bi, bj, split, 0} in launch order (see podsgen_api.cpp syrk_items)
hipError_t launch_syrk(const double* AT, int ns, int64_t Kdim, const double* mean, const int* items, int nitems,
                       int nsplit, int64_t ksplit, double* C, int64_t ldc, int divide, double* work, int centred,
                       hipStream_t st);
// A <- A - mean in place (K-tiled layout, rowpad rows x ns snapshots)
hipError_t launch_center(double* AT, int64_t rowpad, int ns, const double* mean, hipStream_t st);
hipError_t launch_divide(double* x, int64_t n, double d, hipStream_t st);
// packed lower triangle (row r at r(r+1)/2) of an n x n row-major C (podsgen_pack.hip)
hipError_t launch_pack_lower(const double* C, int64_t ldc, int n, double* packed, hipStream_t st);
// C[r][c] = C[c][r] = packed[r(r+1)/2 + c] / divisor
hipError_t launch_unpack_lower(const double* packed, int n, double divisor, double* C, int64_t ldc,
                               hipStream_t st);
hipError_t launch_recip(const double* x, int n, double* y, hipStream_t st);
hipError_t launch_temporal(const double* V, int64_t v_rs, int64_t v_cs, int ns, int ncols,
                           int nvalid, const double* lam, double* mag, double* T, hipStream_t st);
size_t spatial_work_bytes(int64_t rowlen, int ns);
hipError_t launch_spatial(const double* AT, int64_t rowlen, int ns, const double* mean,
                          const double* T, int ldT, int nm, const double* inv_lam, double* phi,
                          double* work, hipStream_t st);
int rank_max_ns();
hipError_t launch_rank(const float* c, int ns, int nm, double et, const int* prog, int nprog,
                       int32_t* c_ind, int64_t* c_count, hipStream_t st);

// ---- symmetric eigensolver (podsgen_eigen.hip) ----------------------------------------
// doubles per k_trd hand-off buffer (one vector, one XCD copy, one column parity): 512 lanes x 8
// slots; the workspace holds 2 vectors x 8 copies x 2 parities of them
constexpr int TRD_HANDOFF = 4096;
struct TrdArgs {
  const double* C;   // n x n row-major symmetric input (read only)
  int64_t ldc;
  int n;
  int G;             // workgroups (= ceil(n / R)), all co-resident
  int klast;         // last column range: (n - 1) / 512
  double* Wm;        // per-workgroup slabs G x S x R x 512 (trd_plan's slab_doubles)
  double* pbuf;      // 2 x n tagged values: p = A v (double-buffered by column parity)
  double* rbuf;      // 2 x n tagged values: next column of A (zeroed before the launches)
  int nrep;          // hand-off copies (1 or 8: one per XCD)
  uint32_t* flags;   // [0]: abort word (set if a hand-off wait timed out), zeroed
  double* D;         // n   diagonal of T
  double* E;         // n-1 off-diagonal of T
  double* tau;       // n-1 reflector scalars
  double* V;         // (n-1) x ldv reflector vectors, row j = v_j
  int64_t ldv;
  int64_t* trace;    // diagnostics: n x 8 s_memrealtime stamps of workgroup trace_wg, or null
  int trace_wg;
};
int trd_plan(int n, int* R, int* G, int64_t* slab_doubles);
hipError_t launch_trd(const TrdArgs& a, int R, hipStream_t st);
// ranges kb..ke only (range K = columns [512K - 1, 512(K + 1) - 1)); klast + 1 ranges in all
hipError_t launch_trd_ranges(const TrdArgs& a, int R, int kb, int ke, hipStream_t st);
// bounds: 4 doubles {gl, gu, pivmin, atol}; lam_desc: n eigenvalues of T, descending
// grid_cnt (tri_grid_bytes(), may be null): counts at shared shifts for the first brackets
// deg: 2n doubles of scratch, needed when n > 10240 ({d, e^2} then live in global memory)
hipError_t launch_tri_eigvals(const double* D, const double* E, int n, double* bounds,
                              double* lam_desc, int* grid_cnt, hipStream_t st, double2* deg = nullptr);
size_t tri_grid_bytes();
// the same in two parts: Gershgorin bounds, then the eigenvalues with ascending index [k0, k1)
hipError_t launch_tri_bounds(const double* D, const double* E, int n, double* bounds, hipStream_t st);
hipError_t launch_tri_bisect(const double* D, const double* E, int n, const double* bounds,
                             double* lam_desc, int k0, int k1, int* grid_cnt, hipStream_t st,
                             double2* deg = nullptr);
// Z: n x nvec row-major eigenvectors of T for lam_desc[0..nvec); X: nvec x n scratch
hipError_t launch_tri_eigvecs(const double* D, const double* E, int n, const double* lam_desc,
                              const double* bounds, int nvec, double* X, double* Z, hipStream_t st);
// Z <- Q Z with Q = H_0 ... H_{n-2} (one k_larft launch + one persistent k_bt_fused launch);
// Tg: ceil((n-1)/64) x 64 x 64, part: bt_part_bytes, W2: bt_w2_bytes, abortw: 0 on entry
// larft_st: the stream for k_larft (it needs V and tau only); the caller orders `st` behind it
// (null: k_larft on `st` too)
hipError_t launch_back_transform(const double* V, int64_t ldv, const double* tau, int n, int nvec,
                                 double* Tg, double* part, double* W2, uint32_t* abortw, double* Z,
                                 hipStream_t st, bool skip_larft = false);
hipError_t launch_larft(const double* V, int64_t ldv, const double* tau, int n, double* Tg, hipStream_t st);
void bt_plan(int n, int nvec, int* CR, int* G);
// cluster modified Gram-Schmidt of the nvec eigenvector columns of Z (k_orth)
hipError_t launch_orth(const double* lam_desc, const double* bounds, int n, int nvec, double* Z, int ldz,
                       hipStream_t st);

// ---- two-stage eigensolver for n > 4096 (podsgen_sy2sb.hip) ---------------------------
struct SyevdPlan {
  int B, np, KS, NZ, RP;
  int64_t off_aw, off_vx, off_t, off_tau, off_y, off_x, off_w, off_zp, off_m, off_pub, off_band, off_band0,
      off_de, off_deg, off_inv, off_end;
};
int sy2sb_band();
int syev2_max_n();  // k_pqr: 64 workgroups x 256 panel rows
// doubles of workspace for n, nvec (and the offsets inside it)
size_t sy2sb_work_doubles(int n, int nvec, SyevdPlan* plan);
// flags: 128 + n uint32 (zeroed once at allocation); ipiv: nvec * n ints; epoch: a counter
// that grows by one per call (the panel hand-off tags); grid_cnt: tri_grid_bytes()
hipError_t launch_syevd2(const double* C, int n, int nvec, double* ws, const SyevdPlan& p, uint32_t* flags,
                         uint32_t epoch, int* ipiv, int* grid_cnt, double* lam_desc, double* vec, hipStream_t st);
// the same solve in stages (eigenvalues only when spread over calls: pods_eigvals_* for n > 4096):
// begin (copies C, clears the chase counters and panel slots), stage-1 panels [pi0, pi1) (plan.np
// panels), the band (band0 kept for the vectors), chase sweep groups [q0, q1) of syevd2_groups(n)
// (every earlier group finished), the eigenvalues (descending)
hipError_t syevd2_begin(const double* C, int n, double* ws, const SyevdPlan& p, uint32_t* flags, hipStream_t st);
hipError_t syevd2_panels(int n, double* ws, const SyevdPlan& p, uint32_t* flags, uint32_t epoch, int pi0, int pi1,
                         hipStream_t st);
hipError_t syevd2_band(int n, double* ws, const SyevdPlan& p, bool keep_band0, hipStream_t st);
int syevd2_groups(int n);
hipError_t syevd2_chase(int n, double* ws, const SyevdPlan& p, uint32_t* flags, int q0, int q1, hipStream_t st);
hipError_t syevd2_eigvals(int n, double* ws, const SyevdPlan& p, int* grid_cnt, double* lam_desc, hipStream_t st);
size_t bt_part_bytes(int n, int nvec);
size_t bt_w2_bytes(int nvec);

}  // namespace pods

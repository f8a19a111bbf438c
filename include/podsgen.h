/*
 * podsgen.h -- C ABI of libpodsgen.so, the MI355X (gfx950) engine behind the
 * digital-filter + PODFS hot path of sidbannet/PODS-digital-filter.
 *
 * The reference has no FFI: its "operator API" is a set of Python functions that
 * mutate numpy arrays.  Each entry point below replaces one of them;
 * the Python drop-in modules (pods-digital-filter_amd/digitalfilters.py, PODFS.py)
 * keep the reference signatures and call these through ctypes.
 *
 * Conventions
 *   - every function returns int: PODS_OK (0) or a negative PODS_ERR_* code; the
 *     message of the last failure on the calling thread is pods_last_error().
 *   - no C++ exception crosses the ABI; HIP errors map to PODS_ERR_HIP.
 *   - the caller owns every output buffer.  "_dev" pointers are device pointers on the
 *     context's device (e.g. torch tensor data_ptr()); "_host" pointers are host memory.
 *   - a context is bound to one device and one HIP stream (pods_set_stream); it is not
 *     thread-safe.  Calls enqueue on that stream; functions that return host data
 *     synchronise the stream before returning.
 *   - plain pointers and sizes only, no torch types.
 */
#ifndef PODSGEN_H
#define PODSGEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PODS_ABI_VERSION 1

enum {
  PODS_OK = 0,
  PODS_ERR_ARG = -1,         /* bad argument / shape                        */
  PODS_ERR_HIP = -2,         /* HIP runtime error                           */
  PODS_ERR_STATE = -3,       /* call order (e.g. generate before configure) */
  PODS_ERR_NOMEM = -4,       /* device allocation failed                    */
  PODS_ERR_INTERNAL = -5,
  PODS_ERR_UNSUPPORTED = -6
};

/* Lund transform variants (digitalfilters.py:143-178 adapt1d, :180-231 adapt2prf). */
enum { PODS_LUND_1D = 0, PODS_LUND_PRF = 1, PODS_LUND_NONE = -1 };

typedef struct pods_ctx pods_ctx;

/* Digital-filter problem description (digitalfilters.py main(), :1244-1397). */
typedef struct pods_df_params {
  int32_t jma, kma;      /* inlet grid: J spanwise rows, K wall-normal columns      */
  int32_t ns;            /* snapshots (time steps)                                  */
  int32_t nfx, nfy, nfz; /* half filter widths: taps = 2*nf+1                       */
  int32_t j0, j1;        /* row slab owned by this context, 0 <= j0 < j1 <= jma     */
  int32_t lund_mode;     /* PODS_LUND_1D | PODS_LUND_PRF | PODS_LUND_NONE           */
  int32_t rotate;        /* 0: rotation is the identity (skipped); 1: apply rot[9]  */
  uint32_t seed;         /* numpy legacy RandomState / np.random.seed value         */
  int32_t reserved;
  double rng_low;        /* uniform low   (-sqrt(3), digitalfilters.py:1340)        */
  double rng_range;      /* high - low    (2*sqrt(3))                               */
} pods_df_params;

const char* pods_last_error(void);
int pods_abi_version(void);

/* Context lifetime.  Replaces nothing in the reference (single Python process). */
int pods_create(pods_ctx** out, int device);
int pods_destroy(pods_ctx* ctx);
/* Enqueue all work on this hipStream_t (NULL = legacy default stream). */
int pods_set_stream(pods_ctx* ctx, void* hip_stream);
int pods_synchronize(pods_ctx* ctx);
/* shared != 0: other processes run persistent grids on this context's device (more ranks than
 * devices, e.g. a gloo run of several ranks on one GPU).  Every entry point that launches a
 * persistent grid (pods_syev, pods_sytrd*, pods_eigvals_begin/advance, pods_syev2) then holds an
 * exclusive per-device lock file (/tmp/podsgen-gpu-<PCI bus id>.lock) from before its launches
 * until its stream has drained, so two processes' grids never wait on each other's workgroups.
 * Those calls become synchronous in this mode.  Replaces nothing in the reference. */
int pods_set_shared_device(pods_ctx* ctx, int shared);

/* ---- generation: digitalfilters.py main() step loop :1403-1477 --------------------
 * bx/by/bz: filter taps (calccoeff, :73-89), lengths 2nf+1, host.
 * lund_host: 9 x P_local SoA rows a00,a10,a11,a20,a21,a22,U,V,W for the slab's points
 *            (P-index j*K + k, j relative to j0), host.
 * rot_host:  3x3 row-major rotation (prof_rotation_matrix, :1064-1116), host, used
 *            when params->rotate != 0.
 * Allocates the device buffers of the run (random stream slab, x-filtered planes,
 * snapshot matrix). */
int pods_df_configure(pods_ctx* ctx, const pods_df_params* params, const double* bx,
                      const double* by, const double* bz, const double* lund_host,
                      const double* rot_host);
/* RNG + 3 separable filter passes + Lund + rotation for all ns steps
 * (filter3DSciPy1D :100-140 x3, adapt1d/adapt2prf, rotate_velocity, A[:,i] = ... :1471).
 * The snapshot matrix stays on the device, snapshot-major: A_T[i][c*P_local + p]. */
int pods_df_generate(pods_ctx* ctx);
/* The same generation in parts, each on the context's current stream (pods_set_stream), so a
 * caller can run the random planes of the NEXT run on a second stream while this run's
 * centring and correlation occupy the first (main :1361-1367, :1454-1467 draw the planes;
 * filter :100-140 axis 0 is the x pass; axes 1-2 + adapt + rotate + A[:,i] = ... :1471 the y/z
 * part).  parts: bit 0 = jump-ahead of the MT19937 substreams, bit 1 = the substreams' random
 * planes, bit 2 = x pass, bit 3 = y/z pass (the snapshot matrix).  Parts run in that order;
 * PODS_GEN_ALL = 15 equals pods_df_generate.  The caller orders the streams (each part needs
 * the one before). */
#define PODS_GEN_JUMP 1
#define PODS_GEN_PLANES 2
#define PODS_GEN_XPASS 4
#define PODS_GEN_YZPASS 8
#define PODS_GEN_ALL 15
/* with PODS_GEN_PLANES: the planes' workgroups are limited to 2 per CU (padded LDS), so they
 * can run beside the late tridiagonalisation ranges of a pods_syev (see pods_syev_marker) */
#define PODS_GEN_BESIDE_SOLVER 16
/* with pods_df_set_exchange: record the segment-start states this rank owns (see below) */
#define PODS_GEN_RECORD 32
int pods_df_generate_parts(pods_ctx* ctx, int parts);
/* Multi-GPU generation without every rank twisting the whole MT19937 stream (the reference
 * draws it sequentially, digitalfilters.py:1361-1367, :1454-1467): the stream is cut into world x
 * ~2048 substreams, rank r owning a contiguous 1/world of them.  PODS_GEN_JUMP then jumps only
 * the owned substreams; PODS_GEN_RECORD twists them once and records, for every rank q and
 * plane, the state at the block where q's row segment (its slab rows plus the 2nfy halo) starts
 * -- when that block is owned here; the caller moves the records with ONE all_to_all between
 * two device buffers it owns (pods_df_exchange_bind; per-peer byte counts from
 * pods_df_exchange_sizes: rank r's send chunk for q, in plane order, lands in q's receive
 * buffer after the chunks of ranks < r); and
 * PODS_GEN_PLANES regenerates this rank's segments from the received states.  The planes are
 * bit-identical to the single-stream generation.  j0s / j1s: every rank's slab [j0, j1) (this
 * rank's must equal the configured one).  world <= 0 turns the exchange off, as pods_df_configure
 * does; world == 1 runs it for one rank (its all_to_all the identity: a single-device check of
 * the collective path). */
int pods_df_set_exchange(pods_ctx* ctx, int world, int rank, const int* j0s, const int* j1s);
int pods_df_exchange_sizes(pods_ctx* ctx, int64_t* send_bytes, int64_t* recv_bytes);
int pods_df_exchange_bind(pods_ctx* ctx, void* send_dev, void* recv_dev);
/* Two snapshot banks (0 = the default): bank selects which snapshot matrix -- with its mean,
 * scale and centring state -- every snapshot call (generation, pods_mean, pods_corr,
 * pods_center, pods_spatial_modes*, pods_df_snapshots) uses from now on.  A multi-GPU run
 * generates and correlates step k in one bank while step k-1's spatial modes (PODFS.py:1330-1333)
 * still read the other.  Bank 1 is allocated (zeroed) on first use; pods_df_configure returns to
 * bank 0.  Replaces nothing in the reference (one step at a time). */
int pods_select_snapshots(pods_ctx* ctx, int bank);
/* A new seed for the next generation (np.random.seed, digitalfilters.py:1344) without
 * reconfiguring: the next PODS_GEN_JUMP starts from it (multi-step runs of different inputs). */
int pods_df_set_seed(pods_ctx* ctx, uint32_t seed);
/* Device pointer and row length (= 3*P_local) of the snapshot matrix.  Device layout is
 * K-tiled: element (snapshot i, row r of the reference A) is at
 * a_dev[((r/16)*ns + i)*16 + r%16], rows padded with zeros to a multiple of 16. */
int pods_df_snapshots(pods_ctx* ctx, double** a_dev, int64_t* row_len);

/* Load an existing snapshot matrix instead of generating one (PODFS.POD called on a
 * user array, PODFS.py:1294).  at_host: snapshot-major ns x row_len (row i = A[:, i]);
 * re-laid out into the K-tiled device layout. */
int pods_set_snapshots(pods_ctx* ctx, const double* at_host, int ns, int64_t row_len);

/* Snapshots [i0, i1) of the device matrix in the reference's column order, one snapshot per
 * row: out_dev[(i - i0) * row_len + r] = A[r, i] (A as digitalfilters.py:1397 lays it out,
 * A[:, i] = the i-th snapshot; SURVEY 8(b) pods_copy_snapshots).  Device output, stream-ordered;
 * the current contents of A (centred after pods_center). */
int pods_copy_snapshots(pods_ctx* ctx, int i0, int i1, double* out_dev);

/* Stream-ordered copy between host/device buffers of this context's device
 * (kind: 0 = host->device, 1 = device->host, 2 = device->device).  device->host
 * synchronises the stream before returning. */
int pods_copy(pods_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);

/* mean over snapshots with numpy's pairwise order, np.mean(A,1) (:1492).  The context
 * keeps the mean for pods_corr / pods_spatial_modes (A - mean, :1493-1495);
 * mean_out (3*P_local doubles) may be NULL. */
int pods_mean(pods_ctx* ctx, double* mean_out, int out_is_device);

/* Centre the snapshots in place, A[:, j] = A[:, j] - mean (main() :1493-1495), after
 * pods_mean.  pods_corr and pods_spatial_modes then read A as it stands instead of
 * subtracting the mean themselves (same values, so the same results).  Worth it for the fp64
 * SYRK (pods_corr mode 0, 7 % faster on a centred A); the default int8 correlation subtracts
 * the mean while forming its residues and needs no centring.  Irreversible until the
 * snapshots are regenerated or reloaded. */
int pods_center(pods_ctx* ctx);

/* Set the mean the correlation / spatial-mode kernels subtract (mean_host: row_len doubles,
 * NULL = zeros, i.e. A is already centred -- PODFS.calculate_correlation_matrix, PODFS.py:1451). */
int pods_set_mean(pods_ctx* ctx, const double* mean_host);

/* Correlation C = (A-m)^T (A-m) [/ns] (PODFS.py:1451-1455).  C_dev: ns x ns row-major,
 * full symmetric.  divide = 1 divides by ns (single device); multi-device callers pass 0,
 * all-reduce the partials, then call pods_divide_inplace(C, ns*ns, ns). */
int pods_corr(pods_ctx* ctx, double* C_dev, int divide);
/* How pods_corr forms the products (replaces numpy's BLAS dgemm behind np.dot, PODFS.py:1455):
 *   1 (default) exact integer products on the int8 matrix cores: A - m scaled by one power of
 *     two to integers of <= 53 bits (2^-53 of max |A - m| is the only input rounding), their
 *     residues modulo 16 coprime moduli <= 255, one int8 SYRK per modulus, the exact 125-bit
 *     integer C' rebuilt by the Chinese remainder theorem and rounded to double once.  Needs
 *     16 bytes per element of residue workspace (in K chunks of PODS_CORR_BUDGET_GB, default 16)
 *     and no pods_center (the mean is subtracted while forming the residues);
 *   0 the fp64 MFMA SYRK (v_mfma_f64_16x16x4), rounding at every accumulation.
 * PODS_CORR=f64 in the environment selects 0 when the context is created. */
int pods_set_corr_mode(pods_ctx* ctx, int mode);
int pods_get_corr_mode(pods_ctx* ctx, int* mode);
/* Measurement: with timing on, every mode-1 pods_corr records HIP events around its int8 SYRK
 * launch on the context's stream; pods_corr_kernel_ms waits for them, returns the summed
 * milliseconds and the number of launches, and starts a new count.  (With the residue buffer
 * cut into several launches the events bracket all of them, residue passes included.) */
int pods_corr_timing(pods_ctx* ctx, int enable);
int pods_corr_kernel_ms(pods_ctx* ctx, double* total_ms, int* count);
/* Host-only: the plan mode 1 would use for ns snapshots of row_len rows (padded to row_pad) under
 * a residue budget of budget_bytes and force_split K splits (0 = planned).  out[8] = {scale bits
 * b, launches, K splits, 64-row chunks per split, chunks per launch, residue bytes, partial bytes,
 * bytes of one modulus' residues per launch (< 2^32: k_residues' offsets are 32-bit)}.
 * PODS_ERR_UNSUPPORTED when no plan exists (K beyond ~2^43, or ns too large for 32-bit offsets). */
int pods_corr_i8_plan_query(int ns, int64_t row_len, int64_t row_pad, int64_t budget_bytes, int force_split,
                            int64_t* out);
/* x[i] = x[i] / divisor for n doubles on the device. */
int pods_divide_inplace(pods_ctx* ctx, double* x_dev, int64_t n, double divisor);
/* The multi-device all-reduce of the partial correlations (PODFS.py:1455 summed over row slabs)
 * moves only the lower triangle: pods_pack_lower copies it from C_dev (n x n row-major) into
 * packed_dev (n(n+1)/2 doubles, row r at r(r+1)/2); after the all-reduce pods_unpack_lower
 * writes packed / divisor (IEEE division, numpy's `/ ns`) to both triangles of C_dev, so C is
 * exactly symmetric.  Device pointers, stream-ordered. */
int pods_pack_lower(pods_ctx* ctx, const double* C_dev, int n, double* packed_dev);
int pods_unpack_lower(pods_ctx* ctx, const double* packed_dev, int n, double divisor, double* C_dev);

/* Temporal modes after sort_eigenvalues + scaling (PODFS.py:1310, :1323-1325).
 * V_dev: eigenvectors from a symmetric solver in ASCENDING eigenvalue order, element
 * (i, j) at V_dev[i*v_rs + j*v_cs].  Output T_dev (ns x ncols, row-major) holds column j
 * = V[:, ns-1-j] (descending order) scaled by sqrt(lambda_j / (sum_i V_ij^2 / ns)) for
 * j < nvalid (sequential sum, Python builtin).  lambda_desc_host: ncols eigenvalues in
 * descending order (copied before the call returns).  Stream-ordered: returns without
 * synchronising the bound stream. */
int pods_temporal_modes(pods_ctx* ctx, const double* V_dev, int64_t v_rs, int64_t v_cs,
                        const double* lambda_desc_host, int nvalid, int ncols, double* T_dev);
/* The same with the eigenvalues on the device (lambda_desc_dev, e.g. pods_syev's output), so
 * the temporal modes can be enqueued before the host has seen the spectrum. */
int pods_temporal_modes_dev(pods_ctx* ctx, const double* V_dev, int64_t v_rs, int64_t v_cs,
                            const double* lambda_desc_dev, int nvalid, int ncols, double* T_dev);

/* Symmetric eigensolve of the POD (replaces `linalg.eig(C)` + `sort_eigenvalues`,
 * PODFS.py:1309-1310 and :1430-1447): all n eigenvalues in descending order and the unit
 * eigenvectors of the nvec largest.  C_dev: n x n row-major symmetric (read only).
 * lambda_desc_dev: n doubles.  vec_dev: n x nvec row-major, column k = eigenvector of
 * lambda_desc[k] (sign arbitrary, as the reference's dgeev vectors).  1 <= n <= 4096,
 * 0 <= nvec <= min(n, 64).  Stream-ordered (returns before the result is ready). */
int pods_syev(pods_ctx* ctx, const double* C_dev, int n, int nvec, double* lambda_desc_dev,
              double* vec_dev);
/* The tridiagonalisation step of pods_syev alone (test entry): C = Q T Q^T with
 * T = tridiag(e, d, e); d_host: n, e_host: n-1 (synchronous). */
int pods_sytrd(pods_ctx* ctx, const double* C_dev, int n, double* d_host, double* e_host);
/* Diagnostics: pods_sytrd with 8 s_memrealtime (100 MHz) stamps per column of workgroup
 * wg written to trace_host (n x 8 int64): column start, inputs arrived, after the dot
 * reduction, after the norm reduction, update start, update end, after the row-sum
 * barrier, column end.  wg < 0 traces every workgroup: trace_host holds 256 x n x 8. */
int pods_sytrd_trace(pods_ctx* ctx, const double* C_dev, int n, int wg, int64_t* trace_host);
/* 0 if the last pods_syev / pods_sytrd ran to completion, PODS_ERR_INTERNAL if its
 * cross-workgroup wait timed out (results invalid).  Synchronises the stream. */
int pods_syev_status(pods_ctx* ctx);
/* The two abort words of the last pods_syev (tridiagonalisation, back-transformation; both 0
 * when it completed) copied to flags_host (2 x uint32, pinned for a truly asynchronous copy),
 * stream-ordered, without synchronising: the caller waits on an event behind it. */
int pods_syev_flags_async(pods_ctx* ctx, uint32_t* flags_host);
/* The next pods_syev records a marker event on the stream once tridiagonalisation column
 * range `after_range` (512 columns each) is done; pods_stream_wait_marker makes `stream` (a
 * hipStream_t) wait for it, and fails if the last pods_syev recorded none (n <= 512 * (after_range
 * + 1)).  Used to start the next run's random planes beside the late ranges, whose workgroups
 * leave registers and LDS free (PODS_GEN_BESIDE_SOLVER). */
int pods_syev_marker(pods_ctx* ctx, int after_range);
int pods_stream_wait_marker(pods_ctx* ctx, void* stream);
/* The same behind the whole tridiagonalisation of the next pods_syev (where = 0: before its
 * bisection, eigenvectors and back-transformation) or behind its eigenvalues (where = 1: before
 * the eigenvectors and back-transformation): the next run's x pass can start there (scheduling
 * plumbing, no reference counterpart). */
int pods_syev_marker_tail(pods_ctx* ctx, int where);
int pods_stream_wait_marker_tail(pods_ctx* ctx, void* stream);

/* All n eigenvalues of C alone (the full spectrum POD.eigenvalues.dat and the valid-mode count
 * consume, PODFS.py:1309-1320, :1339), as a sequence of stream-ordered units that a caller can
 * spread over several calls.  n <= 4096: units 0..U-2 are the column ranges of the on-chip
 * tridiagonalisation (512 columns each, U - 1 = (n-1)/512 + 1), unit U-1 the bisection.
 * 4096 < n <= 16384: the two-stage solver of pods_syev2 without vectors -- units of 32 stage-1
 * panels (1024 columns reduced to band 32), then units of 512 bulge-chasing sweep groups (1024
 * sweeps), then the bisection (n = 8192: 8 + 8 + 1 units).  Each slot (0..15) has its own
 * workspace, so several matrices may be in flight at once.
 *   pods_eigvals_begin    starts slot on C_dev (n x n row-major, read by unit 0 only, so C may
 *                         be reused by work enqueued after this call) and runs unit 0
 *   pods_eigvals_advance  runs up to max_units more units; *remaining = units still to run
 *   pods_eigvals_fetch    when none remain: copies the n eigenvalues, descending, to lam_desc_dev
 *   pods_eigvals_status   synchronises; PODS_ERR_INTERNAL if a hand-off wait timed out
 *   pods_eigvals_flags_async  the slot's abort word (0: completed) copied to flags_dst (1 x
 *                         uint32; pinned host or device), stream-ordered behind the slot's
 *                         units, without synchronising -- captured when the spectrum finishes,
 *                         so a later matrix that reuses the slot cannot overwrite it */
int pods_eigvals_begin(pods_ctx* ctx, int slot, const double* C_dev, int n);
int pods_eigvals_advance(pods_ctx* ctx, int slot, int max_units, int* remaining);
int pods_eigvals_fetch(pods_ctx* ctx, int slot, double* lam_desc_dev);
int pods_eigvals_status(pods_ctx* ctx, int slot);
int pods_eigvals_flags_async(pods_ctx* ctx, int slot, uint32_t* flags_dst);
/* Test entry: sets the slot's abort word (stream-ordered), as a timed-out hand-off wait would,
 * so a caller's abort handling can be exercised without starving the device. */
int pods_eigvals_inject_abort(pods_ctx* ctx, int slot);
/* The two abort words of the last pods_syev2 (panel hand-offs, bulge chasing; both 0 when it
 * completed) copied to flags_dst (2 x uint32), stream-ordered, without synchronising
 * (PODFS.py:1309 on the ns > 4096 path; the counterpart of pods_syev_flags_async). */
int pods_syev2_flags_async(pods_ctx* ctx, uint32_t* flags_dst);

/* Prepares C_dev (n x n row-major) for pods_cheb_step: a 64 x 64-tiled copy in the context
 * (each tile contiguous, so the step streams C at the MFMA rate).  Call again whenever C_dev
 * or its contents change; pods_cheb_step refuses a C it was not prepared for. */
int pods_cheb_prepare(pods_ctx* ctx, const double* C_dev, int n);
/* One step of the Chebyshev-filtered subspace iteration that finds the nm leading eigenpairs
 * (podsgen/subspace.py; PODFS.py:1309-1333 consumes only those): out = alpha (C Y) + beta Y +
 * gamma Z on fp64 MFMA, C_dev n x n row-major, Y_dev / Z_dev / out_dev n x m row-major with
 * m = 64, out_dev distinct from Y_dev and Z_dev; Z_dev may be NULL (gamma ignored).
 * Deterministic (fixed reduction order).  Stream-ordered. */
int pods_cheb_step(pods_ctx* ctx, const double* C_dev, int n, const double* Y_dev, const double* Z_dev, int m,
                   double alpha, double beta, double gamma, double* out_dev);

/* The block operations around pods_cheb_step (n x m row-major device blocks, outputs distinct
 * from inputs, stream-ordered, deterministic):
 *   pods_gram       G_dev (m x m) = Y^T Z, m = 64 (row-slice partials summed in order)
 *   pods_cholqr     one Cholesky-QR pass: X = Y R^{-1} with R^T R = Y^T Y (m = 64); twice in a
 *                   row gives orthonormal columns to working precision (CholQR2)
 *   pods_right_mul  out = Y M for an m x m row-major M_dev (the Rayleigh-Ritz rotation)
 *   pods_ritz_residual  E = CX - X H (H = X^T C X): the residual block of the Rayleigh-Ritz
 *                   step, whose Gram E^T E gives every Ritz pair's residual norm
 *                   ||C X v - theta X v|| = ||E v|| without cancellation */
int pods_gram(pods_ctx* ctx, const double* Y_dev, const double* Z_dev, int n, int m, double* G_dev);
int pods_cholqr(pods_ctx* ctx, const double* Y_dev, int n, int m, double* X_dev);
int pods_right_mul(pods_ctx* ctx, const double* Y_dev, const double* M_dev, int n, int m, double* out_dev);
int pods_ritz_residual(pods_ctx* ctx, const double* X_dev, const double* CX_dev, const double* H_dev, int n, int m,
                       double* E_dev);

/* Two-stage eigensolver for correlation matrices beyond pods_syev's on-chip limit (BASELINE
 * configs 4/5, PODFS.py:1309-1310 at ns = 8192, 16384): dense -> band (bandwidth 32, fp64 MFMA
 * blocked updates), band -> tridiagonal (bulge chasing), bisection, inverse iteration on the
 * band matrix, back-transformation.  Same arguments and outputs as pods_syev; 3 <= n <=
 * 16384, nvec <= 64.  Asynchronous on the bound stream; pods_syev2_status reports a hand-off
 * timeout after the stream has drained. */
int pods_syev2(pods_ctx* ctx, const double* C_dev, int n, int nvec, double* lambda_desc_dev,
               double* vec_dev);
int pods_syev2_status(pods_ctx* ctx);
/* Diagnostics: copy `count` doubles of the last pods_syev2's workspace to the host:
 * what = 0 the stage-1 band (n x 64, band[c*64 + d] = A[c+d][c]), 1 the same after stage 2,
 * 2 the tridiagonal {D (n), E (n-1)}, 3 the reduced dense matrix (n x n). */
int pods_syev2_inspect(pods_ctx* ctx, int n, int nvec, int what, double* out_host, int64_t count);

/* Spatial modes Phi = ((A-m) T[:, :nm]) * (1/lambda) / ns (PODFS.py:1330-1333).
 * T_dev: ns x ldT row-major.  phi_dev: 3*P_local x nm row-major (reference layout).
 * lambda_host is copied before the call returns; stream-ordered (no synchronisation). */
int pods_spatial_modes(pods_ctx* ctx, const double* T_dev, int ldT, const double* lambda_host,
                       int nm, double* phi_dev);
/* The same with lambda on the device (1/lambda formed there, IEEE division as numpy's). */
int pods_spatial_modes_dev(pods_ctx* ctx, const double* T_dev, int ldT, const double* lambda_dev,
                           int nm, double* phi_dev);

/* Twiddle table of the DFT below, made on the host by the reference expression itself
 * (podsgen.host.dft_twiddles: np.exp(-1j*2*k*np.pi*time/period), PODFS.py:1566) so that the
 * device never evaluates sin/cos: w_host holds R x ns (cos, sin) pairs, row q = k for
 * q < nk (nk = ns/2 for even ns, ns/2 + 1 for odd), and for even ns a last row for
 * k = -ns/2; R = nk + (ns even).  Kept on the device for (ns, t_host, period) (synchronous). */
int pods_fourier_twiddles(pods_ctx* ctx, int ns, const double* t_host, double period, const double* w_host);
/* Shifted direct DFT of the temporal modes (PODFS.py:1562-1571), bit-exact:
 * c[n][i] = sum_m T[m][i] exp(-1j 2 k pi t_m / period) / ns,  k = n - ns//2, in numpy's
 * pairwise complex summation order, complex64 interleaved (re, im), row-major ns x nm.
 * t_host / period must be the ones of the last pods_fourier_twiddles (else PODS_ERR_STATE).
 * Asynchronous: enqueued on the bound stream and returns (the summation program is kept on
 * the device and re-uploaded only when ns changes). */
int pods_fourier(pods_ctx* ctx, const double* T_dev, int ldT, int nm, int ns,
                 const double* t_host, double period, float* c_dev);

/* Ranking and energy count of the Fourier coefficients (PODFS.py:1575-1593):
 * per mode i, c_ind[i][:] = indices n ordered by (|c[n][i]| as float32, n) descending
 * (sorted(zip(cmod, idx), reverse=True)), and c_count[i] = the number of leading
 * coefficients whose float64 running sum of |c| first reaches float64(sum_f32 |c|) * et;
 * 0 when that target is not positive, -1 when it is never reached (et > 1; the
 * reference raises IndexError).  c_dev: pods_fourier's ns x nm complex64 output.
 * c_ind_dev: nm x ns int32, c_count_dev: nm int64 (device).  ns <= 16384.
 * Asynchronous, like pods_fourier. */
int pods_fourier_rank(pods_ctx* ctx, const float* c_dev, int nm, int ns, double et,
                      int32_t* c_ind_dev, int64_t* c_count_dev);

/* ---- unit-level entry points (reference operator API, one call each) ------------- */
/* filter3DSciPy1D(x, y, ...) (:100-140) on one host block x of shape
 * (2nfx+1, 2nfy+J, 2nfz+K) C-order -> y (J, K). */
int pods_filter_block(pods_ctx* ctx, const double* x_host, int nfx, int nfy, int nfz, int jma,
                      int kma, const double* bx, const double* by, const double* bz,
                      double* y_host);
/* adapt1d / adapt2prf (:143-231) and/or rotate_velocity (:1119-1131) on one step's fields
 * yu, yv, yw (P doubles each, host, updated in place).  lund_host: 9 x P rows as in
 * pods_df_configure (ignored for PODS_LUND_NONE); rot_host: 3x3 row-major or NULL. */
int pods_lund_apply(pods_ctx* ctx, double* yu, double* yv, double* yw, int64_t P,
                    const double* lund_host, int lund_mode, const double* rot_host);
/* The first n doubles of np.random.RandomState(seed).uniform(low, low+range) computed
 * on the device with jump-ahead substreams; out_dev: n doubles. */
int pods_rng_uniform(pods_ctx* ctx, uint32_t seed, int64_t n, double low, double range,
                     double* out_dev);

/* ---- host-only self checks (no GPU needed) ------------------------------------------ */
/* MT19937 jump-ahead math check: jumps mt^(1) of `seed` by 624*(nblocks-1) words with the
 * GF(2) polynomial machinery on the host and compares with sequential twisting.
 * Returns PODS_OK when equal. */
int pods_host_mt_jump_check(uint32_t seed, int64_t nblocks);
/* Characteristic polynomial degree found by Berlekamp-Massey (expect 19937). */
int pods_host_mt_charpoly_degree(void);
/* The co-residency rule applied before every persistent (spin-waiting) launch -- k_trd,
 * k_bt_fused, k_pqr, k_sbtrd_win: PODS_OK when grid <= blocks_per_cu x cus (both from the
 * occupancy API at launch time), else PODS_ERR_UNSUPPORTED, which the solvers then return
 * instead of launching a grid whose hand-offs could never complete. */
int pods_host_persistent_grid_fits(int blocks_per_cu, int cus, int64_t grid);

#ifdef __cplusplus
}
#endif
#endif /* PODSGEN_H */

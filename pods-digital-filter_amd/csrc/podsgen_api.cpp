// C ABI of libpodsgen.so (include/podsgen.h): context, buffers, call sequencing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include "mt_host.h"
#include "podsgen.h"
#include "podsgen_kernels.h"
#include "podsgen_ext.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// hipErrorCooperativeLaunchTooLarge comes from pods::check_persistent: a spin-waiting grid
// that the device cannot hold resident at once is refused before launch, not left to time out
#define PODS_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e == hipErrorCooperativeLaunchTooLarge)                                        \
      return fail(PODS_ERR_UNSUPPORTED, std::string(#expr) +                           \
                                            ": persistent grid cannot be co-resident on this device"); \
    if (_e != hipSuccess)                                                               \
      return fail(PODS_ERR_HIP, std::string(#expr) + " failed: " + hipGetErrorString(_e)); \
  } while (0)

#define PODS_TRY try {
#define PODS_CATCH                                          \
  }                                                         \
  catch (const std::exception& e) {                         \
    return fail(PODS_ERR_INTERNAL, std::string("exception: ") + e.what()); \
  }                                                         \
  catch (...) {                                             \
    return fail(PODS_ERR_INTERNAL, "unknown exception");   \
  }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

hipError_t ensure(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return hipSuccess;
  if (b.p) {
    hipError_t e = hipFree(b.p);
    if (e != hipSuccess) return e;
    b.p = nullptr;
    b.bytes = 0;
  }
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e != hipSuccess) {
    b.p = nullptr;
    return e;
  }
  b.bytes = bytes;
  return hipSuccess;
}

void release(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

// numpy pairwise-sum programs (oracle/pods_oracle.py pairwise_program / cpairwise_program)
constexpr int PW_BLOCKSIZE = 128;
constexpr int NPY_BUFSIZE = 8192;

void pw_rec(std::vector<int>& prog, int start, int m) {
  if (m <= PW_BLOCKSIZE) {
    prog.push_back(start);
    prog.push_back(m);
    return;
  }
  int m2 = m / 2;
  m2 -= m2 % 8;
  pw_rec(prog, start, m2);
  pw_rec(prog, start + m2, m - m2);
  prog.push_back(-1);
  prog.push_back(0);
}

std::vector<int> pairwise_program(int n) {
  std::vector<int> prog;
  for (int s = 0; s < n; s += NPY_BUFSIZE) {
    pw_rec(prog, s, std::min(NPY_BUFSIZE, n - s));
    if (s) {
      prog.push_back(-1);
      prog.push_back(0);
    }
  }
  return prog;
}

void cpw_rec(std::vector<int>& prog, int start, int m) {
  if (2 * m <= PW_BLOCKSIZE) {
    prog.push_back(start);
    prog.push_back(m);
    return;
  }
  int h = m - m % 8;
  int m2 = h / 2;
  cpw_rec(prog, start, m2);
  cpw_rec(prog, start + m2, m - m2);
  prog.push_back(-1);
  prog.push_back(0);
}

std::vector<int> cpairwise_program(int n) {
  std::vector<int> prog;
  for (int s = 0; s < n; s += NPY_BUFSIZE) {
    cpw_rec(prog, s, std::min(NPY_BUFSIZE, n - s));
    if (s) {
      prog.push_back(-1);
      prog.push_back(0);
    }
  }
  return prog;
}

// Substream layout of an MT19937 stream of `ntot` doubles (312 per 624-word block).
struct RngLayout {
  int64_t ntot = 0, Bs = 0;
  int G = 0, G1 = 0, G2 = 64;
  std::vector<int> j1_src, j1_poly, j1_dst, j2_src, j2_poly, j2_dst;
};

// One jump level: substream g >= 1 starts from mt^(1) jumped by t^(624(g*Bs - 1)) mod phi
// (seed-independent polynomials, cached per layout), so every substream state is one
// independent job of a single k_mt_jump launch.
RngLayout make_layout(int64_t ntot) {
  RngLayout L;
  L.ntot = ntot;
  const int64_t blocks = (ntot + 311) / 312;
  // about 2048 substreams (PODS_MT_SUBSTREAMS overrides the target): more substreams shorten
  // the generator's per-substream twist chains but add jump-ahead jobs
  const char* env = std::getenv("PODS_MT_SUBSTREAMS");
  const int64_t target = env ? std::max(64, std::atoi(env)) : 2048;
  int64_t want = (blocks + target - 1) / target;
  int64_t Bs = 1024;
  while (Bs < want) Bs *= 2;
  L.Bs = Bs;
  L.G = (int)std::max<int64_t>(1, (blocks + Bs - 1) / Bs);
  L.G1 = 1;
  L.G2 = std::max(1, L.G - 1);
  for (int g = 1; g < L.G; ++g) {
    L.j2_src.push_back(0);
    L.j2_poly.push_back(g);
    L.j2_dst.push_back(g);
  }
  return L;
}

struct RngBuffers {
  DevBuf states, bases, poly1, poly2, j1, j2;
  int64_t Bs_loaded = 0;
  int G1_loaded = 0, G2_loaded = 0;
  std::vector<uint32_t> seed_host;  // 2 x 624 staging (mt^(0), mt^(1))
  void free_all() {
    release(states); release(bases); release(poly1); release(poly2); release(j1); release(j2);
    Bs_loaded = 0;
    G1_loaded = 0;
    G2_loaded = 0;
  }
};

// Multi-GPU state exchange (pods_df_set_exchange): the stream cut into world * (about 2048)
// substreams of Bs blocks, owner r twisting substreams [g_lo, g_hi) once; the start state of
// every rank's row segment in every plane is recorded by that segment's owner and sent to the
// rank in one all_to_all (the caller's collective, pods_df_exchange_buffers); each rank then
// regenerates only its own segments from those states (k_mt_chains).
struct Exchange {
  bool on = false;
  int world = 1, rank = 0;
  int64_t Bs = 0, blocks = 0;
  int G = 0, g_lo = 0, g_hi = 0;
  int nrec_out = 0, nseg = 0;                        // records this rank sends, segments it makes
  std::vector<int64_t> send_counts, recv_counts;     // records per peer
  DevBuf poly2, jobs, states, bases;                 // the owner's jump-ahead
  DevBuf ch_b0, ch_nb, rec_block, rec_slot, rec_first;  // phase A (record)
  DevBuf seg_b0, seg_nb;                             // phase C (segments)
  uint32_t* send = nullptr;                          // caller-owned (pods_df_exchange_bind)
  uint32_t* recv = nullptr;
  std::vector<uint32_t> seed_host;
  uint32_t seed = 0;
  void free_all() {
    for (DevBuf* b : {&poly2, &jobs, &states, &bases, &ch_b0, &ch_nb, &rec_block, &rec_slot, &rec_first, &seg_b0,
                      &seg_nb})
      release(*b);
    send = recv = nullptr;
    on = false;
  }
};

// SYRK work items {bi, bj, split, 0}: split-major, then 8x8 super-blocks of 128x128 tiles
// in the lower triangle, tiles row-major inside a super-block.  Consecutive items go to one
// XCD, so the 64 workgroups an XCD holds at once (two per CU) cover one super-block: 16
// panels, one K range.
std::vector<int> syrk_items(int ns, int nsplit) {
  std::vector<int> it;
  auto push = [&](int bi, int bj, int s) {
    it.push_back(bi);
    it.push_back(bj);
    it.push_back(s);
    it.push_back(0);
  };
  const int T = 128, SB = 8;
  const int nb = (ns + T - 1) / T;
  const int nsb = (nb + SB - 1) / SB;
  for (int s = 0; s < nsplit; ++s)
    for (int I = 0; I < nsb; ++I)
      for (int Jb = 0; Jb <= I; ++Jb)
        for (int bi = I * SB; bi < std::min(nb, (I + 1) * SB); ++bi)
          for (int bj = Jb * SB; bj < std::min(nb, (Jb + 1) * SB); ++bj)
            if (bj <= bi) push(bi, bj, s);
  return it;
}

}  // namespace

// One eigenvalues-only tridiagonalisation in flight (pods_eigvals_*): its own workspace, so
// several matrices can be at different column ranges at once.
struct EigvalSlot {
  DevBuf wm, x, flags, det, v, cnt, lam;
  int n = 0, R = 0, klast = 0;
  int next = 0;       // next unit: ranges 0..klast, then klast + 1 = the bisection
  bool active = false;
  pods::TrdArgs args{};
  // n > 4096: the two-stage solver in units (stage-1 panel groups, chase sweep-group ranges,
  // the eigenvalues); flags: 64 panel flags, 64 abort words, n sweep counters
  bool two = false;
  DevBuf ws2;
  pods::SyevdPlan plan{};
  uint32_t epoch = 0;
  size_t flag_words = 0;
};

struct pods_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool configured = false;
  pods_df_params p{};
  int NX = 0, NY = 0, NZ = 0, Kp = 0, jl = 0;
  int64_t S = 0, Sl = 0, Pl = 0, rowlen = 0, rowpad = 0;  // rowpad: rowlen rounded up to 16
  RngLayout layout;
  RngBuffers rng;
  Exchange xch;
  // the other snapshot bank (pods_select_snapshots): a second A with its mean / scale / state, so
  // a multi-GPU run can generate step k while step k-1's spatial modes still read its snapshots
  struct SnapBank {
    DevBuf A, mean, devmax;
    bool have_snapshots = false, mean_valid = false, centered = false, dev_valid = false;
  } alt;
  int bank = 0;
  DevBuf R, T1, A, mean, lund, taps, rot, prog_mean, prog_dft, mag, lam, cwork, items, spwork, prog_rank;
  DevBuf e_wm, e_x, e_flags, e_det, e_v, e_t, e_part, e_w2, e_inv, e_cnt;  // pods_syev workspace
  int e_G = 0;
  DevBuf e2_ws, e2_flags, e2_ipiv;  // pods_syev2 (two-stage) workspace
  size_t e2_flag_words = 0;
  uint32_t e2_epoch = 0;
  int nitems = 0;
  int64_t items_key = -1;
  int64_t lund_sj = 0;  // j-stride of the Lund table (0: constant along j)
  int nprog_mean = 0, nleaf_mean = 0;
  bool mean_valid = false;
  bool have_snapshots = false;  // A holds ns x rowlen snapshots (generated or loaded)
  bool centered = false;        // A holds A - mean (pods_center); consumers subtract zero
  DevBuf zero;                  // rowpad zeros: the mean operand once A is centred
  std::vector<double> stage;  // host staging for small uploads
  // device-resident DFT / ranking programs and time axis, re-uploaded only on change
  int dft_ns = -1, dft_nprog = 0, dft_nleaf = 0, rank_ns = -1, rank_nprog = 0;
  std::vector<double> dft_t;
  // host twiddle table of the DFT (pods_fourier_twiddles) and the time axis it was made for
  DevBuf dft_w;
  int dft_w_ns = -1;
  double dft_w_period = 0.0;
  std::vector<double> dft_w_t;
  std::vector<EigvalSlot> eslots;
  DevBuf sub_part, sub_R, sub_cheb, sub_ct;  // subspace iteration: Gram partials, G / R^{-1}, split-K
                                             // partials, the tiled copy of C
  const double* sub_ct_src = nullptr;        // the C that sub_ct holds (pods_cheb_prepare)
  int sub_ct_n = 0;
  DevBuf inv_lam;  // 1 / lambda of the spatial modes (its own buffer: no reuse hazard with lam)
  // pinned staging ring for small host -> device uploads: a slot is reused only after the
  // event recorded behind its copy, so uploads need no stream synchronisation
  static constexpr int kStageSlots = 16;
  static constexpr size_t kStageSlot = 64 * 1024;
  char* pin = nullptr;
  hipEvent_t pin_ev[kStageSlots] = {};
  bool pin_used[kStageSlots] = {};
  int pin_next = 0;
  // marker recorded behind a tridiagonalisation column range of the next pods_syev
  // (pods_syev_marker), for work another stream may start once that range is done
  hipEvent_t marker = nullptr;
  int marker_after = -1;
  bool marker_recorded = false;
  // the same behind the whole tridiagonalisation (pods_syev_marker_tail)
  hipEvent_t marker_tail = nullptr;
  bool marker_tail_req = false, marker_tail_recorded = false;
  // pods_syev: k_larft on a second stream beside the bisection and eigenvectors of T
  hipStream_t aux = nullptr;
  hipEvent_t aux_fork = nullptr, aux_join = nullptr;
  int marker_tail_where = 0;  // 0: behind the tridiagonalisation, 1: behind the eigenvalues
  // pods_set_shared_device: the per-device lock file persistent launches hold (-1: not shared)
  int lock_fd = -1;
  // pods_corr: 1 = exact int8-MFMA modular products + CRT (podsgen_corr_i8.hip), 0 = fp64 MFMA
  // SYRK; PODS_CORR=f64 selects 0 at pods_create
  int corr_mode = 1;
  DevBuf devmax;           // max |fl(a - mean)| (k_mean / k_absdev), the int8 path's scale
  bool dev_valid = false;  // devmax belongs to the current snapshots and mean
  DevBuf i8_res, i8_part, i8_items, i8_xitems, i8_pace;  // + the persistent SYRK's table, counters
  int i8_per_xcd = 0;
  // the int8 plan's inputs, compared field by field (every one of them changes the plan)
  struct I8Key {
    int ns = -1;
    int64_t rowlen = -1, rowpad = -1, budget = -1;
    int force = -1;
    char order = 0;  // PODS_CORR_ORDER (diagnostic library only)
    bool operator==(const I8Key& o) const {
      return ns == o.ns && rowlen == o.rowlen && rowpad == o.rowpad && budget == o.budget && force == o.force &&
             order == o.order;
    }
  } i8_key;
  pods::CorrI8Plan i8_plan{};
  // pods_corr_timing: HIP events around each int8 SYRK launch (the roofline kernel), read back
  // by pods_corr_kernel_ms
  bool corr_timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> corr_ev;
  size_t corr_ev_used = 0;
};

namespace {

// Persistent grids (k_trd, k_bt_fused, k_pqr, k_sbtrd_win) spin on hand-offs between their own
// workgroups, so all of them must be resident at once.  Two processes on one device can each
// hold part of the CUs and starve the other's grid until its spin limit aborts it (r3's 2-rank
// run on one GPU).  With pods_set_shared_device every entry point that launches one takes this
// per-device file lock first and keeps it until its stream has drained.
class PersistentLock {
 public:
  explicit PersistentLock(pods_ctx* c) : c_(c) {
    if (c_->lock_fd >= 0) held_ = flock(c_->lock_fd, LOCK_EX) == 0;
  }
  // drain the stream, then unlock (the success path of the entry point)
  int release() {
    if (!held_) return PODS_OK;
    const hipError_t e = hipStreamSynchronize(c_->stream);
    (void)flock(c_->lock_fd, LOCK_UN);
    held_ = false;
    if (e != hipSuccess) return fail(PODS_ERR_HIP, std::string("persistent grid: ") + hipGetErrorString(e));
    return PODS_OK;
  }
  ~PersistentLock() {
    if (held_) {
      (void)hipStreamSynchronize(c_->stream);
      (void)flock(c_->lock_fd, LOCK_UN);
    }
  }
  PersistentLock(const PersistentLock&) = delete;
  PersistentLock& operator=(const PersistentLock&) = delete;

 private:
  pods_ctx* c_;
  bool held_ = false;
};

// dst_dev <- bytes of src (host) on the context's stream, without synchronising it: through
// the pinned ring (slot reused after its copy's event), or a synchronous copy when too large
hipError_t stage_upload(pods_ctx* c, void* dst_dev, const void* src, size_t bytes) {
  if (bytes == 0) return hipSuccess;
  if (bytes > pods_ctx::kStageSlot) {
    hipError_t e = hipMemcpyAsync(dst_dev, src, bytes, hipMemcpyHostToDevice, c->stream);
    return e != hipSuccess ? e : hipStreamSynchronize(c->stream);
  }
  hipError_t e = hipSuccess;
  if (!c->pin) {
    e = hipHostMalloc(reinterpret_cast<void**>(&c->pin), pods_ctx::kStageSlots * pods_ctx::kStageSlot,
                      hipHostMallocDefault);
    if (e != hipSuccess) {
      c->pin = nullptr;
      return e;
    }
    for (int i = 0; i < pods_ctx::kStageSlots; ++i) {
      e = hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
  }
  const int sl = c->pin_next;
  c->pin_next = (sl + 1) % pods_ctx::kStageSlots;
  if (c->pin_used[sl]) {
    e = hipEventSynchronize(c->pin_ev[sl]);
    if (e != hipSuccess) return e;
  }
  char* slot = c->pin + (size_t)sl * pods_ctx::kStageSlot;
  std::memcpy(slot, src, bytes);
  e = hipMemcpyAsync(dst_dev, slot, bytes, hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) return e;
  e = hipEventRecord(c->pin_ev[sl], c->stream);
  c->pin_used[sl] = e == hipSuccess;
  return e;
}


int upload_rng(pods_ctx* c, const RngLayout& L, uint32_t seed, RngBuffers& rb) {
  using namespace pods::mt;
  const JumpTables& jt = jump_tables(L.Bs, L.G2, std::max(L.G1, 1));
  PODS_HIP(ensure(rb.states, (size_t)L.G * N * 4));
  PODS_HIP(ensure(rb.bases, (size_t)std::max(L.G1, 1) * N * 4));
  if (rb.Bs_loaded != L.Bs || rb.G1_loaded < L.G1 || rb.G2_loaded != L.G2) {
    PODS_HIP(ensure(rb.poly1, (size_t)std::max(L.G1, 1) * N * 4));
    PODS_HIP(ensure(rb.poly2, (size_t)(L.G2 + 1) * N * 4));
    PODS_HIP(hipMemcpy(rb.poly1.p, jt.level1.data(), (size_t)std::max(L.G1, 1) * N * 4,
                       hipMemcpyHostToDevice));
    PODS_HIP(hipMemcpy(rb.poly2.p, jt.level2.data(), (size_t)(L.G2 + 1) * N * 4,
                       hipMemcpyHostToDevice));
    rb.Bs_loaded = L.Bs;
    rb.G1_loaded = L.G1;
    rb.G2_loaded = L.G2;
  }
  const size_t n1 = L.j1_src.size(), n2 = L.j2_src.size();
  std::vector<int> jobs;
  jobs.insert(jobs.end(), L.j1_src.begin(), L.j1_src.end());
  jobs.insert(jobs.end(), L.j1_poly.begin(), L.j1_poly.end());
  jobs.insert(jobs.end(), L.j1_dst.begin(), L.j1_dst.end());
  jobs.insert(jobs.end(), L.j2_src.begin(), L.j2_src.end());
  jobs.insert(jobs.end(), L.j2_poly.begin(), L.j2_poly.end());
  jobs.insert(jobs.end(), L.j2_dst.begin(), L.j2_dst.end());
  PODS_HIP(ensure(rb.j1, jobs.size() * sizeof(int) + 16));
  PODS_HIP(hipMemcpy(rb.j1.p, jobs.data(), jobs.size() * sizeof(int), hipMemcpyHostToDevice));
  (void)n1;
  (void)n2;
  rb.seed_host.assign(2 * N, 0);
  seed_state(seed, rb.seed_host.data());
  std::memcpy(rb.seed_host.data() + N, rb.seed_host.data(), N * 4);
  twist(rb.seed_host.data() + N);
  return PODS_OK;
}

// Enqueue: seed states, level-1 and level-2 jumps (stream-ordered after the uploads).
int run_jumps(pods_ctx* c, const RngLayout& L, RngBuffers& rb) {
  using namespace pods::mt;
  PODS_HIP(hipMemcpyAsync(rb.states.p, rb.seed_host.data(), N * 4, hipMemcpyHostToDevice, c->stream));
  PODS_HIP(hipMemcpyAsync(rb.bases.p, rb.seed_host.data() + N, N * 4, hipMemcpyHostToDevice,
                          c->stream));
  const int n1 = (int)L.j1_src.size(), n2 = (int)L.j2_src.size();
  const int* jb = rb.j1.as<int>();
  PODS_HIP(pods::launch_mt_jump(rb.bases.as<uint32_t>(), jb, rb.poly1.as<uint32_t>(), jb + n1,
                                rb.bases.as<uint32_t>(), jb + 2 * n1, n1, c->stream));
  const int* j2 = jb + 3 * n1;
  PODS_HIP(pods::launch_mt_jump(rb.bases.as<uint32_t>(), j2, rb.poly2.as<uint32_t>(), j2 + n2,
                                rb.states.as<uint32_t>(), j2 + 2 * n2, n2, c->stream));
  return PODS_OK;
}

int check_ctx(pods_ctx* c) {
  if (!c) return fail(PODS_ERR_ARG, "null context");
  return PODS_OK;
}

}  // namespace

extern "C" {

const char* pods_last_error(void) { return g_err.c_str(); }
int pods_abi_version(void) { return PODS_ABI_VERSION; }

int pods_create(pods_ctx** out, int device) {
  PODS_TRY
  if (!out) return fail(PODS_ERR_ARG, "out is null");
  *out = nullptr;
  int n = 0;
  PODS_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n)
    return fail(PODS_ERR_ARG, "device " + std::to_string(device) + " out of range (" +
                                  std::to_string(n) + " devices)");
  PODS_HIP(hipSetDevice(device));
  pods_ctx* c = new pods_ctx();
  c->device = device;
  if (const char* cm = std::getenv("PODS_CORR")) c->corr_mode = std::string(cm) == "f64" ? 0 : 1;
  *out = c;
  return PODS_OK;
  PODS_CATCH
}

int pods_destroy(pods_ctx* c) {
  PODS_TRY
  if (!c) return PODS_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->R, &c->T1, &c->A, &c->mean, &c->lund, &c->taps, &c->rot, &c->prog_mean,
                    &c->prog_dft, &c->mag, &c->lam, &c->cwork, &c->items, &c->e_wm,
                    &c->e_x, &c->e_flags, &c->e_det, &c->e_v, &c->e_t, &c->e_part, &c->e_w2,
                    &c->e_inv, &c->e_cnt, &c->spwork, &c->prog_rank, &c->zero, &c->e2_ws, &c->e2_flags,
                    &c->e2_ipiv, &c->dft_w})
    release(*b);
  c->rng.free_all();
  c->xch.free_all();
  for (DevBuf* b : {&c->alt.A, &c->alt.mean, &c->alt.devmax}) release(*b);
  release(c->sub_part);
  release(c->sub_R);
  release(c->sub_cheb);
  release(c->sub_ct);
  for (EigvalSlot& sl : c->eslots)
    for (DevBuf* b : {&sl.wm, &sl.x, &sl.flags, &sl.det, &sl.v, &sl.cnt, &sl.lam, &sl.ws2}) release(*b);
  release(c->inv_lam);
  for (DevBuf* b : {&c->devmax, &c->i8_res, &c->i8_part, &c->i8_items, &c->i8_xitems, &c->i8_pace}) release(*b);
  for (auto& ev : c->corr_ev) {
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  if (c->pin) {
    for (int i = 0; i < pods_ctx::kStageSlots; ++i)
      if (c->pin_ev[i]) (void)hipEventDestroy(c->pin_ev[i]);
    (void)hipHostFree(c->pin);
  }
  if (c->marker) (void)hipEventDestroy(c->marker);
  if (c->marker_tail) (void)hipEventDestroy(c->marker_tail);
  if (c->aux_fork) (void)hipEventDestroy(c->aux_fork);
  if (c->aux_join) (void)hipEventDestroy(c->aux_join);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->lock_fd >= 0) (void)close(c->lock_fd);
  delete c;
  return PODS_OK;
  PODS_CATCH
}

int pods_set_stream(pods_ctx* c, void* stream) {
  if (int e = check_ctx(c)) return e;
  c->stream = static_cast<hipStream_t>(stream);
  return PODS_OK;
}

int pods_synchronize(pods_ctx* c) {
  if (int e = check_ctx(c)) return e;
  PODS_HIP(hipStreamSynchronize(c->stream));
  return PODS_OK;
}

int pods_set_shared_device(pods_ctx* c, int shared) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (c->lock_fd >= 0) {
    (void)close(c->lock_fd);
    c->lock_fd = -1;
  }
  if (!shared) return PODS_OK;
  char bus[64] = {0};
  PODS_HIP(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, c->device));
  std::string path = "/tmp/podsgen-gpu-";
  for (const char* q = bus; *q; ++q) path += (*q == ':' || *q == '.') ? '-' : *q;
  path += ".lock";
  const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return fail(PODS_ERR_STATE, "pods_set_shared_device: cannot open " + path);
  c->lock_fd = fd;
  return PODS_OK;
  PODS_CATCH
}

namespace {
// np.mean's pairwise program over ns snapshots (k_mean), uploaded once per snapshot count.
int upload_mean_program(pods_ctx* c, int ns) {
  std::vector<int> prog = pairwise_program(ns);
  c->nprog_mean = (int)prog.size() / 2;
  // the leaves (start, length) in program order follow the program (k_mean_leaves)
  int nleaf = 0;
  for (int k = 0; k < c->nprog_mean; ++k)
    if (prog[2 * k] >= 0) ++nleaf;
  const std::vector<int> ops(prog);
  for (int k = 0; k < c->nprog_mean; ++k)
    if (ops[2 * k] >= 0) prog.insert(prog.end(), {ops[2 * k], ops[2 * k + 1]});
  c->nleaf_mean = nleaf;
  PODS_HIP(ensure(c->prog_mean, prog.size() * sizeof(int)));
  PODS_HIP(hipMemcpy(c->prog_mean.p, prog.data(), prog.size() * sizeof(int), hipMemcpyHostToDevice));
  return PODS_OK;
}
}  // namespace

int pods_df_configure(pods_ctx* c, const pods_df_params* prm, const double* bx, const double* by,
                      const double* bz, const double* lund_host, const double* rot_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!prm || !bx || !by || !bz) return fail(PODS_ERR_ARG, "null params/taps");
  const pods_df_params& p = *prm;
  if (p.jma <= 0 || p.kma <= 0 || p.ns <= 0) return fail(PODS_ERR_ARG, "jma, kma, ns must be > 0");
  if (p.nfx < 0 || p.nfy < 0 || p.nfz < 0) return fail(PODS_ERR_ARG, "negative filter width");
  if (2 * p.nfx + 1 > 49) return fail(PODS_ERR_UNSUPPORTED, "2*nfx+1 > 49 taps");
  if (2 * p.nfy + 1 > 25) return fail(PODS_ERR_UNSUPPORTED, "2*nfy+1 > 25 taps");
  if (p.j0 < 0 || p.j1 > p.jma || p.j0 >= p.j1) return fail(PODS_ERR_ARG, "bad row slab [j0, j1)");
  if (p.lund_mode != PODS_LUND_1D && p.lund_mode != PODS_LUND_PRF && p.lund_mode != PODS_LUND_NONE)
    return fail(PODS_ERR_ARG, "bad lund_mode");
  if (p.lund_mode != PODS_LUND_NONE && !lund_host) return fail(PODS_ERR_ARG, "lund_host is null");
  if (p.rotate && !rot_host) return fail(PODS_ERR_ARG, "rot_host is null");
  PODS_HIP(hipSetDevice(c->device));
  if (c->bank == 1) {  // back to bank 0; the other bank is rebuilt on demand for the new shape
    std::swap(c->A, c->alt.A);
    std::swap(c->mean, c->alt.mean);
    std::swap(c->devmax, c->alt.devmax);
    c->bank = 0;
  }
  for (DevBuf* b : {&c->alt.A, &c->alt.mean, &c->alt.devmax}) release(*b);
  c->alt = pods_ctx::SnapBank{};
  c->p = p;
  c->NX = 2 * p.nfx + 1;
  c->NY = 2 * p.nfy + 1;
  c->NZ = 2 * p.nfz + 1;
  c->Kp = p.kma + 2 * p.nfz;
  c->jl = p.j1 - p.j0;
  c->S = (int64_t)(p.jma + 2 * p.nfy) * c->Kp;
  c->Sl = (int64_t)(c->jl + 2 * p.nfy) * c->Kp;
  c->Pl = (int64_t)c->jl * p.kma;
  c->rowlen = 3 * c->Pl;
  c->rowpad = (c->rowlen + 15) / 16 * 16;
  if (p.kma > pods::filter_yz_max_K(c->Kp))
    return fail(PODS_ERR_UNSUPPORTED, "kma too large for the y/z filter kernel");
  const int64_t nplanes = 3 * (int64_t)(c->NX + p.ns - 1);
  const int64_t ntot = nplanes * c->S;  // doubles of the stream that reach A
  c->layout = make_layout(ntot);
  PODS_HIP(ensure(c->R, (size_t)nplanes * c->Sl * sizeof(double)));
  PODS_HIP(ensure(c->T1, (size_t)3 * p.ns * c->Sl * sizeof(double)));
  PODS_HIP(ensure(c->A, (size_t)p.ns * c->rowpad * sizeof(double)));
  PODS_HIP(ensure(c->mean, (size_t)c->rowpad * sizeof(double)));
  // padded K columns of the K-tiled snapshot matrix (and of the mean) stay zero
  PODS_HIP(hipMemset(c->A.p, 0, (size_t)p.ns * c->rowpad * sizeof(double)));
  PODS_HIP(hipMemset(c->mean.p, 0, (size_t)c->rowpad * sizeof(double)));
  PODS_HIP(ensure(c->lund, (size_t)std::max<int64_t>(9 * c->Pl, pods::lund_chunk_size(c->jl, p.kma)) *
                                sizeof(double)));
  PODS_HIP(ensure(c->taps, (size_t)(c->NX + c->NY + c->NZ) * sizeof(double)));
  PODS_HIP(ensure(c->rot, 9 * sizeof(double)));
  std::vector<double> taps(c->NX + c->NY + c->NZ);
  std::copy(bx, bx + c->NX, taps.begin());
  std::copy(by, by + c->NY, taps.begin() + c->NX);
  std::copy(bz, bz + c->NZ, taps.begin() + c->NX + c->NY);
  PODS_HIP(hipMemcpy(c->taps.p, taps.data(), taps.size() * sizeof(double), hipMemcpyHostToDevice));
  c->lund_sj = p.kma;
  if (lund_host) {
    // a profile that does not vary along j (adapt1d's 1-D profiles) is staged per block in LDS
    // from its first row; a j-varying one is stored chunk-major (coalesced 16-B loads)
    bool same = true;
    for (int e = 0; e < 9 && same; ++e) {
      const double* row0 = lund_host + (int64_t)e * c->Pl;
      for (int jj = 1; jj < c->jl && same; ++jj)
        same = std::memcmp(row0, row0 + (int64_t)jj * p.kma, (size_t)p.kma * sizeof(double)) == 0;
    }
    if (same) {
      c->lund_sj = 0;
      PODS_HIP(hipMemcpy(c->lund.p, lund_host, (size_t)9 * c->Pl * sizeof(double), hipMemcpyHostToDevice));
    } else {
      std::vector<double> ch((size_t)pods::lund_chunk_size(c->jl, p.kma), 0.0);
      for (int64_t jj = 0; jj < c->jl; ++jj)
        for (int e = 0; e < 9; ++e)
          for (int k = 0; k < p.kma; ++k)
            ch[pods::lund_chunk_index(jj, e, k, p.kma)] = lund_host[(int64_t)e * c->Pl + jj * p.kma + k];
      PODS_HIP(hipMemcpy(c->lund.p, ch.data(), ch.size() * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  double r9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (p.rotate) std::memcpy(r9, rot_host, sizeof(r9));
  PODS_HIP(hipMemcpy(c->rot.p, r9, sizeof(r9), hipMemcpyHostToDevice));
  if (int e = upload_mean_program(c, p.ns)) return e;
  if (int e = upload_rng(c, c->layout, p.seed, c->rng)) return e;
  c->xch.free_all();  // a new configuration: pods_df_set_exchange again for a multi-GPU run
  c->configured = true;
  c->have_snapshots = false;
  c->mean_valid = false;
  c->dev_valid = false;
  c->centered = false;
  return PODS_OK;
  PODS_CATCH
}

int pods_df_set_exchange(pods_ctx* c, int world, int rank, const int* j0s, const int* j1s) {
  PODS_TRY
  using namespace pods::mt;
  if (int e = check_ctx(c)) return e;
  if (!c->configured) return fail(PODS_ERR_STATE, "pods_df_set_exchange before pods_df_configure");
  Exchange& X = c->xch;
  X.free_all();
  if (world <= 0) return PODS_OK;  // off
  // world == 1 is allowed (its all_to_all is the identity): a one-rank job can run the exchange
  // path, e.g. to exercise a collective backend on a single device (tests)
  const pods_df_params& p = c->p;
  if (rank < 0 || rank >= world || !j0s || !j1s) return fail(PODS_ERR_ARG, "pods_df_set_exchange: bad rank/slabs");
  if (j0s[rank] != p.j0 || j1s[rank] != p.j1)
    return fail(PODS_ERR_ARG, "pods_df_set_exchange: this rank's slab differs from the configured one");
  for (int q = 0; q < world; ++q)
    if (j0s[q] < 0 || j1s[q] > p.jma || j0s[q] >= j1s[q]) return fail(PODS_ERR_ARG, "pods_df_set_exchange: bad slab");
  if (c->S < 312) return fail(PODS_ERR_UNSUPPORTED, "pods_df_set_exchange: planes shorter than one block");
  PODS_HIP(hipSetDevice(c->device));
  const int64_t nplanes = 3 * (int64_t)(c->NX + p.ns - 1);
  const int64_t ntot = nplanes * c->S;
  X.world = world;
  X.rank = rank;
  X.blocks = (ntot + 311) / 312;
  // the owners' substreams are 1/world of the one-GPU length, so a chain is as long as ... / world
  // (short streams: at least 8 substreams per rank)
  X.Bs = std::max<int64_t>(1, std::min<int64_t>((c->layout.Bs + world - 1) / world, X.blocks / (8 * (int64_t)world)));
  X.G = (int)((X.blocks + X.Bs - 1) / X.Bs);
  if (X.G < world) return fail(PODS_ERR_UNSUPPORTED, "pods_df_set_exchange: stream too short for the ranks");
  std::vector<int> glo(world + 1);
  for (int r = 0; r <= world; ++r) glo[r] = (int)((int64_t)X.G * r / world);
  X.g_lo = glo[rank];
  X.g_hi = glo[rank + 1];
  auto owner = [&](int64_t block) {
    const int g = (int)(block / X.Bs);
    return (int)(std::upper_bound(glo.begin(), glo.end(), g) - glo.begin()) - 1;
  };
  // jump jobs of this owner's substreams g >= 1: mt^(1) jumped by t^(624 (g Bs - 1)) mod phi
  const int pfirst = std::max(1, X.g_lo);
  const int npoly = X.g_hi - pfirst;
  if (npoly > 0) {
    const JumpTables& jt = jump_tables(X.Bs, std::max(1, X.G - 1), 1);
    PODS_HIP(ensure(X.poly2, (size_t)npoly * N * 4));
    PODS_HIP(hipMemcpy(X.poly2.p, &jt.level2[(size_t)pfirst * N], (size_t)npoly * N * 4, hipMemcpyHostToDevice));
    std::vector<int> jobs(3 * (size_t)npoly);
    for (int k = 0; k < npoly; ++k) {
      jobs[k] = 0;                              // source: mt^(1)
      jobs[npoly + k] = k;                      // polynomial of substream pfirst + k
      jobs[2 * npoly + k] = pfirst + k - X.g_lo;  // local state index
    }
    PODS_HIP(ensure(X.jobs, jobs.size() * sizeof(int)));
    PODS_HIP(hipMemcpy(X.jobs.p, jobs.data(), jobs.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  const int nch = X.g_hi - X.g_lo;
  PODS_HIP(ensure(X.states, (size_t)nch * N * 4));
  PODS_HIP(ensure(X.bases, (size_t)N * 4));
  X.seed_host.assign(2 * N, 0);
  seed_state(p.seed, X.seed_host.data());
  std::memcpy(X.seed_host.data() + N, X.seed_host.data(), N * 4);
  twist(X.seed_host.data() + N);
  // phase A chains and the records: every rank's segment start in every plane whose block this
  // rank owns, grouped by target rank (plane order within), sorted by block for the chains
  std::vector<int64_t> cb0(nch);
  std::vector<int> cnb(nch);
  for (int k = 0; k < nch; ++k) {
    const int64_t g = X.g_lo + k;
    cb0[k] = g * X.Bs;
    cnb[k] = (int)std::min<int64_t>(X.Bs, X.blocks - g * X.Bs);
  }
  X.send_counts.assign(world, 0);
  X.recv_counts.assign(world, 0);
  std::vector<std::pair<int64_t, int>> recs;  // (block, slot)
  std::vector<int64_t> send_off(world + 1, 0);
  for (int q = 0; q < world; ++q) {
    for (int64_t pl = 0; pl < nplanes; ++pl) {
      const int64_t b = (pl * c->S + (int64_t)j0s[q] * c->Kp) / 312;
      const int r = owner(b);
      if (r == rank) recs.push_back({b, (int)(send_off[q] + X.send_counts[q]++)});
      if (q == rank) ++X.recv_counts[r];
    }
    send_off[q + 1] = send_off[q] + X.send_counts[q];
  }
  std::stable_sort(recs.begin(), recs.end(),
                   [](const std::pair<int64_t, int>& a, const std::pair<int64_t, int>& b) { return a.first < b.first; });
  X.nrec_out = (int)recs.size();
  std::vector<int64_t> rb(recs.size());
  std::vector<int> rs(recs.size()), rf(nch + 1, 0);
  for (size_t k = 0; k < recs.size(); ++k) {
    rb[k] = recs[k].first;
    rs[k] = recs[k].second;
    ++rf[(int)(recs[k].first / X.Bs) - X.g_lo + 1];
  }
  for (int k = 0; k < nch; ++k) rf[k + 1] += rf[k];
  // phase C: this rank's segment of every plane (the 2nfy halo rows included)
  X.nseg = (int)nplanes;
  std::vector<int64_t> sb0(nplanes);
  std::vector<int> snb(nplanes);
  for (int64_t pl = 0; pl < nplanes; ++pl) {
    const int64_t s0 = pl * c->S + (int64_t)p.j0 * c->Kp;
    const int64_t s1 = std::min(ntot, pl * c->S + (int64_t)(p.j1 + 2 * p.nfy) * c->Kp);
    sb0[pl] = s0 / 312;
    snb[pl] = (int)((s1 + 311) / 312 - sb0[pl]);
  }
  auto up = [&](DevBuf& d, const void* src, size_t bytes) -> hipError_t {
    hipError_t e = ensure(d, bytes);
    if (e == hipSuccess && bytes) e = hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice);
    return e;
  };
  PODS_HIP(up(X.ch_b0, cb0.data(), cb0.size() * 8));
  PODS_HIP(up(X.ch_nb, cnb.data(), cnb.size() * 4));
  PODS_HIP(up(X.rec_block, rb.data(), rb.size() * 8));
  PODS_HIP(up(X.rec_slot, rs.data(), rs.size() * 4));
  PODS_HIP(up(X.rec_first, rf.data(), rf.size() * 4));
  PODS_HIP(up(X.seg_b0, sb0.data(), sb0.size() * 8));
  PODS_HIP(up(X.seg_nb, snb.data(), snb.size() * 4));
  X.on = true;
  return PODS_OK;
  PODS_CATCH
}

int pods_df_exchange_sizes(pods_ctx* c, int64_t* send_bytes, int64_t* recv_bytes) {
  if (int e = check_ctx(c)) return e;
  const Exchange& X = c->xch;
  if (!X.on) return fail(PODS_ERR_STATE, "pods_df_exchange_sizes: no exchange configured");
  for (int r = 0; r < X.world; ++r) {
    if (send_bytes) send_bytes[r] = X.send_counts[r] * pods::mt::N * 4;
    if (recv_bytes) recv_bytes[r] = X.recv_counts[r] * pods::mt::N * 4;
  }
  return PODS_OK;
}

int pods_df_exchange_bind(pods_ctx* c, void* send_dev, void* recv_dev) {
  if (int e = check_ctx(c)) return e;
  Exchange& X = c->xch;
  if (!X.on) return fail(PODS_ERR_STATE, "pods_df_exchange_bind: no exchange configured");
  if (!send_dev || !recv_dev) return fail(PODS_ERR_ARG, "pods_df_exchange_bind: null buffer");
  X.send = static_cast<uint32_t*>(send_dev);
  X.recv = static_cast<uint32_t*>(recv_dev);
  return PODS_OK;
}

// workgroups per CU of the x pass beside the solver's tail, in halves (variant builds: -DPODS_XPASS_CAP=)
#ifndef PODS_XPASS_CAP
#define PODS_XPASS_CAP 4
#endif
int pods_df_generate_parts(pods_ctx* c, int parts) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->configured) return fail(PODS_ERR_STATE, "pods_df_generate before pods_df_configure");
  if (parts & ~(PODS_GEN_ALL | PODS_GEN_BESIDE_SOLVER | PODS_GEN_RECORD))
    return fail(PODS_ERR_ARG, "bad generation parts");
  PODS_HIP(hipSetDevice(c->device));
  const pods_df_params& p = c->p;
  const RngLayout& L = c->layout;
  Exchange& X = c->xch;
  if (X.on) {
    // the multi-GPU state exchange: JUMP = this owner's substreams, RECORD = its segment-start
    // records (the caller then runs the all_to_all), PLANES = this rank's segments
    using pods::mt::N;
    if ((parts & (PODS_GEN_RECORD | PODS_GEN_PLANES)) && (!X.send || !X.recv))
      return fail(PODS_ERR_STATE, "exchange buffers not bound (pods_df_exchange_bind)");
    if (parts & PODS_GEN_JUMP) {
      if (X.g_lo == 0)
        PODS_HIP(hipMemcpyAsync(X.states.p, X.seed_host.data(), N * 4, hipMemcpyHostToDevice, c->stream));
      PODS_HIP(hipMemcpyAsync(X.bases.p, X.seed_host.data() + N, N * 4, hipMemcpyHostToDevice, c->stream));
      const int pfirst = std::max(1, X.g_lo), npoly = X.g_hi - pfirst;
      if (npoly > 0) {
        const int* jb = X.jobs.as<int>();
        PODS_HIP(pods::launch_mt_jump(X.bases.as<uint32_t>(), jb, X.poly2.as<uint32_t>(), jb + npoly,
                                      X.states.as<uint32_t>(), jb + 2 * npoly, npoly, c->stream));
      }
    }
    if (parts & PODS_GEN_RECORD) {
      const int64_t ntot = 3 * (int64_t)(c->NX + p.ns - 1) * c->S;
      PODS_HIP(pods::launch_mt_chains(0, X.states.as<uint32_t>(), X.ch_b0.as<int64_t>(), X.ch_nb.as<int>(),
                                      X.g_hi - X.g_lo, X.rec_block.as<int64_t>(), X.rec_slot.as<int>(),
                                      X.rec_first.as<int>(), X.send, ntot, c->S, c->Kp, 0, 0, c->Sl,
                                      p.rng_low, p.rng_range, nullptr, c->stream));
    }
    if (parts & PODS_GEN_PLANES) {
      const int64_t ntot = 3 * (int64_t)(c->NX + p.ns - 1) * c->S;
      PODS_HIP(pods::launch_mt_chains(1, X.recv, X.seg_b0.as<int64_t>(), X.seg_nb.as<int>(), X.nseg,
                                      nullptr, nullptr, nullptr, nullptr, ntot, c->S, c->Kp, p.j0,
                                      p.j1 + 2 * p.nfy, c->Sl, p.rng_low, p.rng_range, c->R.as<double>(),
                                      c->stream));
    }
  } else if (parts & PODS_GEN_RECORD) {
    return fail(PODS_ERR_STATE, "PODS_GEN_RECORD without pods_df_set_exchange");
  }
  if (!X.on && (parts & PODS_GEN_JUMP)) {
    if (int e = run_jumps(c, L, c->rng)) return e;
  }
  if (!X.on && (parts & PODS_GEN_PLANES)) {
    PODS_HIP(pods::launch_mt_generate(c->rng.states.as<uint32_t>(), L.G, L.Bs, L.ntot, c->S, c->Kp, p.j0,
                                      p.j1 + 2 * p.nfy, c->Sl, p.rng_low, p.rng_range, c->R.as<double>(),
                                      c->stream, (parts & PODS_GEN_BESIDE_SOLVER) ? 2 : 0));
  }
  const double* taps = c->taps.as<double>();
  if (parts & PODS_GEN_XPASS) {
    // x pass: enough (component, point, step-chunk) threads to fill the chip
    const int64_t pts = 3 * c->Sl;
    int64_t nch = (256LL * 2048 + pts - 1) / pts;
    nch = std::max<int64_t>(1, std::min<int64_t>(nch, std::max(1, p.ns / 16)));
    const int chunk = (int)((p.ns + nch - 1) / nch);
    // beside the eigensolver's tail (PODS_GEN_BESIDE_SOLVER): 2 workgroups per CU, so the
    // latency-bound bisection / eigenvector / back-transformation kernels keep room on every CU
    int cus = 0, dev = 0;
    if ((parts & PODS_GEN_BESIDE_SOLVER) && hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    PODS_HIP(pods::launch_filter_x(c->NX, c->R.as<double>(), taps, p.ns, c->Sl, 3, chunk,
                                   c->T1.as<double>(), c->stream, 0, -1, PODS_XPASS_CAP * cus / 2));
  }
  if (parts & PODS_GEN_YZPASS) {
    PODS_HIP(pods::launch_filter_yz(c->NY, c->T1.as<double>(), taps + c->NX, taps + c->NX + c->NY,
                                    c->NZ, p.ns, c->jl, p.kma, c->Kp, c->Sl, 3, c->lund.as<double>(),
                                    c->lund_sj, p.lund_mode, c->rot.as<double>(), p.rotate,
                                    c->A.as<double>(), c->stream));
    c->have_snapshots = true;
    c->mean_valid = false;
    c->dev_valid = false;
    c->centered = false;
  }
  return PODS_OK;
  PODS_CATCH
}

int pods_df_generate(pods_ctx* c) { return pods_df_generate_parts(c, PODS_GEN_ALL); }

int pods_df_set_seed(pods_ctx* c, uint32_t seed) {
  PODS_TRY
  using namespace pods::mt;
  if (int e = check_ctx(c)) return e;
  if (!c->configured) return fail(PODS_ERR_STATE, "pods_df_set_seed before pods_df_configure");
  c->p.seed = seed;
  // the host seed states (mt^(0), mt^(1)) the next PODS_GEN_JUMP uploads; the jump polynomials
  // do not depend on the seed
  for (std::vector<uint32_t>* h : {&c->rng.seed_host, &c->xch.seed_host}) {
    if (h->size() != 2 * (size_t)N) continue;
    seed_state(seed, h->data());
    std::memcpy(h->data() + N, h->data(), N * 4);
    twist(h->data() + N);
  }
  return PODS_OK;
  PODS_CATCH
}

int pods_select_snapshots(pods_ctx* c, int bank) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (bank != 0 && bank != 1) return fail(PODS_ERR_ARG, "pods_select_snapshots: bank must be 0 or 1");
  if (bank == c->bank) return PODS_OK;
  if (!c->configured) return fail(PODS_ERR_STATE, "pods_select_snapshots before pods_df_configure");
  PODS_HIP(hipSetDevice(c->device));
  pods_ctx::SnapBank& o = c->alt;
  const size_t abytes = (size_t)c->p.ns * c->rowpad * sizeof(double), mbytes = (size_t)c->rowpad * sizeof(double);
  if (o.A.bytes < abytes || o.mean.bytes < mbytes) {
    // padded K rows of the K-tiled matrix (and of the mean) must read as zero, as in bank 0
    PODS_HIP(ensure(o.A, abytes));
    PODS_HIP(ensure(o.mean, mbytes));
    PODS_HIP(hipMemsetAsync(o.A.p, 0, abytes, c->stream));
    PODS_HIP(hipMemsetAsync(o.mean.p, 0, mbytes, c->stream));
  }
  PODS_HIP(ensure(o.devmax, sizeof(double)));
  std::swap(c->A, o.A);
  std::swap(c->mean, o.mean);
  std::swap(c->devmax, o.devmax);
  std::swap(c->have_snapshots, o.have_snapshots);
  std::swap(c->mean_valid, o.mean_valid);
  std::swap(c->centered, o.centered);
  std::swap(c->dev_valid, o.dev_valid);
  c->bank = bank;
  return PODS_OK;
  PODS_CATCH
}

int pods_df_snapshots(pods_ctx* c, double** a_dev, int64_t* row_len) {
  if (int e = check_ctx(c)) return e;
  if (!c->configured && !c->have_snapshots) return fail(PODS_ERR_STATE, "no snapshot buffer");
  if (a_dev) *a_dev = c->A.as<double>();
  if (row_len) *row_len = c->rowlen;
  return PODS_OK;
}

int pods_set_snapshots(pods_ctx* c, const double* at, int ns, int64_t rowlen) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!at || ns <= 0 || rowlen <= 0) return fail(PODS_ERR_ARG, "bad snapshot matrix");
  PODS_HIP(hipSetDevice(c->device));
  const int64_t rowpad = (rowlen + 15) / 16 * 16;
  // host-side re-layout into the K-tiled device layout (podsgen_kernels.hip at_off)
  std::vector<double> tiled((size_t)ns * rowpad, 0.0);
  for (int64_t kb = 0; kb < rowpad / 16; ++kb)
    for (int64_t i = 0; i < ns; ++i)
      for (int64_t e = 0; e < 16; ++e) {
        const int64_t r = kb * 16 + e;
        if (r < rowlen) tiled[(size_t)((kb * ns + i) * 16 + e)] = at[(size_t)(i * rowlen + r)];
      }
  PODS_HIP(ensure(c->A, tiled.size() * sizeof(double)));
  PODS_HIP(ensure(c->mean, (size_t)rowpad * sizeof(double)));
  PODS_HIP(hipMemset(c->mean.p, 0, (size_t)rowpad * sizeof(double)));
  PODS_HIP(hipMemcpy(c->A.p, tiled.data(), tiled.size() * sizeof(double), hipMemcpyHostToDevice));
  if (int e = upload_mean_program(c, ns)) return e;
  c->p = pods_df_params{};
  c->p.ns = ns;
  c->rowlen = rowlen;
  c->rowpad = rowpad;
  c->configured = false;
  c->have_snapshots = true;
  c->mean_valid = false;
  c->dev_valid = false;
  c->centered = false;
  return PODS_OK;
  PODS_CATCH
}

int pods_copy(pods_ctx* c, void* dst, const void* src, size_t bytes, int kind) {
  if (int e = check_ctx(c)) return e;
  if (!dst || !src) return fail(PODS_ERR_ARG, "null pointer");
  if (bytes == 0) return PODS_OK;
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                          : kind == 1 ? hipMemcpyDeviceToHost
                                      : hipMemcpyDeviceToDevice;
  if (kind < 0 || kind > 2) return fail(PODS_ERR_ARG, "bad copy kind");
  PODS_HIP(hipMemcpyAsync(dst, src, bytes, k, c->stream));
  if (kind != 2) PODS_HIP(hipStreamSynchronize(c->stream));
  return PODS_OK;
}

int pods_mean(pods_ctx* c, double* mean_out, int out_is_device) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots) return fail(PODS_ERR_STATE, "pods_mean before snapshots exist");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(ensure(c->devmax, sizeof(double)));
  PODS_HIP(pods::launch_mean(c->A.as<double>(), c->rowlen, c->p.ns, c->prog_mean.as<int>(),
                             c->nprog_mean, c->mean.as<double>(), c->stream, c->devmax.as<double>(),
                             c->nleaf_mean));
  c->mean_valid = true;
  c->dev_valid = true;
  if (mean_out) {
    const size_t bytes = (size_t)c->rowlen * sizeof(double);
    if (out_is_device) {
      PODS_HIP(hipMemcpyAsync(mean_out, c->mean.p, bytes, hipMemcpyDeviceToDevice, c->stream));
    } else {
      PODS_HIP(hipMemcpyAsync(mean_out, c->mean.p, bytes, hipMemcpyDeviceToHost, c->stream));
      PODS_HIP(hipStreamSynchronize(c->stream));
    }
  }
  return PODS_OK;
  PODS_CATCH
}

int pods_corr(pods_ctx* c, double* C_dev, int divide) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots || !c->mean_valid) return fail(PODS_ERR_STATE, "pods_corr needs pods_mean first");
  if (!C_dev) return fail(PODS_ERR_ARG, "C_dev is null");
  PODS_HIP(hipSetDevice(c->device));
  const int ns = c->p.ns;
  const double* mean = c->centered ? c->zero.as<double>() : c->mean.as<double>();
  if (c->corr_mode == 1) {
    const char* bud = std::getenv("PODS_CORR_BUDGET_GB");
    const int64_t budget = (int64_t)((bud ? std::atof(bud) : 16.0) * (double)(1LL << 30));
    const char* fsp = std::getenv("PODS_CORR_SPLITS");  // tests: a fixed number of K splits
    const int force = fsp ? std::max(0, std::atoi(fsp)) : 0;
    pods_ctx::I8Key key;
    key.ns = ns;
    key.rowlen = c->rowlen;
    key.rowpad = c->rowpad;
    key.budget = budget;
    key.force = force;
#ifdef PODS_DIAG
    if (const char* ord = std::getenv("PODS_CORR_ORDER")) key.order = ord[0];
#endif
    if (!(c->i8_key == key)) {
      if (pods::corr_i8_plan(ns, c->rowlen, c->rowpad, budget, &c->i8_plan, force) != 0)
        return fail(PODS_ERR_UNSUPPORTED, "pods_corr: K too large for the int8 correlation (PODS_CORR=f64)");
      const std::vector<int> items = pods::corr_i8_items(ns, c->i8_plan);
      c->i8_plan.nitems = (int)(items.size() / 4);  // the order decides the (padded) item count
      PODS_HIP(ensure(c->i8_items, items.size() * sizeof(int)));
      PODS_HIP(hipMemcpy(c->i8_items.p, items.data(), items.size() * sizeof(int), hipMemcpyHostToDevice));
      const std::vector<int> xit = pods::corr_i8_xcd_items(items, c->i8_plan.nitems, &c->i8_per_xcd);
      PODS_HIP(ensure(c->i8_xitems, xit.size() * sizeof(int)));
      PODS_HIP(hipMemcpy(c->i8_xitems.p, xit.data(), xit.size() * sizeof(int), hipMemcpyHostToDevice));
      PODS_HIP(ensure(c->i8_pace, 8 * 32 * sizeof(unsigned)));
      c->i8_key = key;
    }
    PODS_HIP(ensure(c->i8_res, (size_t)(c->i8_plan.r_bytes + pods::CORR_I8_RPAD)));
    PODS_HIP(ensure(c->i8_part, (size_t)c->i8_plan.p_bytes));
    PODS_HIP(ensure(c->devmax, sizeof(double)));
    if (!c->dev_valid) {
      PODS_HIP(pods::launch_absdev(c->A.as<double>(), ns, c->rowlen, c->rowpad, mean, c->devmax.as<double>(),
                                   c->stream));
      c->dev_valid = true;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->corr_timing) {
      if (c->corr_ev_used == c->corr_ev.size()) {
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        PODS_HIP(hipEventCreate(&ev.first));
        PODS_HIP(hipEventCreate(&ev.second));
        c->corr_ev.push_back(ev);
      }
      e0 = c->corr_ev[c->corr_ev_used].first;
      e1 = c->corr_ev[c->corr_ev_used].second;
      ++c->corr_ev_used;
    }
    PODS_HIP(pods::launch_corr_i8(c->A.as<double>(), ns, c->rowlen, c->rowpad, mean, c->devmax.as<double>(),
                                  c->i8_plan, c->i8_items.as<int>(), c->i8_res.as<int8_t>(),
                                  c->i8_part.as<uint8_t>(), C_dev, ns, divide, c->stream, e0, e1,
                                  c->i8_xitems.as<int>(), c->i8_per_xcd, c->i8_pace.as<unsigned>()));
    return PODS_OK;
  }
  int64_t ksplit = 0;
  const int nsplit = pods::syrk_plan(ns, c->rowpad, &ksplit);
  PODS_HIP(ensure(c->cwork, (size_t)nsplit * ns * ns * sizeof(double)));
  const int64_t key = ((int64_t)ns << 20) | nsplit;
  if (c->items_key != key) {
    std::vector<int> items = syrk_items(ns, nsplit);
    PODS_HIP(ensure(c->items, items.size() * sizeof(int)));
    PODS_HIP(hipMemcpy(c->items.p, items.data(), items.size() * sizeof(int), hipMemcpyHostToDevice));
    c->nitems = (int)items.size() / 4;
    c->items_key = key;
  }
  PODS_HIP(pods::launch_syrk(c->A.as<double>(), ns, c->rowpad, mean, c->items.as<int>(), c->nitems, nsplit,
                             ksplit, C_dev, ns, divide, c->cwork.as<double>(), c->centered ? 1 : 0, c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_set_corr_mode(pods_ctx* c, int mode) {
  if (int e = check_ctx(c)) return e;
  if (mode != 0 && mode != 1) return fail(PODS_ERR_ARG, "corr mode must be 0 (fp64) or 1 (int8 CRT)");
  c->corr_mode = mode;
  return PODS_OK;
}

int pods_corr_timing(pods_ctx* c, int enable) {
  if (int e = check_ctx(c)) return e;
  c->corr_timing = enable != 0;
  c->corr_ev_used = 0;
  return PODS_OK;
}

int pods_corr_kernel_ms(pods_ctx* c, double* total_ms, int* count) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!total_ms || !count) return fail(PODS_ERR_ARG, "null output");
  double t = 0.0;
  for (size_t k = 0; k < c->corr_ev_used; ++k) {
    PODS_HIP(hipEventSynchronize(c->corr_ev[k].second));
    float ms = 0.0f;
    PODS_HIP(hipEventElapsedTime(&ms, c->corr_ev[k].first, c->corr_ev[k].second));
    t += ms;
  }
  *total_ms = t;
  *count = (int)c->corr_ev_used;
  c->corr_ev_used = 0;
  return PODS_OK;
  PODS_CATCH
}

int pods_corr_i8_plan_query(int ns, int64_t row_len, int64_t row_pad, int64_t budget_bytes, int force_split,
                            int64_t* out) {
  PODS_TRY
  if (!out || ns <= 0 || row_len <= 0 || row_pad < row_len || budget_bytes <= 0)
    return fail(PODS_ERR_ARG, "pods_corr_i8_plan_query: bad arguments");
  pods::CorrI8Plan p{};
  if (pods::corr_i8_plan(ns, row_len, row_pad, budget_bytes, &p, std::max(0, force_split)) != 0)
    return fail(PODS_ERR_UNSUPPORTED, "pods_corr_i8_plan_query: no int8 plan for this shape");
  const int64_t v[8] = {p.bbits, p.nlaunch, p.nsplit, p.kcs, p.chunks, p.r_bytes, p.p_bytes,
                        p.chunks * ns * 64};
  for (int k = 0; k < 8; ++k) out[k] = v[k];
  return PODS_OK;
  PODS_CATCH
}

int pods_get_corr_mode(pods_ctx* c, int* mode) {
  if (int e = check_ctx(c)) return e;
  if (!mode) return fail(PODS_ERR_ARG, "mode is null");
  *mode = c->corr_mode;
  return PODS_OK;
}

int pods_center(pods_ctx* c) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots || !c->mean_valid) return fail(PODS_ERR_STATE, "pods_center needs pods_mean first");
  if (c->centered) return PODS_OK;
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(ensure(c->zero, (size_t)c->rowpad * sizeof(double)));
  PODS_HIP(hipMemsetAsync(c->zero.p, 0, (size_t)c->rowpad * sizeof(double), c->stream));
  PODS_HIP(pods::launch_center(c->A.as<double>(), c->rowpad, c->p.ns, c->mean.as<double>(), c->stream));
  c->centered = true;
  return PODS_OK;
  PODS_CATCH
}

int pods_set_mean(pods_ctx* c, const double* mean_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots) return fail(PODS_ERR_STATE, "pods_set_mean before snapshots exist");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(hipMemsetAsync(c->mean.p, 0, (size_t)c->rowpad * sizeof(double), c->stream));
  if (mean_host) {
    PODS_HIP(hipMemcpyAsync(c->mean.p, mean_host, (size_t)c->rowlen * sizeof(double),
                            hipMemcpyHostToDevice, c->stream));
    PODS_HIP(hipStreamSynchronize(c->stream));
  }
  c->mean_valid = true;
  c->dev_valid = false;
  c->centered = false;  // an explicit mean is subtracted by the consumers again
  return PODS_OK;
  PODS_CATCH
}

int pods_lund_apply(pods_ctx* c, double* yu, double* yv, double* yw, int64_t P, const double* lund,
                    int lund_mode, const double* rot) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!yu || !yv || !yw || P <= 0) return fail(PODS_ERR_ARG, "bad fields");
  if (lund_mode >= 0 && !lund) return fail(PODS_ERR_ARG, "lund_host is null");
  PODS_HIP(hipSetDevice(c->device));
  DevBuf d;
  const size_t fb = (size_t)P * sizeof(double);
  hipError_t e = ensure(d, 3 * fb + 9 * fb + 9 * sizeof(double));
  if (e) return fail(PODS_ERR_NOMEM, "device allocation failed");
  double* base = d.as<double>();
  double* du = base;
  double* dv = base + P;
  double* dw = base + 2 * P;
  double* dl = base + 3 * P;
  double* dr = base + 12 * P;
  double r9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (rot) std::memcpy(r9, rot, sizeof(r9));
  if (!e) e = hipMemcpy(du, yu, fb, hipMemcpyHostToDevice);
  if (!e) e = hipMemcpy(dv, yv, fb, hipMemcpyHostToDevice);
  if (!e) e = hipMemcpy(dw, yw, fb, hipMemcpyHostToDevice);
  if (!e && lund_mode >= 0) e = hipMemcpy(dl, lund, 9 * fb, hipMemcpyHostToDevice);
  if (!e) e = hipMemcpy(dr, r9, sizeof(r9), hipMemcpyHostToDevice);
  if (!e) e = pods::launch_lund_apply(du, dv, dw, P, dl, lund_mode, dr, rot ? 1 : 0, c->stream);
  if (!e) e = hipStreamSynchronize(c->stream);
  if (!e) e = hipMemcpy(yu, du, fb, hipMemcpyDeviceToHost);
  if (!e) e = hipMemcpy(yv, dv, fb, hipMemcpyDeviceToHost);
  if (!e) e = hipMemcpy(yw, dw, fb, hipMemcpyDeviceToHost);
  release(d);
  if (e) return fail(PODS_ERR_HIP, std::string("lund_apply: ") + hipGetErrorString(e));
  return PODS_OK;
  PODS_CATCH
}

int pods_divide_inplace(pods_ctx* c, double* x, int64_t n, double d) {
  if (int e = check_ctx(c)) return e;
  PODS_HIP(pods::launch_divide(x, n, d, c->stream));
  return PODS_OK;
}

int pods_copy_snapshots(pods_ctx* c, int i0, int i1, double* out_dev) {
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots) return fail(PODS_ERR_STATE, "pods_copy_snapshots: no snapshots");
  if (!out_dev || i0 < 0 || i1 > c->p.ns || i0 > i1) return fail(PODS_ERR_ARG, "pods_copy_snapshots: bad range");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(pods::launch_gather_snapshots(c->A.as<double>(), c->p.ns, c->rowlen, i0, i1, out_dev, c->stream));
  return PODS_OK;
}

int pods_cheb_prepare(pods_ctx* c, const double* C, int n) {
  if (int e = check_ctx(c)) return e;
  if (!C || n < 1) return fail(PODS_ERR_ARG, "pods_cheb_prepare: bad arguments");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(ensure(c->sub_ct, pods::cheb_tiled_doubles(n) * sizeof(double)));
  PODS_HIP(pods::launch_tile_c(C, n, n, c->sub_ct.as<double>(), c->stream));
  c->sub_ct_src = C;
  c->sub_ct_n = n;
  return PODS_OK;
}

int pods_cheb_step(pods_ctx* c, const double* C, int n, const double* Y, const double* Z, int m, double alpha,
                   double beta, double gamma, double* out) {
  if (int e = check_ctx(c)) return e;
  if (!C || !Y || !out || n < 1 || m != 64 || out == Y || (Z && out == Z))
    return fail(PODS_ERR_ARG, "pods_cheb_step: bad arguments (m = 64, out distinct)");
  if (C != c->sub_ct_src || n != c->sub_ct_n)
    return fail(PODS_ERR_STATE, "pods_cheb_step: C was not prepared (pods_cheb_prepare)");
  PODS_HIP(ensure(c->sub_cheb, (size_t)pods::cheb_splits(n) * n * 64 * sizeof(double)));
  PODS_HIP(pods::launch_cheb_step(c->sub_ct.as<double>(), n, Y, Z, m, alpha, beta, gamma, c->sub_cheb.as<double>(),
                                  out, c->stream));
  return PODS_OK;
}

int pods_gram(pods_ctx* c, const double* Y, const double* Z, int n, int m, double* G) {
  if (int e = check_ctx(c)) return e;
  if (!Y || !Z || !G || n < 1 || m != 64) return fail(PODS_ERR_ARG, "pods_gram: bad arguments (m = 64)");
  PODS_HIP(ensure(c->sub_part, (size_t)pods::gram_slices(n) * m * m * sizeof(double)));
  PODS_HIP(pods::launch_gram(Y, Z, n, c->sub_part.as<double>(), G, c->stream));
  return PODS_OK;
}

int pods_cholqr(pods_ctx* c, const double* Y, int n, int m, double* X) {
  if (int e = check_ctx(c)) return e;
  if (!Y || !X || X == Y || n < m || m != 64) return fail(PODS_ERR_ARG, "pods_cholqr: bad arguments");
  PODS_HIP(ensure(c->sub_part, (size_t)pods::gram_slices(n) * m * m * sizeof(double)));
  PODS_HIP(ensure(c->sub_R, (size_t)2 * m * m * sizeof(double)));
  double* G = c->sub_R.as<double>();
  double* Rinv = G + m * m;
  PODS_HIP(pods::launch_gram(Y, Y, n, c->sub_part.as<double>(), G, c->stream));
  PODS_HIP(pods::launch_chol_inv(G, Rinv, c->stream));
  PODS_HIP(pods::launch_right_mul(Y, Rinv, nullptr, n, m, X, c->stream));
  return PODS_OK;
}

int pods_right_mul(pods_ctx* c, const double* Y, const double* M, int n, int m, double* out) {
  if (int e = check_ctx(c)) return e;
  if (!Y || !M || !out || out == Y || n < 1 || m < 16 || m % 16) return fail(PODS_ERR_ARG, "pods_right_mul: bad arguments");
  PODS_HIP(pods::launch_right_mul(Y, M, nullptr, n, m, out, c->stream));
  return PODS_OK;
}

int pods_ritz_residual(pods_ctx* c, const double* X, const double* CX, const double* H, int n, int m, double* E) {
  if (int e = check_ctx(c)) return e;
  if (!X || !CX || !H || !E || E == X || E == CX || n < 1 || m < 16 || m % 16)
    return fail(PODS_ERR_ARG, "pods_ritz_residual: bad arguments");
  PODS_HIP(pods::launch_right_mul(X, H, CX, n, m, E, c->stream));
  return PODS_OK;
}

int pods_pack_lower(pods_ctx* c, const double* C, int n, double* packed) {
  if (int e = check_ctx(c)) return e;
  if (!C || !packed || n < 1) return fail(PODS_ERR_ARG, "pods_pack_lower: bad arguments");
  PODS_HIP(pods::launch_pack_lower(C, n, n, packed, c->stream));
  return PODS_OK;
}

int pods_unpack_lower(pods_ctx* c, const double* packed, int n, double divisor, double* C) {
  if (int e = check_ctx(c)) return e;
  if (!C || !packed || n < 1) return fail(PODS_ERR_ARG, "pods_unpack_lower: bad arguments");
  PODS_HIP(pods::launch_unpack_lower(packed, n, divisor, C, n, c->stream));
  return PODS_OK;
}

int pods_temporal_modes(pods_ctx* c, const double* V, int64_t v_rs, int64_t v_cs,
                        const double* lam_desc, int nvalid, int ncols, double* T) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!V || !T || !lam_desc) return fail(PODS_ERR_ARG, "null pointer");
  const int ns = c->have_snapshots ? c->p.ns : 0;
  if (ns <= 0) return fail(PODS_ERR_STATE, "no snapshots");
  if (ncols <= 0 || ncols > ns || nvalid > ncols) return fail(PODS_ERR_ARG, "bad ncols/nvalid");
  PODS_HIP(ensure(c->lam, (size_t)ncols * sizeof(double)));
  PODS_HIP(ensure(c->mag, (size_t)ncols * sizeof(double)));
  PODS_HIP(stage_upload(c, c->lam.p, lam_desc, (size_t)ncols * sizeof(double)));
  PODS_HIP(pods::launch_temporal(V, v_rs, v_cs, ns, ncols, std::max(nvalid, 0), c->lam.as<double>(),
                                 c->mag.as<double>(), T, c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_temporal_modes_dev(pods_ctx* c, const double* V, int64_t v_rs, int64_t v_cs,
                            const double* lam_desc_dev, int nvalid, int ncols, double* T) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!V || !T || !lam_desc_dev) return fail(PODS_ERR_ARG, "null pointer");
  const int ns = c->have_snapshots ? c->p.ns : 0;
  if (ns <= 0) return fail(PODS_ERR_STATE, "no snapshots");
  if (ncols <= 0 || ncols > ns || nvalid > ncols) return fail(PODS_ERR_ARG, "bad ncols/nvalid");
  PODS_HIP(ensure(c->mag, (size_t)ncols * sizeof(double)));
  PODS_HIP(pods::launch_temporal(V, v_rs, v_cs, ns, ncols, std::max(nvalid, 0), lam_desc_dev,
                                 c->mag.as<double>(), T, c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_spatial_modes_dev(pods_ctx* c, const double* T, int ldT, const double* lam_dev, int nm, double* phi) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots || !c->mean_valid) return fail(PODS_ERR_STATE, "pods_spatial_modes needs pods_mean");
  if (!T || !lam_dev || !phi || nm <= 0 || ldT < nm) return fail(PODS_ERR_ARG, "bad arguments");
  PODS_HIP(ensure(c->inv_lam, (size_t)nm * sizeof(double)));
  PODS_HIP(pods::launch_recip(lam_dev, nm, c->inv_lam.as<double>(), c->stream));
  const size_t wb = pods::spatial_work_bytes(c->rowlen, c->p.ns);
  if (wb) PODS_HIP(ensure(c->spwork, wb));
  PODS_HIP(pods::launch_spatial(c->A.as<double>(), c->rowlen, c->p.ns,
                                c->centered ? c->zero.as<double>() : c->mean.as<double>(), T, ldT, nm,
                                c->inv_lam.as<double>(), phi, wb ? c->spwork.as<double>() : nullptr, c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_spatial_modes(pods_ctx* c, const double* T, int ldT, const double* lam, int nm, double* phi) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->have_snapshots || !c->mean_valid) return fail(PODS_ERR_STATE, "pods_spatial_modes needs pods_mean");
  if (!T || !lam || !phi || nm <= 0 || ldT < nm) return fail(PODS_ERR_ARG, "bad arguments");
  PODS_HIP(ensure(c->inv_lam, (size_t)nm * sizeof(double)));
  c->stage.resize(nm);
  for (int m = 0; m < nm; ++m) c->stage[m] = 1.0 / lam[m];  // np.ones(nm)/energy (PODFS.py:1331)
  PODS_HIP(stage_upload(c, c->inv_lam.p, c->stage.data(), (size_t)nm * sizeof(double)));
  const size_t wb = pods::spatial_work_bytes(c->rowlen, c->p.ns);
  if (wb) PODS_HIP(ensure(c->spwork, wb));
  PODS_HIP(pods::launch_spatial(c->A.as<double>(), c->rowlen, c->p.ns,
                                c->centered ? c->zero.as<double>() : c->mean.as<double>(), T, ldT, nm,
                                c->inv_lam.as<double>(), phi, wb ? c->spwork.as<double>() : nullptr, c->stream));
  return PODS_OK;
  PODS_CATCH
}

namespace {

// Tridiagonalisation into the context workspace: D at e_det, E at +n, tau at +2n.
int run_sytrd(pods_ctx* c, const double* C, int n, int* R_out, int64_t* trace = nullptr,
              int trace_wg = 0) {
  int R = 0, G = 0;
  int64_t slab = 0;
  if (pods::trd_plan(n, &R, &G, &slab) != 0)
    return fail(PODS_ERR_UNSUPPORTED, "pods_syev: n = " + std::to_string(n) + " > 4096");
  PODS_HIP(ensure(c->e_wm, (size_t)slab * sizeof(double)));
  PODS_HIP(ensure(c->e_x, (size_t)32 * pods::TRD_HANDOFF * sizeof(double)));  // 2 vectors x 8 XCD copies x 2 parities x n
  PODS_HIP(ensure(c->e_flags, 64));
  PODS_HIP(ensure(c->e_det, ((size_t)4 * n + 8) * sizeof(double)));
  PODS_HIP(ensure(c->e_v, (size_t)std::max(n - 1, 1) * n * sizeof(double)));
  PODS_HIP(hipMemsetAsync(c->e_flags.p, 0, 64, c->stream));
  PODS_HIP(hipMemsetAsync(c->e_x.p, 0, (size_t)32 * pods::TRD_HANDOFF * sizeof(double), c->stream));
  c->e_G = 0;
  double* det = c->e_det.as<double>();
  pods::TrdArgs a{};
  a.C = C;
  a.ldc = n;
  a.n = n;
  a.G = G;
  a.klast = (n - 1) / 512;
  a.Wm = c->e_wm.as<double>();
  a.pbuf = c->e_x.as<double>();
  a.rbuf = c->e_x.as<double>() + 16 * (int64_t)pods::TRD_HANDOFF;
  a.flags = c->e_flags.as<uint32_t>();
  a.D = det;
  a.E = det + n;
  a.tau = det + 2 * (int64_t)n;
  a.V = c->e_v.as<double>();
  a.ldv = n;
  a.trace = trace;
  a.trace_wg = trace_wg;
  a.nrep = 8;  // one hand-off copy per XCD (-0.8 ms at n = 4096 against a single copy)
  const int mk = c->marker_after;
  c->marker_after = -1;
  c->marker_recorded = false;
  if (mk >= 0 && mk < a.klast && c->marker) {
    PODS_HIP(pods::launch_trd_ranges(a, R, 0, mk, c->stream));
    PODS_HIP(hipEventRecord(c->marker, c->stream));
    c->marker_recorded = true;
    PODS_HIP(pods::launch_trd_ranges(a, R, mk + 1, a.klast, c->stream));
  } else {
    PODS_HIP(pods::launch_trd(a, R, c->stream));
  }
  c->marker_tail_recorded = false;
  if (c->marker_tail_req && c->marker_tail && c->marker_tail_where == 0) {
    PODS_HIP(hipEventRecord(c->marker_tail, c->stream));
    c->marker_tail_recorded = true;
    c->marker_tail_req = false;
  }
  *R_out = R;
  return PODS_OK;
}

}  // namespace

namespace {
constexpr int EIGVAL_SLOTS = 16;

// two-stage units: PANEL_UNIT stage-1 panels (32 columns each) or CHASE_UNIT sweep groups (two
// sweeps each) per unit; at n = 8192: 8 + 8 units and the eigenvalues
constexpr int PANEL_UNIT = 32, CHASE_UNIT = 512;
int two_panel_units(const EigvalSlot& sl) { return (sl.plan.np + PANEL_UNIT - 1) / PANEL_UNIT; }
int two_chase_units(const EigvalSlot& sl) { return (pods::syevd2_groups(sl.n) + CHASE_UNIT - 1) / CHASE_UNIT; }

int eigval_units(const EigvalSlot& sl) {
  if (sl.two) return two_panel_units(sl) + two_chase_units(sl) + 1;
  return sl.klast + 2;  // trd ranges + the bisection
}

// the slot's abort words: the tridiagonalisation's one, or the two-stage solver's two
uint32_t* slot_abort(const EigvalSlot& sl) { return sl.flags.as<uint32_t>() + (sl.two ? 64 : 0); }
int slot_abort_words(const EigvalSlot& sl) { return sl.two ? 2 : 1; }

int eigval_run_two(pods_ctx* c, EigvalSlot& sl, int end) {
  const int npu = two_panel_units(sl), ncu = two_chase_units(sl);
  double* ws = sl.ws2.as<double>();
  uint32_t* fl = sl.flags.as<uint32_t>();
  for (int u = sl.next; u < end; ++u) {
    if (u < npu) {
      PODS_HIP(pods::syevd2_panels(sl.n, ws, sl.plan, fl, sl.epoch, u * PANEL_UNIT, (u + 1) * PANEL_UNIT, c->stream));
      if (u == npu - 1) PODS_HIP(pods::syevd2_band(sl.n, ws, sl.plan, false, c->stream));
    } else if (u < npu + ncu) {
      const int q0 = (u - npu) * CHASE_UNIT;
      PODS_HIP(pods::syevd2_chase(sl.n, ws, sl.plan, fl, q0, q0 + CHASE_UNIT, c->stream));
    } else {
      PODS_HIP(pods::syevd2_eigvals(sl.n, ws, sl.plan, sl.cnt.as<int>(), sl.lam.as<double>(), c->stream));
    }
  }
  sl.next = end;
  return PODS_OK;
}

// launch the slot's units [next, next + count)
int eigval_run(pods_ctx* c, EigvalSlot& sl, int count) {
  const int total = eigval_units(sl);
  const int end = std::min(total, sl.next + count);
  if (sl.two) return eigval_run_two(c, sl, end);
  if (sl.next <= sl.klast && end > sl.next) {
    const int ke = std::min(end - 1, sl.klast);
    PODS_HIP(pods::launch_trd_ranges(sl.args, sl.R, sl.next, ke, c->stream));
  }
  if (end == total && sl.next < total) {  // the bisection: all n eigenvalues of T
    double* det = sl.det.as<double>();
    PODS_HIP(pods::launch_tri_eigvals(det, det + sl.n, sl.n, det + 3 * (int64_t)sl.n, sl.lam.as<double>(),
                                      sl.cnt.as<int>(), c->stream));
  }
  sl.next = end;
  return PODS_OK;
}
}  // namespace

int pods_eigvals_begin(pods_ctx* c, int slot, const double* C, int n) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= EIGVAL_SLOTS || !C || n < 1) return fail(PODS_ERR_ARG, "pods_eigvals_begin: bad arguments");
  int R = 0, G = 0;
  int64_t slab = 0;
  const bool two = pods::trd_plan(n, &R, &G, &slab) != 0;
  if (two && (n < 3 || n > pods::syev2_max_n()))
    return fail(PODS_ERR_UNSUPPORTED, "pods_eigvals_begin: n = " + std::to_string(n) + " > " +
                                          std::to_string(pods::syev2_max_n()));
  PODS_HIP(hipSetDevice(c->device));
  PersistentLock lk(c);
  if ((int)c->eslots.size() <= slot) c->eslots.resize(slot + 1);
  EigvalSlot& sl = c->eslots[slot];
  if (sl.active && sl.next < eigval_units(sl))
    return fail(PODS_ERR_STATE, "pods_eigvals_begin: slot " + std::to_string(slot) + " still running");
  if (two) {  // the two-stage solver, eigenvalues only, in units (stage 1, chase, eigenvalues)
    const size_t wsd = pods::sy2sb_work_doubles(n, 0, &sl.plan);
    PODS_HIP(ensure(sl.ws2, wsd * sizeof(double)));
    const size_t fw = 128 + (size_t)n;
    if (sl.flag_words < fw) {  // panel flags start zeroed; the epoch keeps their tags apart
      PODS_HIP(ensure(sl.flags, fw * sizeof(uint32_t)));
      PODS_HIP(hipMemsetAsync(sl.flags.p, 0, fw * sizeof(uint32_t), c->stream));
      sl.flag_words = fw;
      sl.epoch = 0;
    }
    PODS_HIP(hipMemsetAsync(sl.flags.as<uint32_t>() + 64, 0, 64 * sizeof(uint32_t), c->stream));  // abort words
    PODS_HIP(ensure(sl.cnt, pods::tri_grid_bytes()));
    PODS_HIP(ensure(sl.lam, (size_t)n * sizeof(double)));
    ++sl.epoch;
    sl.two = true;
    sl.n = n;
    sl.next = 0;
    sl.active = true;
    PODS_HIP(pods::syevd2_begin(C, n, sl.ws2.as<double>(), sl.plan, sl.flags.as<uint32_t>(), c->stream));
    if (int e = eigval_run(c, sl, 1)) return e;  // unit 0, like the tridiagonalisation (C is copied)
    return lk.release();
  }
  if (sl.two) {  // the slot held a two-stage solve before: its flag layout differs
    sl.two = false;
    sl.flag_words = 0;
  }
  PODS_HIP(ensure(sl.wm, (size_t)slab * sizeof(double)));
  PODS_HIP(ensure(sl.x, (size_t)32 * pods::TRD_HANDOFF * sizeof(double)));
  PODS_HIP(ensure(sl.flags, 64));
  PODS_HIP(ensure(sl.det, ((size_t)4 * n + 8) * sizeof(double)));
  PODS_HIP(ensure(sl.v, (size_t)std::max(n - 1, 1) * n * sizeof(double)));
  PODS_HIP(ensure(sl.cnt, pods::tri_grid_bytes()));
  PODS_HIP(ensure(sl.lam, (size_t)n * sizeof(double)));
  PODS_HIP(hipMemsetAsync(sl.flags.p, 0, 64, c->stream));
  PODS_HIP(hipMemsetAsync(sl.x.p, 0, (size_t)32 * pods::TRD_HANDOFF * sizeof(double), c->stream));
  double* det = sl.det.as<double>();
  pods::TrdArgs a{};
  a.C = C;
  a.ldc = n;
  a.n = n;
  a.G = G;
  a.klast = (n - 1) / 512;
  a.Wm = sl.wm.as<double>();
  a.pbuf = sl.x.as<double>();
  a.rbuf = sl.x.as<double>() + 16 * (int64_t)pods::TRD_HANDOFF;
  a.flags = sl.flags.as<uint32_t>();
  a.D = det;
  a.E = det + n;
  a.tau = det + 2 * (int64_t)n;
  a.V = sl.v.as<double>();
  a.ldv = n;
  a.nrep = 8;
  sl.args = a;
  sl.n = n;
  sl.R = R;
  sl.klast = a.klast;
  sl.next = 0;
  sl.active = true;
  if (int e = eigval_run(c, sl, 1)) return e;  // range 0 is the only one that reads C
  return lk.release();
  PODS_CATCH
}

int pods_eigvals_advance(pods_ctx* c, int slot, int max_units, int* remaining) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= (int)c->eslots.size() || !c->eslots[slot].active || max_units < 0)
    return fail(PODS_ERR_ARG, "pods_eigvals_advance: no such slot");
  PODS_HIP(hipSetDevice(c->device));
  EigvalSlot& sl = c->eslots[slot];
  PersistentLock lk(c);
  if (int e = eigval_run(c, sl, max_units)) return e;
  if (remaining) *remaining = eigval_units(sl) - sl.next;
  return lk.release();
  PODS_CATCH
}

int pods_eigvals_fetch(pods_ctx* c, int slot, double* lam_desc_dev) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= (int)c->eslots.size() || !c->eslots[slot].active || !lam_desc_dev)
    return fail(PODS_ERR_ARG, "pods_eigvals_fetch: no such slot");
  EigvalSlot& sl = c->eslots[slot];
  if (sl.next < eigval_units(sl)) return fail(PODS_ERR_STATE, "pods_eigvals_fetch: units still to run");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(hipMemcpyAsync(lam_desc_dev, sl.lam.p, (size_t)sl.n * sizeof(double), hipMemcpyDeviceToDevice,
                          c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_eigvals_status(pods_ctx* c, int slot) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= (int)c->eslots.size() || !c->eslots[slot].active)
    return fail(PODS_ERR_ARG, "pods_eigvals_status: no such slot");
  const EigvalSlot& sl = c->eslots[slot];
  uint32_t abort_word[2] = {0, 0};
  PODS_HIP(hipMemcpyAsync(abort_word, slot_abort(sl), slot_abort_words(sl) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                          c->stream));
  PODS_HIP(hipStreamSynchronize(c->stream));
  if (abort_word[0] || abort_word[1]) return fail(PODS_ERR_INTERNAL, "pods_eigvals: hand-off wait timed out (aborted)");
  return PODS_OK;
  PODS_CATCH
}

int pods_eigvals_flags_async(pods_ctx* c, int slot, uint32_t* flags_dst) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= (int)c->eslots.size() || !c->eslots[slot].active || !flags_dst)
    return fail(PODS_ERR_ARG, "pods_eigvals_flags_async: no such slot");
  PODS_HIP(hipSetDevice(c->device));
  const EigvalSlot& sl = c->eslots[slot];
  PODS_HIP(hipMemcpyAsync(flags_dst, slot_abort(sl), slot_abort_words(sl) * sizeof(uint32_t), hipMemcpyDefault,
                          c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_eigvals_inject_abort(pods_ctx* c, int slot) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (slot < 0 || slot >= (int)c->eslots.size() || !c->eslots[slot].active)
    return fail(PODS_ERR_ARG, "pods_eigvals_inject_abort: no such slot");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(hipMemsetAsync(slot_abort(c->eslots[slot]), 1, sizeof(uint32_t), c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_syev2_flags_async(pods_ctx* c, uint32_t* flags_dst) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!flags_dst) return fail(PODS_ERR_ARG, "flags_dst is null");
  if (!c->e2_flags.p) return fail(PODS_ERR_STATE, "no pods_syev2 ran");
  PODS_HIP(hipSetDevice(c->device));
  PODS_HIP(hipMemcpyAsync(flags_dst, c->e2_flags.as<uint32_t>() + 64, 2 * sizeof(uint32_t), hipMemcpyDefault,
                          c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_syev(pods_ctx* c, const double* C, int n, int nvec, double* lam_desc, double* vec) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!C || !lam_desc || n < 1 || nvec < 0 || nvec > std::min(n, 64) || (nvec > 0 && !vec))
    return fail(PODS_ERR_ARG, "pods_syev: bad arguments");
  int R = 0;
  PersistentLock lk(c);
  if (int e = run_sytrd(c, C, n, &R)) return e;
  double* det = c->e_det.as<double>();
  double* D = det;
  double* E = det + n;
  double* tau = det + 2 * (int64_t)n;
  double* bounds = det + 3 * (int64_t)n;
  // All n eigenvalues start from brackets given by Sturm counts at 64 Ki shared shifts
  // (k_sturm_grid, 0.16 ms): k_bisect 2.09 -> 1.41 ms against every eigenvalue from the
  // Gershgorin interval.
  // (Bisecting the nvec wanted eigenvalues first and the rest on a side stream was measured
  // slower: each eigenvalue's bisection is latency bound (13 sequential n-step Sturm
  // passes), so the top nvec alone cost as much as all n, and the side launch slowed the
  // back-transformation kernels it shared CUs with.)
  PODS_HIP(ensure(c->e_cnt, pods::tri_grid_bytes()));
  int* gcnt = c->e_cnt.as<int>();
  // the compact-WY blocks of the back-transformation (k_larft) need V and tau only: on a second
  // stream beside the bisection and the eigenvectors of T, joined before k_bt_fused
  const bool fork = nvec > 0 && n > 1;
  if (fork) {
    const int nblk = std::max((n - 1 + 63) / 64, 1);
    PODS_HIP(ensure(c->e_t, (size_t)nblk * 64 * 64 * sizeof(double)));
    if (!c->aux) PODS_HIP(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    if (!c->aux_fork) PODS_HIP(hipEventCreateWithFlags(&c->aux_fork, hipEventDisableTiming));
    if (!c->aux_join) PODS_HIP(hipEventCreateWithFlags(&c->aux_join, hipEventDisableTiming));
    PODS_HIP(hipEventRecord(c->aux_fork, c->stream));
    PODS_HIP(hipStreamWaitEvent(c->aux, c->aux_fork, 0));
    PODS_HIP(pods::launch_larft(c->e_v.as<double>(), n, tau, n, c->e_t.as<double>(), c->aux));
    PODS_HIP(hipEventRecord(c->aux_join, c->aux));
  }
  PODS_HIP(pods::launch_tri_eigvals(D, E, n, bounds, lam_desc, gcnt, c->stream));
  if (c->marker_tail_req && c->marker_tail) {  // pods_syev_marker_tail(ctx, 1): behind the eigenvalues
    PODS_HIP(hipEventRecord(c->marker_tail, c->stream));
    c->marker_tail_recorded = true;
  }
  c->marker_tail_req = false;
  if (nvec > 0) {
    const int nblk = std::max((n - 1 + 63) / 64, 1);
    PODS_HIP(ensure(c->e_inv, (size_t)nvec * n * sizeof(double)));
    PODS_HIP(ensure(c->e_t, (size_t)nblk * 64 * 64 * sizeof(double)));
    PODS_HIP(ensure(c->e_part, pods::bt_part_bytes(n, nvec)));
    PODS_HIP(ensure(c->e_w2, pods::bt_w2_bytes(nvec)));
    PODS_HIP(pods::launch_tri_eigvecs(D, E, n, lam_desc, bounds, nvec, c->e_inv.as<double>(), vec,
                                      c->stream));
    if (fork) PODS_HIP(hipStreamWaitEvent(c->stream, c->aux_join, 0));
    PODS_HIP(pods::launch_back_transform(c->e_v.as<double>(), n, tau, n, nvec, c->e_t.as<double>(),
                                         c->e_part.as<double>(), c->e_w2.as<double>(),
                                         c->e_flags.as<uint32_t>() + 1, vec,
                                         c->stream, /*skip_larft=*/fork));
  }
  return lk.release();
  PODS_CATCH
}

int pods_syev2(pods_ctx* c, const double* C, int n, int nvec, double* lam_desc, double* vec) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!C || !lam_desc || n < 3 || nvec < 0 || nvec > std::min(n, 64) || (nvec > 0 && !vec))
    return fail(PODS_ERR_ARG, "pods_syev2: bad arguments");
  if (n > pods::syev2_max_n())
    return fail(PODS_ERR_UNSUPPORTED, "pods_syev2: n > " + std::to_string(pods::syev2_max_n()));
  PODS_HIP(hipSetDevice(c->device));
  pods::SyevdPlan plan{};
  const size_t wsd = pods::sy2sb_work_doubles(n, nvec, &plan);
  PODS_HIP(ensure(c->e2_ws, wsd * sizeof(double)));
  const size_t fw = 128 + (size_t)n;
  if (c->e2_flag_words < fw) {
    PODS_HIP(ensure(c->e2_flags, fw * sizeof(uint32_t)));
    PODS_HIP(hipMemset(c->e2_flags.p, 0, fw * sizeof(uint32_t)));
    c->e2_flag_words = fw;
    c->e2_epoch = 0;
  }
  PODS_HIP(hipMemsetAsync(c->e2_flags.as<uint32_t>() + 64, 0, 64 * sizeof(uint32_t), c->stream));  // abort words
  PODS_HIP(ensure(c->e2_ipiv, (size_t)std::max(nvec, 1) * n * sizeof(int)));
  PODS_HIP(ensure(c->e_cnt, pods::tri_grid_bytes()));
  ++c->e2_epoch;
  PersistentLock lk(c);
  PODS_HIP(pods::launch_syevd2(C, n, nvec, c->e2_ws.as<double>(), plan, c->e2_flags.as<uint32_t>(), c->e2_epoch,
                               c->e2_ipiv.as<int>(), c->e_cnt.as<int>(), lam_desc, vec, c->stream));
  return lk.release();
  PODS_CATCH
}

int pods_syev2_inspect(pods_ctx* c, int n, int nvec, int what, double* out_host, int64_t count) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->e2_ws.p || !out_host || count < 0) return fail(PODS_ERR_ARG, "pods_syev2_inspect: bad arguments");
  pods::SyevdPlan plan{};
  pods::sy2sb_work_doubles(n, nvec, &plan);
  const int64_t offs[10] = {plan.off_band0, plan.off_band, plan.off_de, plan.off_aw, plan.off_vx,
                            plan.off_t, plan.off_tau, plan.off_y, plan.off_x, plan.off_w};
  if (what < 0 || what > 9) return fail(PODS_ERR_ARG, "pods_syev2_inspect: what");
  if ((size_t)(offs[what] + count) * sizeof(double) > c->e2_ws.bytes) return fail(PODS_ERR_ARG, "count");
  PODS_HIP(hipMemcpyAsync(out_host, c->e2_ws.as<double>() + offs[what], (size_t)count * sizeof(double),
                          hipMemcpyDeviceToHost, c->stream));
  PODS_HIP(hipStreamSynchronize(c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_syev2_status(pods_ctx* c) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->e2_flags.p) return PODS_OK;
  uint32_t abort_word[2] = {0, 0};  // [0]: panel QR hand-offs, [1]: bulge chasing
  PODS_HIP(hipMemcpyAsync(abort_word, c->e2_flags.as<uint32_t>() + 64, sizeof(abort_word), hipMemcpyDeviceToHost,
                          c->stream));
  PODS_HIP(hipStreamSynchronize(c->stream));
  if (abort_word[0] || abort_word[1]) return fail(PODS_ERR_INTERNAL, "pods_syev2: hand-off wait timed out (aborted)");
  return PODS_OK;
  PODS_CATCH
}

int pods_sytrd(pods_ctx* c, const double* C, int n, double* d_host, double* e_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!C || !d_host || (n > 1 && !e_host) || n < 1) return fail(PODS_ERR_ARG, "pods_sytrd: bad arguments");
  int R = 0;
  PersistentLock lk(c);
  if (int e = run_sytrd(c, C, n, &R)) return e;
  const double* det = c->e_det.as<double>();
  PODS_HIP(hipMemcpyAsync(d_host, det, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (n > 1)
    PODS_HIP(hipMemcpyAsync(e_host, det + n, (size_t)(n - 1) * sizeof(double), hipMemcpyDeviceToHost,
                            c->stream));
  uint32_t abort_word = 0;
  PODS_HIP(hipMemcpyAsync(&abort_word, c->e_flags.as<uint32_t>() + c->e_G, sizeof(uint32_t),
                          hipMemcpyDeviceToHost, c->stream));
  PODS_HIP(hipStreamSynchronize(c->stream));
  if (abort_word) return fail(PODS_ERR_INTERNAL, "pods_sytrd: hand-off wait timed out (aborted)");
  return PODS_OK;
  PODS_CATCH
}

int pods_sytrd_trace(pods_ctx* c, const double* C, int n, int wg, int64_t* trace_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!C || !trace_host || n < 2) return fail(PODS_ERR_ARG, "pods_sytrd_trace: bad arguments");
  DevBuf tb;
  const size_t tbytes = (size_t)(wg < 0 ? 256 : 1) * n * 8 * sizeof(int64_t);  // wg < 0: every workgroup
  PODS_HIP(ensure(tb, tbytes));
  PODS_HIP(hipMemsetAsync(tb.p, 0, tbytes, c->stream));
  int R = 0;
  PersistentLock lk(c);
  int e = run_sytrd(c, C, n, &R, tb.as<int64_t>(), wg);
  if (e == PODS_OK) {
    hipError_t he = hipMemcpyAsync(trace_host, tb.p, tbytes, hipMemcpyDeviceToHost,
                                   c->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(c->stream);
    if (he != hipSuccess) e = fail(PODS_ERR_HIP, std::string("pods_sytrd_trace: ") + hipGetErrorString(he));
  }
  (void)hipStreamSynchronize(c->stream);
  release(tb);
  return e;
  PODS_CATCH
}

int pods_syev_marker(pods_ctx* c, int after_range) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->marker) PODS_HIP(hipEventCreateWithFlags(&c->marker, hipEventDisableTiming));
  c->marker_after = after_range;
  return PODS_OK;
  PODS_CATCH
}

int pods_syev_marker_tail(pods_ctx* c, int where) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (where != 0 && where != 1) return fail(PODS_ERR_ARG, "pods_syev_marker_tail: where must be 0 or 1");
  if (!c->marker_tail) PODS_HIP(hipEventCreateWithFlags(&c->marker_tail, hipEventDisableTiming));
  c->marker_tail_req = true;
  c->marker_tail_where = where;
  return PODS_OK;
  PODS_CATCH
}

int pods_stream_wait_marker_tail(pods_ctx* c, void* stream) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->marker_tail_recorded) return fail(PODS_ERR_STATE, "the last pods_syev recorded no tail marker");
  PODS_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->marker_tail, 0));
  return PODS_OK;
  PODS_CATCH
}

int pods_stream_wait_marker(pods_ctx* c, void* stream) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->marker_recorded) return fail(PODS_ERR_STATE, "the last pods_syev recorded no marker");
  PODS_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), c->marker, 0));
  return PODS_OK;
  PODS_CATCH
}

int pods_syev_flags_async(pods_ctx* c, uint32_t* flags_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!flags_host) return fail(PODS_ERR_ARG, "flags_host is null");
  if (!c->e_flags.p) return fail(PODS_ERR_STATE, "no pods_syev ran");
  PODS_HIP(hipMemcpyAsync(flags_host, c->e_flags.as<uint32_t>(), 2 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                          c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_syev_status(pods_ctx* c) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c->e_flags.p) return PODS_OK;
  uint32_t abort_word[2] = {0, 0};  // [0]: tridiagonalisation, [1]: back-transformation
  PODS_HIP(hipMemcpyAsync(abort_word, c->e_flags.as<uint32_t>(), sizeof(abort_word),
                          hipMemcpyDeviceToHost, c->stream));
  PODS_HIP(hipStreamSynchronize(c->stream));
  if (abort_word[0] || abort_word[1])
    return fail(PODS_ERR_INTERNAL, "pods_syev: hand-off wait timed out (aborted)");
  return PODS_OK;
  PODS_CATCH
}

int pods_fourier_twiddles(pods_ctx* c, int ns, const double* t_host, double period, const double* w_host) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (ns <= 0 || !t_host || !w_host) return fail(PODS_ERR_ARG, "pods_fourier_twiddles: bad arguments");
  PODS_HIP(hipSetDevice(c->device));
  const size_t bytes = (size_t)pods::dft_table_rows(ns) * ns * 2 * sizeof(double);
  PODS_HIP(hipDeviceSynchronize());  // a DFT in flight (any stream) may read the old table
  PODS_HIP(ensure(c->dft_w, bytes));
  PODS_HIP(hipMemcpy(c->dft_w.p, w_host, bytes, hipMemcpyHostToDevice));
  c->dft_w_ns = ns;
  c->dft_w_period = period;
  c->dft_w_t.assign(t_host, t_host + ns);
  return PODS_OK;
  PODS_CATCH
}

int pods_fourier(pods_ctx* c, const double* T, int ldT, int nm, int ns, const double* t_host,
                 double period, float* c_dev) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!T || !t_host || !c_dev || nm <= 0 || ns <= 0 || ldT < nm) return fail(PODS_ERR_ARG, "bad arguments");
  if (c->dft_w_ns != ns || c->dft_w_period != period ||
      std::memcmp(c->dft_w_t.data(), t_host, (size_t)ns * sizeof(double)) != 0)
    return fail(PODS_ERR_STATE, "pods_fourier: no twiddle table for this time axis (pods_fourier_twiddles)");
  PODS_HIP(hipSetDevice(c->device));
  // The summation program (depends on ns) is uploaded only when ns changes (blocking copy,
  // once per configuration), so the DFT itself is enqueued asynchronously on the bound stream
  // and can overlap the caller's next work.  Buffer prog_dft: the program, then its leaves.
  if (c->dft_ns != ns) {
    std::vector<int> prog = cpairwise_program(ns);
    std::vector<int> leaves;
    for (size_t i = 0; i < prog.size(); i += 2)
      if (prog[i] >= 0) {
        leaves.push_back(prog[i]);
        leaves.push_back(prog[i + 1]);
      }
    std::vector<int> buf(prog);
    buf.insert(buf.end(), leaves.begin(), leaves.end());
    PODS_HIP(hipDeviceSynchronize());
    PODS_HIP(ensure(c->prog_dft, buf.size() * sizeof(int)));
    PODS_HIP(hipMemcpy(c->prog_dft.p, buf.data(), buf.size() * sizeof(int), hipMemcpyHostToDevice));
    c->dft_nprog = (int)prog.size() / 2;
    c->dft_nleaf = (int)leaves.size() / 2;
    c->dft_ns = ns;
  }
  const int* prog = c->prog_dft.as<int>();
  PODS_HIP(pods::launch_dft_tab(T, ldT, nm, ns, c->dft_w.as<double2>(), prog, c->dft_nprog,
                                prog + 2 * c->dft_nprog, c->dft_nleaf, 1.0 / (double)ns,
                                reinterpret_cast<float2*>(c_dev), c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_fourier_rank(pods_ctx* c, const float* c_dev, int nm, int ns, double et, int32_t* c_ind_dev,
                      int64_t* c_count_dev) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!c_dev || !c_ind_dev || !c_count_dev || nm <= 0 || ns <= 0) return fail(PODS_ERR_ARG, "bad arguments");
  if (ns > pods::rank_max_ns())
    return fail(PODS_ERR_UNSUPPORTED, "pods_fourier_rank: ns > " + std::to_string(pods::rank_max_ns()));
  PODS_HIP(hipSetDevice(c->device));
  if (c->rank_ns != ns) {  // uploaded once per ns (blocking); the ranking itself is async
    std::vector<int> prog = pairwise_program(ns);
    PODS_HIP(hipDeviceSynchronize());
    PODS_HIP(ensure(c->prog_rank, prog.size() * sizeof(int)));
    PODS_HIP(hipMemcpy(c->prog_rank.p, prog.data(), prog.size() * sizeof(int), hipMemcpyHostToDevice));
    c->rank_nprog = (int)prog.size() / 2;
    c->rank_ns = ns;
  }
  PODS_HIP(pods::launch_rank(c_dev, ns, nm, et, c->prog_rank.as<int>(), c->rank_nprog, c_ind_dev,
                             c_count_dev, c->stream));
  return PODS_OK;
  PODS_CATCH
}

int pods_filter_block(pods_ctx* c, const double* x, int nfx, int nfy, int nfz, int jma, int kma,
                      const double* bx, const double* by, const double* bz, double* y) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!x || !y || !bx || !by || !bz || jma <= 0 || kma <= 0 || nfx < 0 || nfy < 0 || nfz < 0)
    return fail(PODS_ERR_ARG, "bad arguments");
  const int NX = 2 * nfx + 1, NY = 2 * nfy + 1, NZ = 2 * nfz + 1;
  if (NX > 49 || NY > 25) return fail(PODS_ERR_UNSUPPORTED, "filter too wide");
  const int Kp = kma + 2 * nfz;
  if (kma > pods::filter_yz_max_K(Kp)) return fail(PODS_ERR_UNSUPPORTED, "kma too large");
  PODS_HIP(hipSetDevice(c->device));
  const int64_t S = (int64_t)(jma + 2 * nfy) * Kp;
  DevBuf dx, dt1, dy, dtap;
  auto cleanup = [&] { release(dx); release(dt1); release(dy); release(dtap); };
  hipError_t e1 = ensure(dx, (size_t)NX * S * 8), e2 = ensure(dt1, (size_t)S * 8),
             e3 = ensure(dy, (size_t)jma * kma * 8), e4 = ensure(dtap, (size_t)(NX + NY + NZ) * 8);
  if (e1 || e2 || e3 || e4) {
    cleanup();
    return fail(PODS_ERR_NOMEM, "device allocation failed");
  }
  std::vector<double> taps(NX + NY + NZ);
  std::copy(bx, bx + NX, taps.begin());
  std::copy(by, by + NY, taps.begin() + NX);
  std::copy(bz, bz + NZ, taps.begin() + NX + NY);
  hipError_t e = hipMemcpy(dx.p, x, (size_t)NX * S * 8, hipMemcpyHostToDevice);
  if (!e) e = hipMemcpy(dtap.p, taps.data(), taps.size() * 8, hipMemcpyHostToDevice);
  const double* tp = dtap.as<double>();
  if (!e) e = pods::launch_filter_x(NX, dx.as<double>(), tp, 1, S, 1, 1, dt1.as<double>(), c->stream);
  if (!e)
    e = pods::launch_filter_yz(NY, dt1.as<double>(), tp + NX, tp + NX + NY, NZ, 1, jma, kma, Kp, S, 1,
                               nullptr, 0, PODS_LUND_NONE, nullptr, 0, dy.as<double>(), c->stream);
  if (!e) e = hipMemcpyAsync(y, dy.p, (size_t)jma * kma * 8, hipMemcpyDeviceToHost, c->stream);
  if (!e) e = hipStreamSynchronize(c->stream);
  cleanup();
  if (e) return fail(PODS_ERR_HIP, std::string("filter_block: ") + hipGetErrorString(e));
  return PODS_OK;
  PODS_CATCH
}

int pods_rng_uniform(pods_ctx* c, uint32_t seed, int64_t n, double low, double range, double* out) {
  PODS_TRY
  if (int e = check_ctx(c)) return e;
  if (!out || n <= 0 || n > 0x7fffffffLL) return fail(PODS_ERR_ARG, "bad n/out");
  PODS_HIP(hipSetDevice(c->device));
  RngLayout L = make_layout(n);
  RngBuffers rb;
  int rc = upload_rng(c, L, seed, rb);
  if (!rc) rc = run_jumps(c, L, rb);
  if (!rc) {
    hipError_t e = pods::launch_mt_generate(rb.states.as<uint32_t>(), L.G, L.Bs, n, n, (int)n, 0, 1, n,
                                            low, range, out, c->stream);
    if (!e) e = hipStreamSynchronize(c->stream);
    if (e) rc = fail(PODS_ERR_HIP, std::string("rng: ") + hipGetErrorString(e));
  }
  rb.free_all();
  return rc;
  PODS_CATCH
}

int pods_host_mt_jump_check(uint32_t seed, int64_t nblocks) {
  PODS_TRY
  using namespace pods::mt;
  if (nblocks < 1) return fail(PODS_ERR_ARG, "nblocks >= 1");
  std::vector<uint32_t> s1(N), ref(N), got(N);
  seed_state(seed, s1.data());
  twist(s1.data());  // mt^(1)
  ref = s1;
  for (int64_t b = 1; b < nblocks; ++b) twist(ref.data());  // mt^(nblocks)
  Poly g = powmod_t((uint64_t)N * (uint64_t)(nblocks - 1));
  apply_poly(g, s1.data(), got.data());
  if (got != ref) return fail(PODS_ERR_INTERNAL, "jump-ahead mismatch");
  return PODS_OK;
  PODS_CATCH
}

int pods_host_mt_charpoly_degree(void) { return pods::mt::charpoly_degree(); }

int pods_host_persistent_grid_fits(int blocks_per_cu, int cus, int64_t grid) {
  if (blocks_per_cu < 0 || cus < 0 || grid < 0) return fail(PODS_ERR_ARG, "negative argument");
  if (!pods::persistent_grid_fits(blocks_per_cu, cus, grid))
    return fail(PODS_ERR_UNSUPPORTED, "grid of " + std::to_string(grid) + " workgroups > " +
                                          std::to_string(blocks_per_cu) + " per CU x " + std::to_string(cus) +
                                          " CUs");
  return PODS_OK;
}

}  // extern "C"

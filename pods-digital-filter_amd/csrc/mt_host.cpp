// Host-side MT19937 jump-ahead machinery.  See mt_host.h for the maths.
#include "mt_host.h"

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>

#include <immintrin.h>

namespace pods {
namespace mt {

void seed_state(uint32_t seed, uint32_t* st) {
  // numpy random/src/mt19937/mt19937.c mt19937_seed (== init_genrand)
  for (int pos = 0; pos < N; ++pos) {
    st[pos] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(pos + 1);
  }
}

static inline uint32_t mix(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t y = (a & UPPER) | (b & LOWER);
  return c ^ (y >> 1) ^ ((y & 1u) ? MATRIX_A : 0u);
}

void twist(uint32_t* st) {
  int i = 0;
  for (; i < N - M; ++i) st[i] = mix(st[i], st[i + 1], st[i + M]);
  for (; i < N - 1; ++i) st[i] = mix(st[i], st[i + 1], st[i + (M - N)]);
  st[N - 1] = mix(st[N - 1], st[0], st[M - 1]);
}

uint32_t temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// ---------------------------------------------------------------------------------------
// carry-less multiply
// ---------------------------------------------------------------------------------------
__attribute__((target("pclmul,sse2"))) static void clmul_poly_hw(const uint64_t* a, const uint64_t* b,
                                                                 uint64_t* out, int n) {
  for (int i = 0; i < 2 * n; ++i) out[i] = 0;
  for (int i = 0; i < n; ++i) {
    if (!a[i]) continue;
    __m128i va = _mm_set_epi64x(0, (long long)a[i]);
    for (int j = 0; j < n; ++j) {
      if (!b[j]) continue;
      __m128i vb = _mm_set_epi64x(0, (long long)b[j]);
      __m128i p = _mm_clmulepi64_si128(va, vb, 0x00);
      out[i + j] ^= (uint64_t)_mm_cvtsi128_si64(p);
      out[i + j + 1] ^= (uint64_t)_mm_cvtsi128_si64(_mm_unpackhi_epi64(p, p));
    }
  }
}

static void clmul_poly_sw(const uint64_t* a, const uint64_t* b, uint64_t* out, int n) {
  for (int i = 0; i < 2 * n; ++i) out[i] = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t x = a[i];
    while (x) {
      int bit = __builtin_ctzll(x);
      x &= x - 1;
      // out ^= b << (64*i + bit)
      for (int j = 0; j < n; ++j) {
        out[i + j] ^= b[j] << bit;
        if (bit) out[i + j + 1] ^= b[j] >> (64 - bit);
      }
    }
  }
}

static void clmul_poly(const uint64_t* a, const uint64_t* b, uint64_t* out, int n) {
  static const bool hw = __builtin_cpu_supports("pclmul");
  if (hw)
    clmul_poly_hw(a, b, out, n);
  else
    clmul_poly_sw(a, b, out, n);
}

// ---------------------------------------------------------------------------------------
// characteristic polynomial via Berlekamp-Massey over GF(2)
// ---------------------------------------------------------------------------------------
static inline bool getbit(const uint64_t* v, int64_t i) { return (v[i >> 6] >> (i & 63)) & 1u; }

static Poly compute_charpoly(int* out_deg) {
  const int NS = 2 * DEG + 128;
  // bit 0 of consecutive raw state words x_624, x_625, ... (all in F's image)
  std::vector<uint32_t> st(N);
  seed_state(5489u, st.data());
  std::vector<uint8_t> s(NS);
  int n = 0;
  while (n < NS) {
    twist(st.data());
    for (int i = 0; i < N && n < NS; ++i) s[n++] = st[i] & 1u;
  }
  // reversed sequence bitset: R bit j = s[NS-1-j]
  const int RW = NS / 64 + 3;
  std::vector<uint64_t> R(RW, 0);
  for (int j = 0; j < NS; ++j)
    if (s[NS - 1 - j]) R[j >> 6] |= 1ull << (j & 63);
  const int CW = (DEG + 64) / 64 + 3;
  std::vector<uint64_t> C(CW + 2, 0), B(CW + 2, 0), T(CW + 2, 0);
  C[0] = 1;
  B[0] = 1;
  int L = 0, m = 1;
  for (int k = 0; k < NS; ++k) {
    // d = sum_{i=0..L} C_i s_{k-i} ; s_{k-i} = R bit (NS-1-k+i)
    const int64_t off = (int64_t)NS - 1 - k;
    const int64_t wo = off >> 6;
    const int sh = (int)(off & 63);
    uint64_t acc = 0;
    const int nw = L / 64 + 1;
    for (int w = 0; w < nw; ++w) {
      uint64_t lo = (wo + w < RW) ? R[wo + w] : 0;
      uint64_t hi = (wo + w + 1 < RW) ? R[wo + w + 1] : 0;
      uint64_t seg = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
      uint64_t cw = C[w];
      if (w == nw - 1) {
        int rem = (L % 64) + 1;  // bits 0..L of C
        if (rem < 64) cw &= (1ull << rem) - 1;
      }
      acc ^= cw & seg;
    }
    int d = __builtin_popcountll(acc) & 1;
    if (!d) {
      ++m;
      continue;
    }
    // C ^= B << m
    auto xor_shifted = [&](std::vector<uint64_t>& dst, const std::vector<uint64_t>& src, int shift) {
      const int q = shift >> 6, r = shift & 63;
      for (int w = CW - 1; w >= 0; --w) {
        uint64_t v = 0;
        if (w - q >= 0) v = src[w - q] << r;
        if (r && w - q - 1 >= 0) v |= src[w - q - 1] >> (64 - r);
        dst[w] ^= v;
      }
    };
    if (2 * L <= k) {
      T = C;
      xor_shifted(C, B, m);
      L = k + 1 - L;
      B = T;
      m = 1;
    } else {
      xor_shifted(C, B, m);
      ++m;
    }
  }
  *out_deg = L;
  // phi(t) = t^L C(1/t): phi_j = C_{L-j}
  Poly phi(PW + 1, 0);
  for (int j = 0; j <= L; ++j)
    if (getbit(C.data(), L - j)) phi[j >> 6] |= 1ull << (j & 63);
  return phi;
}

struct CharPoly {
  Poly phi;
  int deg = 0;
  std::vector<Poly> shifted;  // phi << s, s = 0..63, PW+1 words each
};

static const CharPoly& cp() {
  static CharPoly* c = [] {
    auto* p = new CharPoly();
    p->phi = compute_charpoly(&p->deg);
    p->shifted.resize(64);
    for (int s = 0; s < 64; ++s) {
      Poly v(PW + 2, 0);
      for (int w = 0; w <= PW; ++w) {
        v[w] ^= p->phi[w] << s;
        if (s) v[w + 1] ^= p->phi[w] >> (64 - s);
      }
      p->shifted[s] = std::move(v);
    }
    return p;
  }();
  return *c;
}

const Poly& charpoly() { return cp().phi; }
int charpoly_degree() { return cp().deg; }

static void reduce_inplace(std::vector<uint64_t>& prod) {
  const CharPoly& c = cp();
  const int top = (int)prod.size() * 64 - 1;
  for (int p = top; p >= DEG; --p) {
    if (!getbit(prod.data(), p)) continue;
    const int shv = p - DEG;
    const int q = shv >> 6, s = shv & 63;
    const Poly& ph = c.shifted[s];
    const int lim = std::min<int>((int)ph.size(), (int)prod.size() - q);
    for (int w = 0; w < lim; ++w) prod[q + w] ^= ph[w];
  }
}

Poly mulmod(const Poly& a, const Poly& b) {
  std::vector<uint64_t> prod(2 * PW, 0);
  clmul_poly(a.data(), b.data(), prod.data(), PW);
  reduce_inplace(prod);
  prod.resize(PW);
  return prod;
}

Poly powmod_t(uint64_t e) {
  Poly r(PW, 0);
  r[0] = 1;
  if (e == 0) return r;
  int hb = 63 - __builtin_clzll(e);
  for (int b = hb; b >= 0; --b) {
    r = mulmod(r, r);
    if ((e >> b) & 1u) {
      // r *= t
      std::vector<uint64_t> v(PW + 1, 0);
      for (int w = 0; w < PW; ++w) {
        v[w] |= r[w] << 1;
        v[w + 1] |= r[w] >> 63;
      }
      reduce_inplace(v);
      v.resize(PW);
      r = v;
    }
  }
  return r;
}

void apply_poly(const Poly& g, const uint32_t* src, uint32_t* dst) {
  std::vector<uint32_t> x(2 * N), acc(N, 0);
  std::memcpy(x.data(), src, N * sizeof(uint32_t));
  std::memcpy(x.data() + N, src, N * sizeof(uint32_t));
  twist(x.data() + N);
  const int Q = (DEG + N - 1) / N;  // 32 blocks of 624 coefficients
  for (int q = Q - 1; q >= 0; --q) {
    if (q != Q - 1) twist(acc.data());
    for (int r = 0; r < N; ++r) {
      const int64_t i = (int64_t)q * N + r;
      if (i >= PW * 64 || !getbit(g.data(), i)) continue;
      for (int w = 0; w < N; ++w) acc[w] ^= x[r + w];
    }
  }
  std::memcpy(dst, acc.data(), N * sizeof(uint32_t));
}

static void poly_to_words32(const Poly& p, uint32_t* out) {
  for (int w = 0; w < PW; ++w) {
    out[2 * w] = (uint32_t)(p[w] & 0xffffffffu);
    out[2 * w + 1] = (uint32_t)(p[w] >> 32);
  }
}

const JumpTables& jump_tables(int64_t Bs, int G2, int G1_needed) {
  static std::mutex mu;
  static std::map<std::pair<int64_t, int>, std::unique_ptr<JumpTables>> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto& slot = cache[{Bs, G2}];
  if (!slot) {
    slot.reset(new JumpTables());
    slot->Bs = Bs;
    slot->G2 = G2;
    slot->level2.assign((size_t)(G2 + 1) * N, 0);
    const Poly step = powmod_t((uint64_t)N * (uint64_t)Bs);
    // chunks of the sequence p_g = t^(624(g Bs - 1)) = p_{g-1} * step on host threads
    const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int per = (G2 + nth - 1) / nth;
    std::vector<std::thread> pool;
    JumpTables* jt = slot.get();
    for (int k = 0; k < nth; ++k) {
      const int a = 1 + k * per, b = std::min(G2, k * per + per);
      if (a > b) break;
      pool.emplace_back([jt, a, b, Bs, &step] {
        Poly p = powmod_t((uint64_t)N * (uint64_t)(a * Bs - 1));
        for (int g2 = a; g2 <= b; ++g2) {
          poly_to_words32(p, &jt->level2[(size_t)g2 * N]);
          if (g2 < b) p = mulmod(p, step);
        }
      });
    }
    for (auto& th : pool) th.join();
    slot->G1 = 1;
    slot->level1.assign(N, 0);
    slot->level1[0] = 1;  // identity polynomial (unused)
  }
  JumpTables& jt = *slot;
  if (jt.G1 < G1_needed) {
    const Poly step = powmod_t((uint64_t)N * (uint64_t)Bs * (uint64_t)G2);
    Poly cur(PW, 0);
    // reconstruct the last polynomial from the words32 table
    const uint32_t* last = &jt.level1[(size_t)(jt.G1 - 1) * N];
    for (int w = 0; w < PW; ++w) cur[w] = (uint64_t)last[2 * w] | ((uint64_t)last[2 * w + 1] << 32);
    jt.level1.resize((size_t)G1_needed * N);
    for (int g1 = jt.G1; g1 < G1_needed; ++g1) {
      cur = (g1 == 1) ? step : mulmod(cur, step);
      poly_to_words32(cur, &jt.level1[(size_t)g1 * N]);
    }
    jt.G1 = G1_needed;
  }
  return jt;
}

}  // namespace mt
}  // namespace pods

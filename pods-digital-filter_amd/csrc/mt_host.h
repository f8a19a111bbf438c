// Host-side MT19937 machinery: numpy-legacy seeding, twisting, the characteristic
// polynomial (Berlekamp-Massey) and GF(2)[t]/phi(t) jump polynomials.
//
// The reference draws every random field from numpy's legacy global RandomState
// (digitalfilters.py:1361-1366, :1460-1467).  The device regenerates exactly that
// stream in parallel substreams; a substream starting at output block q needs the
// state mt^(q) (the 624-word array after q twists).  With F the one-word transition
// and phi its characteristic polynomial, mt^(q) = (t^(624(q-1)) mod phi)(F) mt^(1) for
// q >= 1 (mt^(1) lies in F's image, where phi(F) = 0).  The polynomials are seed- and
// config-independent, so they are computed here once per substream length and cached.
#pragma once
#include <cstdint>
#include <vector>

namespace pods {
namespace mt {

constexpr int N = 624;
constexpr int M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu;
constexpr uint32_t UPPER = 0x80000000u;
constexpr uint32_t LOWER = 0x7fffffffu;
constexpr int DEG = 19937;         // degree of phi
constexpr int PW = 312;            // 64-bit words holding a polynomial of degree < DEG
constexpr int PW32 = 624;          // the same as 32-bit words (device layout)

void seed_state(uint32_t seed, uint32_t* st);   // numpy mt19937_seed == init_genrand
void twist(uint32_t* st);                        // one full twist (mt19937_gen)
uint32_t temper(uint32_t y);

using Poly = std::vector<uint64_t>;              // bit i = coefficient of t^i

const Poly& charpoly();                          // phi, degree DEG (computed once)
int charpoly_degree();
Poly mulmod(const Poly& a, const Poly& b);
Poly powmod_t(uint64_t e);                       // t^e mod phi
// Horner evaluation of g(F) applied to a state in F's image (host reference of the
// device jump kernel).
void apply_poly(const Poly& g, const uint32_t* src, uint32_t* dst);

// Jump tables for a substream layout: substream g (g >= 1) starts at output block g*Bs.
// With g = g1*G2 + g2, g2 in [1, G2]:
//   base[g1]  = (t^(624*g1*G2*Bs) mod phi)(F) mt^(1)          -> level1[g1]
//   start[g]  = (t^(624*(g2*Bs - 1)) mod phi)(F) base[g1]      -> level2[g2]
struct JumpTables {
  int64_t Bs = 0;            // blocks (of 624 words) per substream
  int G2 = 0;                // substreams per level-1 base
  int G1 = 0;                // level-1 bases available
  std::vector<uint32_t> level1;   // G1 x 624 words (level1[0] = identity, unused)
  std::vector<uint32_t> level2;   // (G2+1) x 624 words (index 0 unused)
};
// Thread-safe, cached by (Bs, G2); grows G1 on demand.
const JumpTables& jump_tables(int64_t Bs, int G2, int G1_needed);

}  // namespace mt
}  // namespace pods

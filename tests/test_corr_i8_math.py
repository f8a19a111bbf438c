"""CPU check of the arithmetic the int8 correlation (podsgen_corr_i8.hip) relies on, restated in
numpy / Python integers (test infrastructure; the kernels themselves are pinned on the GPU by
tests/test_gpu_corr_i8.py):

  * the 16 moduli are pairwise coprime, their product M lies in [2^124, 2^125), and the
    precision b the plan picks keeps 2 K 2^2b < M for every BASELINE K (C3, C4, C5 slabs);
  * k_residues' f32 arithmetic (k_residues<1>: four signed 14-bit limbs split in fp64 and balanced
    coefficients, see residues_signed_limbs_like_kernel; k_residues<0>): five 11-bit limbs of z = a' + 2^52, s = sum z_k (2^11k mod m)
    + (-2^52 mod m) < 2^24, q = fl32(s * fl32(1/m) + 1.5 * 2^23) - 1.5 * 2^23 = rint(s / m)
    exactly, and the low byte of fl32(s - q m + 1.5 * 2^23) is the balanced residue;
  * k_crt: Garner's mixed-radix digits and Horner give back any integer |X| < M / 2 from its
    16 residues.
"""
import math

import numpy as np

MODULI = [255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 211, 199, 197, 193, 191, 181]
LOG2M = 124.689
MAG = 12582912.0  # 1.5 * 2^23


def bbits(K):
    return min(52, math.floor((LOG2M - 1.0 - math.log2(K)) / 2.0))


def test_moduli_and_precision_bounds():
    for a in range(16):
        for b in range(a + 1, 16):
            assert math.gcd(MODULI[a], MODULI[b]) == 1
    M = math.prod(MODULI)
    assert 2 ** 124 <= M < 2 ** 125 and math.log2(M) >= LOG2M
    for K in (196608, 786432, 3 * 1024 * 1024 // 8 * 8, 3 * 1024 * 1024):   # C3, C4, C5 slab, C5
        b = bbits(K)
        assert 2 * K * 2 ** (2 * b) < M and b >= 51
    assert bbits(196608) == 52 and bbits(786432) == 52 and bbits(3 * 1024 * 1024) == 51


def f32(x):
    return np.float32(x)


def residues_like_kernel(a):
    """a: int64 array, |a| <= 2^52 -> (16, len) int8 balanced residues, computed the kernel's way."""
    z = a + (1 << 52)
    lo = (z & 0xFFFFFFFF).astype(np.uint64)
    hi = (z >> 32).astype(np.uint64)
    limbs = [lo & 0x7FF, (lo >> 11) & 0x7FF, ((lo >> 22) | (hi << 10)) & 0x7FF, (hi >> 1) & 0x7FF, hi >> 12]
    F = [l.astype(np.float32) for l in limbs]
    out = np.empty((16, a.size), dtype=np.int8)
    for li, m in enumerate(MODULI):
        c = [pow(2, 11 * k, m) for k in range(5)]
        o = (m - pow(2, 52, m)) % m
        s = F[0]
        for k in range(1, 5):
            # exact in f32 (every partial sum < 2^24), so a separate multiply and add equal the fma
            s = (s + F[k] * f32(c[k])).astype(np.float32)
        s = (s + f32(o)).astype(np.float32)
        assert float(np.max(s)) < 2 ** 24
        inv = f32(1.0 / m)
        # fma(s, inv, MAG): the exact s * inv + MAG rounded once (float64 holds s * inv exactly)
        q = (s.astype(np.float64) * np.float64(inv) + MAG).astype(np.float32) - f32(MAG)
        r = (s.astype(np.float64) - q.astype(np.float64) * m).astype(np.float32)   # exact integer
        rb = (r + f32(MAG)).astype(np.float32)
        out[li] = (rb.view(np.uint32) & 0xFF).astype(np.uint8).view(np.int8)
    return out


def residues_signed_limbs_like_kernel(a):
    """k_residues<1>: a' (|a'| <= 2^52) as four signed 14-bit limbs split in fp64, balanced
    c_k = 2^14k mod m, s = d0 + c1 d1 + c2 d2 + c3 d3 in f32, the same quotient / byte steps."""
    ap = a.astype(np.float64)
    hh = np.rint(ap * 2.0 ** -28)
    lo = ap - hh * 2.0 ** 28            # exact (fma in the kernel; here every term fits in 53 bits)
    d3 = np.rint(hh * 2.0 ** -14)
    d1 = np.rint(lo * 2.0 ** -14)
    d = [lo - d1 * 2.0 ** 14, d1, hh - d3 * 2.0 ** 14, d3]
    assert max(float(np.max(np.abs(x))) for x in d[:3]) <= 2 ** 13 and float(np.max(np.abs(d3))) <= 2 ** 10
    F = [x.astype(np.float32) for x in d]
    out = np.empty((16, a.size), dtype=np.int8)
    for li, m in enumerate(MODULI):
        c = [pow(2, 14 * k, m) for k in range(4)]
        c = [x - m if x > m // 2 else x for x in c]
        s = F[0]
        for k in range(1, 4):
            s = (s.astype(np.float64) + F[k].astype(np.float64) * c[k]).astype(np.float32)  # exact
        assert float(np.max(np.abs(s))) < 2 ** 21.1
        inv = f32(1.0 / m)
        q = (s.astype(np.float64) * np.float64(inv) + MAG).astype(np.float32) - f32(MAG)
        assert np.array_equal(q.astype(np.float64), np.rint(s.astype(np.float64) / m))
        r = (s.astype(np.float64) - q.astype(np.float64) * m).astype(np.float32)
        rb = (r + f32(MAG)).astype(np.float32)
        out[li] = (rb.view(np.uint32) & 0xFF).astype(np.uint8).view(np.int8)
    return out


def test_residue_signed_limbs_exact():
    rng = np.random.default_rng(9)
    a = np.concatenate([rng.integers(-(1 << 52), (1 << 52) + 1, 200000, dtype=np.int64),
                        np.array([0, 1, -1, 1 << 52, -(1 << 52), (1 << 27) + 8191, -(1 << 41) - 1],
                                 dtype=np.int64)])
    got = residues_signed_limbs_like_kernel(a)
    for li, m in enumerate(MODULI):
        want = np.array([int(x) % m for x in a], dtype=np.int64)
        want = np.where(want > m // 2, want - m, want)
        assert np.array_equal(got[li].astype(np.int64), want), m


def test_residue_arithmetic_exact():
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.integers(-(1 << 52), (1 << 52) + 1, 200000, dtype=np.int64),
                        np.array([0, 1, -1, 1 << 52, -(1 << 52), 12345, -987654321], dtype=np.int64)])
    got = residues_like_kernel(a)
    for li, m in enumerate(MODULI):
        want = np.array([int(x) % m for x in a], dtype=np.int64)
        want = np.where(want > m // 2, want - m, want)
        assert np.array_equal(got[li].astype(np.int64), want), m


def crt_like_kernel(c):
    """c: 16 residues -> the integer X in [-(M-1)/2, (M-1)/2], k_crt's way: Garner's digits kept
    balanced and computed in f32 (x = (t - v_k) * inv, q = fl32(x * fl32(1/m) + 1.5 * 2^23) - 1.5 * 2^23,
    t = x - q m; every operand an integer below 2^17, so each step is exact), then a signed Horner."""
    v = []
    for l, ml in enumerate(MODULI):
        rm = f32(1.0 / ml)

        def bal(x):
            q = float(f32(float(x) * float(rm) + MAG)) - MAG   # fma: exact product, one rounding
            assert q == round(x / ml)
            return int(x - q * ml)

        t = bal(c[l])
        for k in range(l):
            x = (t - v[k]) * pow(MODULI[k], -1, ml)
            assert abs(x) < 2 ** 17
            t = bal(x)
        assert abs(t) <= (ml - 1) // 2
        v.append(t)
    X = v[-1]
    for l in range(14, -1, -1):
        X = X * MODULI[l] + v[l]
    return X


def test_crt_roundtrip():
    rng = np.random.default_rng(5)
    M = math.prod(MODULI)
    vals = [0, 1, -1, (M - 1) // 2, -((M - 1) // 2), 2 ** 123, -(2 ** 123)]
    vals += [int(x) * (2 ** 70) + int(y) for x, y in zip(rng.integers(-2 ** 53, 2 ** 53, 300),
                                                         rng.integers(0, 2 ** 62, 300))]
    for X in vals:
        assert crt_like_kernel([X % m for m in MODULI]) == X


def test_scaled_product_matches_float():
    """The whole chain on a small matrix: scale, residues, per-modulus integer products (what
    the int8 SYRK forms mod m), CRT -> within one rounding of the exact product."""
    rng = np.random.default_rng(7)
    K, ns = 300, 6
    d = rng.standard_normal((K, ns)) * 3.0
    b = bbits(K)
    s = b - 1 - (math.frexp(float(np.max(np.abs(d))))[1] - 1)
    a = np.rint(np.ldexp(d, s)).astype(np.int64)
    res = residues_like_kernel(a.ravel()).reshape(16, K, ns).astype(np.int64)
    exact = [[sum(int(a[k, i]) * int(a[k, j]) for k in range(K)) for j in range(ns)] for i in range(ns)]
    for i in range(ns):
        for j in range(ns):
            c = [int(np.dot(res[l, :, i], res[l, :, j])) % MODULI[l] for l in range(16)]
            assert crt_like_kernel(c) == exact[i][j]

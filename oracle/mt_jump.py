"""CPU jump-ahead for the reference's random stream (numpy's legacy MT19937), independent of
the product.

TEST INFRASTRUCTURE, like the rest of oracle/: only tests/ (and through them the GPU parity
checks) use it.  The reference draws ALL of its random numbers from one sequential
np.random.RandomState(seed) stream (digitalfilters.py:1344, :1361-1367, :1454-1467); at BASELINE
config 5 a late step's planes sit ~53 G doubles into it, which a sequential numpy pass takes
minutes to reach.  This module positions a RandomState at any double offset D of that stream in
a couple of seconds, by the textbook MT19937 jump (the state after k words is p(F) s_0 with
p(t) = t^k mod phi(t), phi the characteristic polynomial of the MT19937 transition F):

  phi(t)    Berlekamp-Massey over GF(2) on one output bit of 2 x 19937 numpy draws (polynomials
            are Python ints, bit i = coefficient of t^i);
  t^k mod phi   left-to-right binary powering (squaring by bit spreading, reduction by shifted
            XORs of phi);
  p(F) s_0  Horner over the 624-word window of untempered words (one MT19937 step per
            coefficient: x_k = x_{k-227} ^ twist(x_{k-624}, x_{k-623})).

Nothing here is shared with the product's jump (GF(2) block Horner on the device,
csrc/mt_host.cpp polynomials); tests/test_oracle_golden.py pins stream_at against plain
sequential draws of numpy itself (RandomState.uniform: two 32-bit words per double).
"""
import numpy as np

N_MT, M_MT = 624, 397
MATRIX_A = 0x9908B0DF
UPPER, LOWER = 0x80000000, 0x7FFFFFFF
DEGREE = 19937

_PHI = None
_SPREAD = None


def _berlekamp_massey(bits):
    """Connection polynomial C (int, bit i = c_i, c_0 = 1) and its length L of the GF(2)
    sequence `bits`: s_n = sum_{i=1..L} c_i s_{n-i}."""
    C, B, L, m, W = 1, 1, 0, 1, 0
    for n, s in enumerate(bits):
        W = (W << 1) | int(s)                 # bit i of W = s_{n-i}
        d = (C & W).bit_count() & 1
        if d == 0:
            m += 1
        elif 2 * L <= n:
            T = C
            C ^= B << m
            L = n + 1 - L
            B = T
            m = 1
        else:
            C ^= B << m
            m += 1
    return C, L


def char_poly():
    """phi(t) of the MT19937 word transition (degree 19937), from numpy's own output stream."""
    global _PHI
    if _PHI is None:
        bg = np.random.MT19937(0)
        out = bg.random_raw(2 * DEGREE + 64).astype(np.uint64)
        C, L = _berlekamp_massey((out & 1).tolist())
        if L != DEGREE:
            raise AssertionError("MT19937 characteristic polynomial has degree %d" % L)
        # phi(t) = t^L C(1/t): coefficient of t^(L-i) is c_i
        phi = 0
        for i in range(L + 1):
            if (C >> i) & 1:
                phi |= 1 << (L - i)
        _PHI = phi
    return _PHI


def _square(a):
    """a(t)^2 over GF(2): bit i -> bit 2i (byte-wise spreading table)."""
    global _SPREAD
    if _SPREAD is None:
        _SPREAD = [sum(((b >> i) & 1) << (2 * i) for i in range(8)) for b in range(256)]
    raw = a.to_bytes((a.bit_length() + 7) // 8 or 1, "little")
    out = bytearray(2 * len(raw))
    for i, b in enumerate(raw):
        v = _SPREAD[b]
        out[2 * i] = v & 0xFF
        out[2 * i + 1] = v >> 8
    return int.from_bytes(bytes(out), "little")


def _reduce(a, phi):
    d = phi.bit_length() - 1
    while a.bit_length() - 1 >= d:
        a ^= phi << (a.bit_length() - 1 - d)
    return a


def t_pow_mod(k, phi=None):
    """t^k mod phi(t) (int polynomial)."""
    phi = phi or char_poly()
    r = 1
    for bit in bin(k)[2:] if k > 0 else "":
        r = _reduce(_square(r), phi)
        if bit == "1":
            r = _reduce(r << 1, phi)
    return r


def _advance(buf, h):
    """One MT19937 step on the window held in the ring `buf` (logical word i at buf[(h+i)%624]);
    returns the new head."""
    a, b = buf[h], buf[(h + 1) % N_MT]
    y = (a & UPPER) | (b & LOWER)
    buf[h] = buf[(h + M_MT) % N_MT] ^ (y >> 1) ^ (MATRIX_A if y & 1 else 0)
    return (h + 1) % N_MT


def jump_window(key, k):
    """The 624-word window (x_{k-624} .. x_{k-1}, untempered) k words after the window `key`
    (numpy's state key with pos = 624), as a uint32 array: Horner evaluation of (t^k mod phi)(F)."""
    key = [int(v) for v in np.asarray(key, dtype=np.uint32)]
    if k == 0:
        return np.asarray(key, dtype=np.uint32)
    p = t_pow_mod(k)
    acc, h = [0] * N_MT, 0
    for i in range(p.bit_length() - 1, -1, -1):
        h = _advance(acc, h)
        if (p >> i) & 1:
            for j in range(N_MT):
                acc[(h + j) % N_MT] ^= key[j]
    return np.asarray([acc[(h + j) % N_MT] for j in range(N_MT)], dtype=np.uint32)


def stream_at(seed, double_offset):
    """A np.random.RandomState whose next uniform() draw is double number `double_offset` of
    np.random.RandomState(seed)'s stream (each double consumes two 32-bit words)."""
    rs = np.random.RandomState(seed)
    name, key, pos, has_gauss, cached = rs.get_state()
    if pos != N_MT:
        raise AssertionError("fresh RandomState expected at pos 624")
    win = jump_window(key, 2 * int(double_offset))
    out = np.random.RandomState()
    out.set_state((name, win, N_MT, 0, 0.0))
    return out

"""The exact int8 correlation (pods_corr mode 1, podsgen_corr_i8.hip) against exact integer
arithmetic on the host.

The kernel path scales A - mean by one power of two 2^s to integers a' (|a'| <= 2^b), forms
C' = a'^T a' exactly from 16 residue SYRKs on the int8 matrix cores and the CRT, and rounds
C' 2^-2s / ns to double once.  The host restates that with int64 limb products (exact) and
Python integers, so the kernel's C must equal it bit for bit: both round the whole integer C'
to double once (the device converts its top 64 bits with the rest folded into a sticky bit),
then scale by 2^-2s and divide by ns in IEEE arithmetic.  Against the fp64 SYRK (mode 0) and
numpy's dot the tolerance of the other correlation tests holds (1e-12 max|C|).
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    c = E.Context(0)
    yield c
    c.close()


LOG2M = 124.689  # log2 of the product of the 16 moduli, rounded down (podsgen_corr_i8.hip kLog2M)


def exact_corr(A, mean, ns_div):
    """(A - mean)^T (A - mean) / ns as the int8 path defines it: exact products of the scaled,
    rounded integers, one rounding to double."""
    d = A - mean[:, None]          # fl(a - mean), the kernel's subtraction
    K = A.shape[0]
    b = min(52, math.floor((LOG2M - 1.0 - math.log2(K)) / 2.0))
    dev = float(np.max(np.abs(d))) if d.size else 0.0
    if dev == 0.0:
        return np.zeros((A.shape[1], A.shape[1]))
    s = b - 1 - (math.frexp(dev)[1] - 1)     # b - 1 - ilogb(dev)
    a = np.rint(np.ldexp(d, s)).astype(np.int64)
    assert np.max(np.abs(a)) <= 2 ** b
    # a = l0 + l1 2^14 + l2 2^28 + l3 2^42: limb products < 2^28, so the float64 GEMM of the
    # limbs sums integers below 2^53 for K < 2^24 -- exact in any order
    assert K < 2 ** 24
    mask = (1 << 14) - 1
    limbs = [((a >> (14 * p)) & mask if p < 3 else a >> 42).astype(np.float64) for p in range(4)]
    Cp = np.zeros((A.shape[1], A.shape[1]), dtype=object)
    for p in range(4):
        for q in range(4):
            G = (limbs[p].T @ limbs[q]).astype(np.int64)
            Cp = Cp + G.astype(object) * (1 << (14 * (p + q)))
    out = np.empty(Cp.shape)
    for idx, v in np.ndenumerate(Cp):
        out[idx] = math.ldexp(float(v), -2 * s) / ns_div
    return out


def corr(ctx, snap_ns, mode):
    ctx.set_corr_mode(mode)
    C = torch.empty((snap_ns, snap_ns), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1), "pods_corr")
    return C.cpu().numpy()


def load(ctx, A):
    snap = E.load_snapshots(A, ctx=ctx)
    mean = torch.empty(A.shape[0], dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")
    return snap, mean.cpu().numpy()


def check_exact(C, ref):
    scale = np.maximum(np.abs(ref), np.finfo(float).tiny)
    rel = np.max(np.abs(C - ref) / scale)
    assert np.array_equal(C, ref), ("not the correctly rounded integer product", rel, int(np.sum(C != ref)))
    assert np.array_equal(C, C.T)


@pytest.mark.parametrize("ns,rows", [(64, 300), (100, 1000), (130, 77), (1, 5), (300, 517), (257, 4099)])
def test_corr_i8_exact(ctx, ns, rows):
    """Asymmetric data (row offsets, column scales): every tile position, ragged tiles (ns not a
    multiple of 256, K not a multiple of 64), one snapshot."""
    rng = np.random.default_rng(ns * 7 + rows)
    A = rng.standard_normal((rows, ns)) * np.arange(1, ns + 1)[None, :] + np.arange(rows)[:, None]
    snap, mean = load(ctx, A)
    C = corr(ctx, ns, 1)
    check_exact(C, exact_corr(A, mean, ns))
    C0 = corr(ctx, ns, 0)
    ref = np.dot((A - mean[:, None]).T, A - mean[:, None]) / ns
    tol = 1e-12 * max(np.max(np.abs(ref)), 1e-300)
    assert np.max(np.abs(C - ref)) <= tol and np.max(np.abs(C0 - ref)) <= tol
    ctx.set_corr_mode(1)
    del snap


def test_corr_i8_splits_chunks_and_fold(ctx, monkeypatch):
    """K split across workgroups, the residue buffer cut into several launches (partials
    accumulated mod m), and one split longer than 2048 K-steps (the accumulators reduced mod m
    mid-way): all equal the exact product, hence each other bit for bit."""
    rng = np.random.default_rng(5)
    ns, rows = 72, 140000
    A = rng.standard_normal((rows, ns)) * 3.0 + 1.5
    snap, mean = load(ctx, A)
    ref = exact_corr(A, mean, ns)
    C_auto = corr(ctx, ns, 1)
    check_exact(C_auto, ref)
    monkeypatch.setenv("PODS_CORR_SPLITS", "1")          # 2188 K-steps in one workgroup: one fold
    C_fold = corr(ctx, ns, 1)
    monkeypatch.setenv("PODS_CORR_SPLITS", "3")
    monkeypatch.setenv("PODS_CORR_BUDGET_GB", "0.0001")  # 64-chunk launches, accumulated
    C_chunk = corr(ctx, ns, 1)
    assert np.array_equal(C_fold, C_auto) and np.array_equal(C_chunk, C_auto)
    del snap


def test_corr_i8_syrk_schedules_exact(ctx, monkeypatch):
    """The product SYRK (persistent, XCD-paced, one extra ring stage) computes the exact integer
    product under every schedule the planner produces, so all equal the host's exact C bit for bit:
    the planner's own split count, a forced 3-way split (the split-major item order), several
    residue launches accumulated mod m (a tiny residue budget), both together.  The measurement
    and A/B variant switches of earlier rounds are not read by libpodsgen.so any more
    (test_host_cpu.py::test_product_library_has_no_variant_switches): setting them changes nothing."""
    rng = np.random.default_rng(17)
    ns, rows = 800, 9000   # 141 K chunks: three 64-chunk launches under the small budget
    A = rng.standard_normal((rows, ns)) * np.linspace(0.5, 3.0, ns)[None, :] + np.arange(rows)[:, None] * 1e-3
    snap, mean = load(ctx, A)
    ref = exact_corr(A, mean, ns)
    for env in ({}, {"PODS_CORR_SPLITS": "3"}, {"PODS_CORR_BUDGET_GB": "0.0001"},
                {"PODS_CORR_SPLITS": "3", "PODS_CORR_BUDGET_GB": "0.0001"},
                {"PODS_SYRK_I8": "9d", "PODS_RES_I8": "3", "PODS_CORR_ORDER": "s", "PODS_SYRK_PACE": "0"}):
        for k in ("PODS_CORR_SPLITS", "PODS_CORR_BUDGET_GB", "PODS_SYRK_I8", "PODS_RES_I8", "PODS_CORR_ORDER",
                  "PODS_SYRK_PACE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        check_exact(corr(ctx, ns, 1), ref)
    del snap


def test_corr_i8_degenerate(ctx):
    """A zero matrix and rows constant in time (A - mean = 0): C = 0 exactly; a single
    non-zero element: C has one entry, exactly a^2 / ns."""
    for A in [np.zeros((40, 9)), np.tile((np.arange(40.0) - 20.0)[:, None], (1, 9))]:
        snap, mean = load(ctx, A)
        assert not np.any(corr(ctx, 9, 1))
        del snap
    A = np.zeros((70, 5))
    A[33, 2] = 0.7
    snap, mean = load(ctx, A)
    C = corr(ctx, 5, 1)
    check_exact(C, exact_corr(A, mean, 5))
    del snap


def test_corr_i8_host_mean_and_centred(ctx):
    """The scale from k_absdev (mean set from the host) and from k_mean agree; a centred A
    (pods_center, mean operand zero) gives the same C bit for bit."""
    rng = np.random.default_rng(9)
    A = rng.standard_normal((3000, 40)) + 10.0
    snap, mean = load(ctx, A)
    C1 = corr(ctx, 40, 1)
    podsgen.check(ctx.lib.pods_set_mean(ctx.h, E.ptr(np.ascontiguousarray(mean))), "pods_set_mean")
    C2 = corr(ctx, 40, 1)
    podsgen.check(ctx.lib.pods_mean(ctx.h, None, 0), "pods_mean")
    podsgen.check(ctx.lib.pods_center(ctx.h), "pods_center")
    C3 = corr(ctx, 40, 1)
    assert np.array_equal(C1, C2) and np.array_equal(C1, C3)
    check_exact(C1, exact_corr(A, mean, 40))
    del snap


@pytest.mark.skipif(os.environ.get("PODS_CORR") == "f64", reason="fp64 SYRK selected")
def test_corr_i8_is_default(ctx):
    c2 = E.Context(0)
    assert c2.corr_mode() == 1
    c2.close()


def test_corr_i8_wide_dynamic_range(ctx):
    """VERDICT r4 item 6a.  One power of two 2^s scales the whole of A - mean to integers (its
    max element gets b bits), so a matrix with a wide dynamic range keeps fewer fixed-point bits on
    its small rows: rows scaled geometrically from 1 down to 1e-8, plus one outlier element of 1e3
    (the scale is then set by it).  C still equals the exact integer product (above), stays within
    1e-12 max|C| of numpy's fp64 np.dot (PODFS.py:1455), and the whole POD through the fused
    pods_syev gives all eigenvalues within 1e-12 lambda_0 of eigh on np.dot's C and the temporal
    modes (relative gap >= 1e-6) sign-aligned within 1e-10 of eigh's scaled vectors."""
    rng = np.random.default_rng(23)
    rows, ns, nm = 6000, 384, 12
    scale = np.logspace(0.0, -8.0, rows)
    A = (rng.standard_normal((rows, ns)) + 0.25) * scale[:, None]
    A[rows // 3, 101] += 1.0e3
    snap, mean = load(ctx, A)
    C = corr(ctx, ns, 1)
    check_exact(C, exact_corr(A, mean, ns))
    Ac = A - mean[:, None]
    ref = np.dot(Ac.T, Ac) / ns
    assert np.max(np.abs(C - ref)) <= 1e-12 * np.max(np.abs(ref))
    pod = E.run_pod(snap, nm)
    w, V = np.linalg.eigh(ref)
    lam, V = w[::-1], V[:, ::-1]
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    T = pod.T.cpu().numpy()
    checked = 0
    for j in range(pod.nm):
        gap = min(abs(lam[j] - lam[j - 1]) if j else np.inf, abs(lam[j] - lam[j + 1]))
        if gap <= 1e-6 * lam[0]:
            continue
        v = V[:, j]
        Tref = v * np.sqrt(lam[j] / (np.sum(v * v) / ns))
        sg = np.sign(np.dot(T[:, j], Tref))
        assert np.max(np.abs(sg * T[:, j] - Tref)) <= 1e-10 * np.max(np.abs(Tref)), j
        checked += 1
    assert checked >= 2
    del snap

"""GPU checks of pods_syev2 (two-stage eigensolver for ns > 4096, PODFS.py:1309-1310 at
BASELINE configs 4/5) against torch.linalg.eigh (rocSOLVER dsyevd) on the same device matrix,
with the tolerances of test_gpu_eigen.py (eigenvalues <= 1e-12 |lambda_0|; residuals,
orthogonality, sign-aligned vectors <= 1e-10 for modes with relative gap > 1e-6)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402
from test_gpu_eigen import check_against_eigh, pod_like  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    return E.Context(0)


def solve2(ctx, C, nvec):
    n = C.shape[0]
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    Y = torch.empty((n, max(nvec, 1)), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, nvec, E.ptr(lam), E.ptr(Y)), "pods_syev2")
    podsgen.check(ctx.lib.pods_syev2_status(ctx.h), "pods_syev2_status")
    return lam.cpu().numpy(), Y.cpu().numpy()[:, :nvec]


@pytest.mark.parametrize("n", [3, 34, 65, 100, 257, 1000, 2049])
def test_syev2_pod_like(ctx, n):
    C = pod_like(n, seed=n)
    lam, Y = solve2(ctx, C, min(n, 20))
    check_against_eigh(C, lam, Y)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [4096, 8192, 16384])
def test_syev2_large(ctx, n):
    C = pod_like(n, seed=7)
    lam, Y = solve2(ctx, C, 20)
    check_against_eigh(C, lam, Y)


@pytest.mark.parametrize("name", ["c1_32x32x64", "mid_40x40x520"])
def test_pipeline_two_stage_vs_reference(ctx, golden_dir, monkeypatch, name):
    """The POD through pods_syev2 (PODS_EIGEN=pods2, the ns > 4096 path) against the
    reference's own eigenvalues, modes and Fourier counts."""
    import os
    from test_gpu_parity import _check_modes, load, setup_from
    monkeypatch.setenv("PODS_EIGEN", "pods2")
    g = load(golden_dir, name)
    s = setup_from(g)
    gen = E.Generator(s, ctx=ctx)
    pod = E.run_pod(gen.generate(), s.nm)
    lam = g["energy"].real
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    assert pod.num_valid == int(g["num_valid_modes"]) and pod.nm == int(g["nm"])
    _check_modes(pod, g, s)
    fo = E.run_fourier(ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    assert np.array_equal(fo.c_count, g["N_FC"])


def _structured(kind, n, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    dev = "cuda"
    if kind == "diagonal":   # every panel column below the band is exactly zero
        return torch.diag(torch.linspace(3.0, -1.0, n, dtype=torch.float64)).to(dev).contiguous()
    if kind == "zero":
        return torch.zeros((n, n), dtype=torch.float64, device=dev)
    if kind == "banded":     # bandwidth 20 < 32: stage 1 meets zero columns under every panel
        B = torch.randn(n, n, generator=g, dtype=torch.float64)
        B = torch.triu(torch.tril(B, 20), -20)
        return (0.5 * (B + B.T)).to(dev).contiguous()
    if kind == "blockdiag":  # two dense blocks, zero coupling
        h = n // 2
        C = torch.zeros((n, n), dtype=torch.float64)
        for a, b in ((0, h), (h, n)):
            X = torch.randn(b - a, b - a, generator=g, dtype=torch.float64)
            C[a:b, a:b] = X @ X.T / (b - a)
        return C.to(dev).contiguous()
    if kind == "repeated":   # I + u u^T: eigenvalue 1 with multiplicity n - 1
        u = torch.randn(n, generator=g, dtype=torch.float64)
        return (torch.eye(n, dtype=torch.float64) + torch.outer(u, u)).to(dev).contiguous()
    raise ValueError(kind)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [34, 4200])
@pytest.mark.parametrize("kind", ["diagonal", "zero", "banded", "blockdiag", "repeated"])
@pytest.mark.parametrize("nvec", [0, 1, 64])
def test_syev2_structured(ctx, kind, n, nvec):
    """Structured and degenerate inputs of the two-stage solver (panel columns that are exactly
    zero below the band, clusters, exact multiplicities) against eigh; with tagged hand-off
    values cleared on read, a zero column stays zero and its reflector is the identity."""
    C = _structured(kind, n, seed=n + nvec)
    lam, Y = solve2(ctx, C, min(nvec, n))
    if kind == "zero":
        assert np.all(np.abs(lam) <= 1e-290)   # bisection of T = 0 (the bracket floor)
        if nvec:
            assert np.max(np.abs(Y.T @ Y - np.eye(Y.shape[1]))) <= 1e-12
        return
    check_against_eigh(C, lam, Y)
    if Y.shape[1]:
        assert np.max(np.abs(Y.T @ Y - np.eye(Y.shape[1]))) <= 1e-12


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [4500, 8192])
def test_eigvals_units_two_stage_equal_syev2(ctx, n):
    """pods_eigvals_* beyond the on-chip limit: the two-stage solver without vectors in resumable
    units (32-panel stage-1 groups, 512-group chase ranges, the bisection), advanced ONE unit
    per call with unrelated work on the stream in between, gives pods_syev2's eigenvalues bit for
    bit (same kernels, same order; the chase split over launches changes no arithmetic), and its
    abort words read 0."""
    import ctypes
    C = pod_like(n, seed=3)
    lam_ref, _ = solve2(ctx, C, 0)
    lib = ctx.lib
    slot = 2
    podsgen.check(lib.pods_eigvals_begin(ctx.h, slot, E.ptr(C), n), "pods_eigvals_begin")
    C2 = C.clone()
    C.zero_()                        # begin copied C: later units must not read it
    rem = ctypes.c_int(1)
    units = 1
    junk = torch.empty(1 << 20, dtype=torch.float64, device="cuda")
    while rem.value:
        junk.normal_()               # other work between units
        podsgen.check(lib.pods_eigvals_advance(ctx.h, slot, 1, ctypes.byref(rem)), "pods_eigvals_advance")
        units += 1
    expect = E.SpectrumQueue.two_stage_costs(n)
    assert units == len(expect), (units, len(expect))
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    podsgen.check(lib.pods_eigvals_fetch(ctx.h, slot, E.ptr(lam)), "pods_eigvals_fetch")
    podsgen.check(lib.pods_eigvals_status(ctx.h, slot), "pods_eigvals_status")
    assert np.array_equal(lam.cpu().numpy(), lam_ref)
    lr = torch.flip(torch.linalg.eigvalsh(C2), (0,)).cpu().numpy()
    assert np.max(np.abs(lam_ref - lr)) <= 1e-12 * lr[0]


@pytest.mark.timeout(600)
def test_spectrum_queue_two_stage_spreads_and_matches(ctx):
    """SpectrumQueue at ns = 8192 (BASELINE config 4) from rank 1's view of a 3-rank run: its
    owned steps' spectra run as two-stage units spread over the following steps and drained at
    the end, each equal to pods_syev2's eigenvalues bit for bit."""
    n = 8192
    mats = [pod_like(n, seed=90 + i) for i in range(3)]
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    q = E.SpectrumQueue(ctx, n, rank=1, world=3)
    assert q.max_slots == 2   # two-stage slots (ns > 4096) are bounded
    grown = 0
    for C in mats:
        q.submit(C)
        torch.cuda.synchronize()
        grown = max(grown, free0 - torch.cuda.mem_get_info()[0])
    assert q.pending or q.finished
    q.drain()
    torch.cuda.synchronize()
    grown = max(grown, free0 - torch.cuda.mem_get_info()[0])
    # device memory the queue added (its two-stage workspaces, ~1.5 n^2 doubles per slot, at most
    # two slots): recorded, and bounded well below what 16 unbounded slots would take
    print("SpectrumQueue two-stage n = %d: device memory grew %.2f GB" % (n, grown / 2 ** 30))
    assert grown < 2 * 1.6 * n * n * 8 + 2 ** 30, grown
    got = q.results()
    owned = [s for s in range(len(mats)) if q.owner(s) == 1]
    assert sorted(got) == owned and owned
    for s in owned:
        ref, _ = solve2(ctx, mats[s], 0)
        assert np.array_equal(got[s], ref), s

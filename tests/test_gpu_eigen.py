"""GPU checks of pods_syev (the POD eigensolve, PODFS.py:1309-1310 + sort_eigenvalues) against
torch.linalg.eigh (rocSOLVER dsyevd) on the same device matrix.

Tolerances (DESIGN.md 'Parity'):
  eigenvalues          |dlambda| <= 1e-12 * |lambda_0|            (all n, descending)
  eigenvectors         ||C y - lambda y|| <= 1e-12 * |lambda_0|, |Y^T Y - I| <= 1e-12,
                       sign-aligned difference <= 1e-10 for modes with relative gap > 1e-6
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    return E.Context(0)


def pod_like(n, seed=0):
    """C = B^T B / m with temporally smoothed columns: a decaying POD-like spectrum."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    m = max(n + n // 2, 8)
    B = torch.randn(m, n, generator=g, dtype=torch.float64)
    k = torch.exp(-0.5 * (torch.arange(-12, 13, dtype=torch.float64) / 4.0) ** 2)
    Bs = torch.nn.functional.conv1d(B.unsqueeze(1), k.view(1, 1, -1), padding=12).squeeze(1) + 0.05 * B
    Bd = Bs.cuda()
    C = Bd.T @ Bd / m
    return (0.5 * (C + C.T)).contiguous()


def solve(ctx, C, nvec):
    n = C.shape[0]
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    Y = torch.empty((n, max(nvec, 1)), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_syev(ctx.h, E.ptr(C), n, nvec, E.ptr(lam), E.ptr(Y)), "pods_syev")
    podsgen.check(ctx.lib.pods_syev_status(ctx.h), "pods_syev_status")
    return lam.cpu().numpy(), Y.cpu().numpy()[:, :nvec]


def check_against_eigh(C, lam, Y):
    n = C.shape[0]
    lr, Vr = torch.linalg.eigh(C)
    lr = torch.flip(lr, (0,)).cpu().numpy()
    Vr = torch.flip(Vr, (1,)).cpu().numpy()
    scale = max(abs(lr[0]), abs(lr[-1]), 1e-300)
    assert np.all(np.diff(lam) <= 0), "not descending"
    assert np.max(np.abs(lam - lr)) <= 1e-12 * scale
    nv = Y.shape[1]
    if nv == 0:
        return
    Ch = C.cpu().numpy()
    res = np.linalg.norm(Ch @ Y - Y * lam[:nv], axis=0)
    assert np.max(res) <= 1e-12 * scale
    assert np.max(np.abs(Y.T @ Y - np.eye(nv))) <= 1e-12
    gl = np.abs(np.diff(lr)) / scale
    gap = np.minimum(np.r_[gl, np.inf][:nv], np.r_[np.inf, gl][:nv])
    for k in np.nonzero(gap > 1e-6)[0]:
        s = np.sign(np.dot(Y[:, k], Vr[:, k]))
        assert np.max(np.abs(s * Y[:, k] - Vr[:, k])) <= 1e-10, (n, k)


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 255, 256, 257, 511, 512, 513, 1000, 1024, 1025,
                               2048, 2049, 3000, 4095, 4096])
def test_syev_pod_like(ctx, n):
    C = pod_like(n, seed=n)
    nvec = min(n, 20)
    lam, Y = solve(ctx, C, nvec)
    check_against_eigh(C, lam, Y)


def test_syev_values_only_and_64_vectors(ctx):
    C = pod_like(700, seed=3)
    lam0, _ = solve(ctx, C, 0)
    lam1, Y = solve(ctx, C, 64)
    assert np.array_equal(lam0, lam1)
    check_against_eigh(C, lam1, Y)


def test_syev_special_matrices(ctx):
    # diagonal (already tridiagonal: every reflector is the identity)
    d = torch.linspace(3.0, -1.0, 300, dtype=torch.float64, device="cuda")
    lam, Y = solve(ctx, torch.diag(d).contiguous(), 5)
    assert np.allclose(lam, np.sort(d.cpu().numpy())[::-1], rtol=0, atol=1e-14)
    # zero matrix
    lam, Y = solve(ctx, torch.zeros((100, 100), dtype=torch.float64, device="cuda"), 3)
    assert np.all(np.abs(lam) <= 1e-290)
    assert np.allclose(np.abs(Y.T @ Y), np.eye(3), atol=1e-12)
    # exactly repeated eigenvalues: I + u u^T (eigenvalue 1 with multiplicity n-1)
    n = 400
    u = torch.randn(n, dtype=torch.float64, device="cuda")
    C = (torch.eye(n, dtype=torch.float64, device="cuda") + torch.outer(u, u)).contiguous()
    lam, Y = solve(ctx, C, 6)
    check_against_eigh(C, lam, Y)   # the degenerate modes are skipped by the gap rule
    # orthonormal basis of the degenerate subspace anyway
    assert np.max(np.abs(Y.T @ Y - np.eye(6))) <= 1e-12


def test_syev_deterministic(ctx):
    C = pod_like(1500, seed=9)
    a = solve(ctx, C, 20)
    b = solve(ctx, C, 20)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_sytrd_similarity(ctx):
    """T from pods_sytrd has C's spectrum (eigvalsh_tridiagonal on the host)."""
    from scipy.linalg import eigvalsh_tridiagonal
    n = 2600
    C = pod_like(n, seed=1)
    d = np.zeros(n)
    e = np.zeros(n - 1)
    podsgen.check(ctx.lib.pods_sytrd(ctx.h, E.ptr(C), n, E.ptr(d), E.ptr(e)), "pods_sytrd")
    lt = np.sort(eigvalsh_tridiagonal(d, e))[::-1]
    lr = torch.flip(torch.linalg.eigvalsh(C), (0,)).cpu().numpy()
    assert np.max(np.abs(lt - lr)) <= 1e-12 * lr[0]


def test_eigen_modes_paths_agree(ctx, monkeypatch):
    """eigen_modes via pods_syev (truncated T) == via torch eigh (full T), first nm columns."""
    n, nm = 900, 20
    C = pod_like(n, seed=4)
    E.load_snapshots(np.random.default_rng(0).standard_normal((48, n)), ctx=ctx)  # sets ns
    monkeypatch.setenv("PODS_EIGEN", "pods")
    la, nva, nma, Ta = E.eigen_modes(ctx, C, n, nm, 1e-15, False)
    monkeypatch.setenv("PODS_EIGEN", "torch")
    lb, nvb, nmb, Tb = E.eigen_modes(ctx, C, n, nm, 1e-15, True)
    assert (nva, nma) == (nvb, nmb) and Ta.shape == (n, nm) and Tb.shape == (n, n)
    assert np.max(np.abs(la - lb)) <= 1e-12 * lb[0]
    Ta, Tb = Ta.cpu().numpy(), Tb.cpu().numpy()[:, :nm]
    for k in range(nm):
        s = np.sign(np.dot(Ta[:, k], Tb[:, k]))
        assert np.max(np.abs(s * Ta[:, k] - Tb[:, k])) <= 1e-9 * np.max(np.abs(Tb[:, k])), k


@pytest.mark.parametrize("n,m", [(1000, 64), (4096, 64), (777, 64), (16, 64), (8192, 64)])
def test_cheb_step_kernel(ctx, n, m):
    """pods_cheb_step: out = alpha C Y + beta Y + gamma Z on fp64 MFMA against torch, ragged n
    included (k-chunks and row tiles past n read zeros)."""
    from podsgen.subspace import Subspace
    if m > n or n > 4096:
        C = torch.randn(n, n, dtype=torch.float64, device="cuda")
    else:
        C = pod_like(n, seed=n)
    Y = torch.randn(n, m, dtype=torch.float64, device="cuda")
    Z = torch.randn(n, m, dtype=torch.float64, device="cuda")
    out = torch.empty_like(Y)
    ws = Subspace.__new__(Subspace)   # the kernel call only
    ws.ctx, ws.lib, ws.n, ws.m = ctx, ctx.lib, n, m
    ws.prepare(C)
    ws.step(C, Y, Z, 0.75, -0.5, 0.25, out)
    ref = 0.75 * (C @ Y) - 0.5 * Y + 0.25 * Z
    assert float((out - ref).abs().max()) <= 1e-13 * float(ref.abs().max())
    ws.step(C, Y, None, 1.0, 0.0, 0.0, out)
    assert float((out - C @ Y).abs().max()) <= 1e-13 * float((C @ Y).abs().max())
    a = out.clone()
    ws.step(C, Y, None, 1.0, 0.0, 0.0, out)
    assert torch.equal(a, out)   # deterministic reduction order
    C2 = C.clone()
    with pytest.raises(RuntimeError):   # a matrix that was not prepared is refused
        ws.step(C2, Y, None, 1.0, 0.0, 0.0, out)


@pytest.mark.parametrize("n,k", [(1024, 20), (2049, 20), (4096, 20), (3000, 40)])
def test_leading_eigenpairs_vs_eigh(ctx, n, k):
    """The subspace solver's k leading pairs: eigenvalues within 1e-12 lambda_0, residuals and
    orthonormality within 1e-12, sign-aligned vectors within 1e-10 (gap rule)."""
    from podsgen.subspace import leading_eigenpairs
    C = pod_like(n, seed=n + 1)
    th, X, info = leading_eigenpairs(ctx, C, k, m=64)
    lr, Vr = torch.linalg.eigh(C)
    lr = torch.flip(lr, (0,)).cpu().numpy()
    Vr = torch.flip(Vr, (1,)).cpu().numpy()
    assert np.max(np.abs(th - lr[:k])) <= 1e-12 * lr[0], info
    Xh = X.cpu().numpy()
    Ch = C.cpu().numpy()
    assert np.max(np.linalg.norm(Ch @ Xh - Xh * th, axis=0)) <= 1e-12 * lr[0]
    assert np.max(np.abs(Xh.T @ Xh - np.eye(k))) <= 1e-12
    assert info["residual"] <= 3e-14 and info["hist"][-1] == info["residual"]
    gl = np.abs(np.diff(lr)) / lr[0]
    for j in range(k):
        if min(gl[j], gl[j - 1] if j else np.inf) <= 1e-6:
            continue
        s = np.sign(np.dot(Xh[:, j], Vr[:, j]))
        assert np.max(np.abs(s * Xh[:, j] - Vr[:, j])) <= 1e-10, (j, info)


def test_eigen_split_path_matches_fused(ctx, monkeypatch):
    """eigen_modes with PODS_EIGEN=split (leading pairs by subspace iteration + eigenvalues-only
    tridiagonalisation) == the fused pods_syev: the same eigenvalues bit for bit (same
    tridiagonalisation and bisection kernels), nm and num_valid, T within 1e-10."""
    n, nm = 2500, 20
    C = pod_like(n, seed=12)
    E.load_snapshots(np.random.default_rng(0).standard_normal((48, n)), ctx=ctx)  # sets ns
    monkeypatch.setenv("PODS_EIGEN", "pods")
    la, nva, nma, Ta = E.eigen_modes(ctx, C, n, nm, 1e-15, False)
    monkeypatch.setenv("PODS_EIGEN", "split")
    lb, nvb, nmb, Tb = E.eigen_modes(ctx, C, n, nm, 1e-15, False)
    assert np.array_equal(la, lb)
    assert (nva, nma) == (nvb, nmb)
    Ta, Tb = Ta.cpu().numpy(), Tb.cpu().numpy()
    gl = np.abs(np.diff(la)) / la[0]
    for j in range(nm):
        if min(gl[j], gl[j - 1] if j else np.inf) <= 1e-6:
            continue
        s = np.sign(np.dot(Ta[:, j], Tb[:, j]))
        assert np.max(np.abs(s * Ta[:, j] - Tb[:, j])) <= 1e-10 * np.max(np.abs(Ta[:, j])), j


def test_split_path_rank_deficient(ctx, monkeypatch):
    """The split path on a rank-6 correlation (rank far below the 64-vector block: the damped
    interval's edge theta_59 is ~0) returns what the fused path returns -- the subspace result is
    checked (finite, residual <= tol) and otherwise replaced by pods_syev, never passed on as NaN
    or unconverged pairs; the eigenvalues-only spectrum is the fused solve's bit for bit."""
    n, nm = 1200, 10
    rng = np.random.default_rng(3)
    B = torch.from_numpy(rng.standard_normal((6, n)) * np.arange(1, 7)[:, None]).cuda()
    C = (B.T @ B / 6.0).contiguous()
    C = (0.5 * (C + C.T)).contiguous()
    E.load_snapshots(np.random.default_rng(0).standard_normal((48, n)), ctx=ctx)  # sets ns
    monkeypatch.setenv("PODS_EIGEN", "pods")
    la, nva, nma, Ta = E.eigen_modes(ctx, C, n, nm, 1e-6, False)
    monkeypatch.setenv("PODS_EIGEN", "split")
    lb, nvb, nmb, Tb = E.eigen_modes(ctx, C, n, nm, 1e-6, False)
    assert np.array_equal(la, lb)
    assert (nva, nma) == (nvb, nmb) and nmb == 6, (nva, nma, nvb, nmb)
    Ta, Tb = Ta.cpu().numpy()[:, :nmb], Tb.cpu().numpy()[:, :nmb]
    assert np.all(np.isfinite(Tb))
    for j in range(nmb):
        s = np.sign(np.dot(Ta[:, j], Tb[:, j]))
        assert np.max(np.abs(s * Ta[:, j] - Tb[:, j])) <= 1e-10 * np.max(np.abs(Ta[:, j])), j


@pytest.mark.parametrize("world", [1, 3, 8])
def test_spectrum_queue_spreads_and_matches(ctx, world):
    """SpectrumQueue (one owner rank's view of a `world`-rank run): the steps it owns are
    solved in units spread over later steps and drained at the end; each spectrum equals
    pods_syev's eigenvalues of the same matrix bit for bit."""
    n = 2100
    mats = [pod_like(n, seed=40 + i) for i in range(7)]
    rank = 1 if world >= 3 else 0   # from world 3 on rank 0 owns no spectrum
    q = E.SpectrumQueue(ctx, n, rank=rank, world=world)
    for C in mats:
        q.submit(C)
    q.drain()
    got = q.results()
    assert sorted(got) == [s for s in range(len(mats)) if q.owner(s) == rank]
    assert got
    for s, lam in got.items():
        ref, _ = solve(ctx, mats[s], 0)
        assert np.array_equal(lam, ref), s


def test_spectrum_queue_abort_captured_before_slot_reuse(ctx):
    """Step 0's spectrum aborts (abort word injected into its slot); step 1 reuses the slot and
    does not.  The abort words are captured when each spectrum finishes, so step 0 is recomputed
    by torch.linalg.eigvalsh (with a warning naming it) and step 1 stays pods_syev's bit for bit;
    every step's C is released once its words were read."""
    n = 1500
    mats = [pod_like(n, seed=70 + i) for i in range(3)]
    lib = ctx.lib
    begun = []

    class _Lib:
        def __getattr__(self, name):
            return getattr(lib, name)

        def pods_eigvals_begin(self, h, slot, C, n_):
            r = lib.pods_eigvals_begin(h, slot, C, n_)
            begun.append(slot)
            if len(begun) == 1:
                podsgen.check(lib.pods_eigvals_inject_abort(h, slot), "pods_eigvals_inject_abort")
            return r

    class _Ctx:
        h, device, lib = ctx.h, ctx.device, _Lib()

    q = E.SpectrumQueue(_Ctx(), n, rank=0, world=1)
    with pytest.warns(UserWarning, match="step 0"):
        for C in mats:
            q.submit(C)
        q.drain()
        got = q.results()
    assert begun[0] == begun[1], begun          # step 1 reused step 0's slot
    assert sorted(got) == [0, 1, 2]
    assert all(ent[3] is None for ent in q.finished.values())
    ref0 = torch.flip(torch.linalg.eigvalsh(mats[0]), (0,)).cpu().numpy()
    assert np.array_equal(got[0], ref0)
    for s in (1, 2):
        ref, _ = solve(ctx, mats[s], 0)
        assert np.array_equal(got[s], ref), s


@pytest.mark.parametrize("n", [64, 1000, 4096])
def test_block_kernels(ctx, n):
    """pods_gram, pods_cholqr (twice = orthonormal), pods_right_mul, pods_ritz_residual against
    torch."""
    import ctypes
    m = 64
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator(device="cpu").manual_seed(n)
    Y = torch.randn(n, m, generator=g, dtype=torch.float64).cuda()
    Z = torch.randn(n, m, generator=g, dtype=torch.float64).cuda()
    G = torch.empty((m, m), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_gram(ctx.h, P(Y), P(Z), n, m, P(G)), "pods_gram")
    ref = Y.T @ Z
    assert float((G - ref).abs().max()) <= 1e-12 * float(ref.abs().max())
    Q0, Q1 = torch.empty_like(Y), torch.empty_like(Y)
    podsgen.check(ctx.lib.pods_cholqr(ctx.h, P(Y), n, m, P(Q0)), "pods_cholqr")
    podsgen.check(ctx.lib.pods_cholqr(ctx.h, P(Q0), n, m, P(Q1)), "pods_cholqr")
    assert float((Q1.T @ Q1 - torch.eye(m, dtype=torch.float64, device="cuda")).abs().max()) <= 1e-13
    # same span: the projection of Y onto Q1 recovers Y
    assert float((Q1 @ (Q1.T @ Y) - Y).abs().max()) <= 1e-11 * float(Y.abs().max())
    M = torch.randn(m, m, generator=g, dtype=torch.float64).cuda()
    out = torch.empty_like(Y)
    podsgen.check(ctx.lib.pods_right_mul(ctx.h, P(Y), P(M), n, m, P(out)), "pods_right_mul")
    assert float((out - Y @ M).abs().max()) <= 1e-13 * float((Y @ M).abs().max())
    # Rayleigh-Ritz residual block E = CX - X H
    E_ = torch.empty_like(Y)
    podsgen.check(ctx.lib.pods_ritz_residual(ctx.h, P(Y), P(Z), P(M), n, m, P(E_)), "pods_ritz_residual")
    ref = Z - Y @ M
    assert float((E_ - ref).abs().max()) <= 1e-13 * float((Y @ M).abs().max())

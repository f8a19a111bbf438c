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

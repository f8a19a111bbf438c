"""GPU parity at the production size (BASELINE config 3: 256 x 256 inlet x 4096 snapshots).

The small golden cases (ns <= 130) never reach the code paths C3 runs: the multi-block
split-K SYRK item table, the split snapshot axis of the spatial-mode pass (ks > 1), the
DFT/ranking at ns = 4096, the tridiagonal eigensolver on a real correlation matrix, and the
RNG at stream offsets up to 885 M doubles.  This module runs the production pipeline ONCE
(module fixture) and checks it through oracle columns and fp64 torch references:

  (i)   generation: sampled steps (first, middle, the last two) bit-exact against the oracle
        (oracle.generate_steps: one pass over the reference's draw stream), plus every
        column's finiteness; the mean bit-exact against numpy's pairwise np.mean(A, 1) of the
        whole 6.4 GB matrix, and pods_center == A - mean bit for bit;
  (ii)  C: exactly symmetric; sampled 256 x 256 tiles (diagonal, bi >= 1, far off-diagonal)
        within 1e-12 * max|C| of torch's fp64 A_c^T A_c / ns;
  (iii) eigenvalues: all 4096 within 1e-12 * lambda_0 of torch.linalg.eigh on the same C;
        T sign-aligned within 1e-10 of eigh's scaled vectors (modes with relative gap > 1e-6);
  (iii') the same POD with the fp64 MFMA SYRK (pods_corr mode 0, which centres A in place)
        against torch tiles, eigh and the int8 run;
  (iv)  Phi within 1e-10 (per mode, of max|Phi_j|) of torch's A_c T Lambda^-1 / ns;
  (v)   c bit-exact against the oracle DFT (the reference expression) on the same T, and
        c_count / c_ind / FC exactly the oracle's ranking (PODFS.py:1575-1593) for every mode.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import pods_oracle as O  # noqa: E402

J, K, NS, SEED = 256, 256, 4096, 12345
STEPS = [0, 1, 2047, NS - 2, NS - 1]


@pytest.fixture(scope="module")
def c3():
    import ctypes
    import podsgen
    from podsgen import engine as E
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=SEED)
    gen = E.Generator(s, device=0)
    snap = gen.generate()
    rowlen = snap.rowlen
    rowpad = (rowlen + 15) // 16 * 16
    nbytes = rowpad * NS * 8

    def device_copy():
        t = torch.empty(rowpad * NS, dtype=torch.float64, device="cuda")
        podsgen.check(gen.ctx.lib.pods_copy(gen.ctx.h, ctypes.c_void_p(t.data_ptr()),
                                            ctypes.c_void_p(snap.data_ptr()), nbytes, 2), "pods_copy")
        torch.cuda.synchronize()
        # K-tiled (rowpad/16, ns, 16) -> reference layout rows (rowlen, ns)
        return t.view(rowpad // 16, NS, 16).permute(0, 2, 1).reshape(rowpad, NS)[:rowlen]

    A_raw = device_copy()
    pod = E.run_pod(snap, s.nm, keep_C=True)
    assert torch.equal(device_copy(), A_raw)   # the int8 correlation leaves A as generated
    # the same POD with the fp64 MFMA SYRK (pods_corr mode 0, PODS_CORR=f64): it centres A in
    # place first (k_center, main() :1493-1495), as the reference does, so A_c comes from there
    mode = gen.ctx.corr_mode()
    gen.ctx.set_corr_mode(0)
    try:
        pod64 = E.run_pod(snap, s.nm, keep_C=True)
    finally:
        gen.ctx.set_corr_mode(mode)
    A_c = device_copy()
    fo = E.run_fourier(gen.ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    torch.cuda.synchronize()
    yield dict(s=s, gen=gen, A_raw=A_raw, A_c=A_c, pod=pod, pod64=pod64, fo=fo)
    gen.ctx.close()


@pytest.mark.timeout(600)
def test_c3_generation_sampled_steps_bit_exact(c3):
    s, A = c3["s"], c3["A_raw"]
    cfg = O.DFConfig(jma=J, kma=K, ns=NS, seed=SEED)
    ref = O.generate_steps(cfg, STEPS)
    for i in STEPS:
        got = A[:, i].cpu().numpy()
        bad = np.nonzero(got != ref[i])[0]
        assert bad.size == 0, (i, bad[:8])
    assert bool(torch.isfinite(A).all())


@pytest.mark.timeout(600)
def test_c3_mean_and_centring_bit_exact(c3):
    A = c3["A_raw"]
    host = np.ascontiguousarray(A.cpu().numpy())          # (3P, ns) C-order, as main() :1397
    mean_ref = np.mean(host, 1)                           # :1492 (numpy pairwise)
    del host
    mean = c3["pod"].mean
    assert np.array_equal(mean.cpu().numpy(), mean_ref)
    assert torch.equal(c3["A_c"], A - mean[:, None])      # :1493-1495 in place


@pytest.mark.timeout(600)
def test_c3_correlation_tiles(c3):
    C = c3["pod"].C
    assert torch.equal(C, C.T)
    Ac = c3["A_c"]
    cmax = float(C.abs().max())
    b = 256
    for bi, bj in [(0, 0), (1, 0), (1, 1), (5, 3), (8, 7), (15, 0), (15, 14), (15, 15)]:
        X = Ac[:, bi * b:(bi + 1) * b]
        Y = Ac[:, bj * b:(bj + 1) * b]
        ref = (X.T @ Y) / NS
        got = C[bi * b:(bi + 1) * b, bj * b:(bj + 1) * b]
        err = float((got - ref).abs().max())
        assert err <= 1e-12 * cmax, (bi, bj, err / cmax)


@pytest.mark.timeout(600)
def test_c3_fp64_syrk_path(c3):
    """the fp64 MFMA contraction north_star names (pods_corr mode 0,
    k_syrk_g128 on the in-place-centred A) stays pinned at full size: C exactly symmetric, the
    sampled tiles within 1e-12 max|C| of torch's fp64 A_c^T A_c / ns and of the int8 path's C, all
    4096 eigenvalues within 1e-12 lambda_0 of eigh on its own C and of the int8 run's, nm /
    num_valid the same, T within 1e-10 of the int8 run's (sign-aligned, gap rule)."""
    pod, p64 = c3["pod"], c3["pod64"]
    C64, C8 = p64.C, pod.C
    assert torch.equal(C64, C64.T)
    assert torch.equal(p64.mean, pod.mean)
    Ac = c3["A_c"]
    cmax = float(C64.abs().max())
    b = 256
    for bi, bj in [(0, 0), (3, 1), (9, 9), (15, 2), (15, 15)]:
        X = Ac[:, bi * b:(bi + 1) * b]
        Y = Ac[:, bj * b:(bj + 1) * b]
        ref = (X.T @ Y) / NS
        got = C64[bi * b:(bi + 1) * b, bj * b:(bj + 1) * b]
        assert float((got - ref).abs().max()) <= 1e-12 * cmax, (bi, bj)
    assert float((C64 - C8).abs().max()) <= 1e-12 * cmax
    lam = torch.flip(torch.linalg.eigvalsh(C64), (0,)).cpu().numpy()
    assert np.max(np.abs(p64.energy - lam)) <= 1e-12 * lam[0]
    assert np.max(np.abs(p64.energy - pod.energy)) <= 1e-12 * lam[0]
    assert (p64.nm, p64.num_valid) == (pod.nm, pod.num_valid)
    T64, T8 = p64.T.cpu().numpy(), pod.T.cpu().numpy()
    for j in range(pod.nm):
        gap = min(abs(lam[j] - lam[j - 1]) if j else np.inf, abs(lam[j] - lam[j + 1]))
        if gap <= 1e-6 * lam[0]:
            continue
        sg = np.sign(np.dot(T64[:, j], T8[:, j]))
        assert np.max(np.abs(sg * T64[:, j] - T8[:, j])) <= 1e-10 * np.max(np.abs(T8[:, j])), j


@pytest.mark.timeout(600)
def test_c3_eigen_and_temporal_modes(c3):
    pod, s = c3["pod"], c3["s"]
    lam_t, V = torch.linalg.eigh(pod.C)
    lam = torch.flip(lam_t, (0,)).cpu().numpy()
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    assert pod.num_valid == O.num_valid_modes(lam, NS) and pod.nm == s.nm
    nm = pod.nm
    Vd = torch.flip(V, (1,))[:, :nm].cpu().numpy()
    T = pod.T.cpu().numpy()[:, :nm]
    for j in range(nm):
        v = Vd[:, j]
        Tref = v * np.sqrt(lam[j] / (np.sum(v * v) / NS))
        gap = min(abs(lam[j] - lam[j - 1]) if j else np.inf, abs(lam[j] - lam[j + 1]))
        if gap <= 1e-6 * lam[0]:
            continue
        sg = np.sign(np.dot(T[:, j], Tref))
        assert np.max(np.abs(sg * T[:, j] - Tref)) <= 1e-10 * np.max(np.abs(Tref)), j


@pytest.mark.timeout(600)
def test_c3_spatial_modes_split_path(c3):
    pod = c3["pod"]
    nm = pod.nm
    T = pod.T[:, :nm]
    lam = torch.from_numpy(np.ascontiguousarray(pod.energy[:nm])).to(T.device)
    ref = (c3["A_c"] @ T) / lam[None, :] / NS             # PODFS.py:1330-1333
    phi = pod.phi
    for j in range(nm):
        err = float((phi[:, j] - ref[:, j]).abs().max())
        assert err <= 1e-10 * float(ref[:, j].abs().max()), j
    # unit 2-norm columns (the POD property the reference's modes carry)
    norms = torch.linalg.vector_norm(phi, dim=0).cpu().numpy()
    assert np.all(np.abs(norms - 1.0) <= 1e-9), norms


@pytest.mark.timeout(600)
def test_c3_fourier_and_ranking(c3):
    from podsgen import engine as E
    pod, fo, s = c3["pod"], c3["fo"], c3["s"]
    T = pod.T.cpu().numpy()
    ref = O.fourier(T, NS, s.dt_eff, pod.nm, s.et)
    assert fo.period == ref["period"]
    # every coefficient bit-equal: the device multiplies by the host's np.exp twiddles
    assert np.array_equal(fo.c, ref["c"]), int(np.sum(fo.c != ref["c"]))
    # so the discrete outputs are the oracle's for every mode, unconditionally
    assert np.array_equal(fo.c_count, ref["c_count"]), (fo.c_count, ref["c_count"])
    assert np.array_equal(fo.c_ind, ref["c_ind"])
    assert np.array_equal(fo.FC, ref["FC"])
    # and the GPU ranking kernel equals the host restatement on the same c
    c_ind, c_count, FC = E.host_rank_and_count(fo.c, s.et)
    assert np.array_equal(fo.c_count, c_count) and np.array_equal(fo.c_ind, c_ind)


@pytest.mark.timeout(600)
def test_c3_split_eigensolve(c3, monkeypatch):
    """The multi-rank eigensolve on the real C3 matrix: the 20 leading pairs by Chebyshev-filtered
    subspace iteration (pods_cheb_step) and the eigenvalues-only tridiagonalisation -- the
    eigenvalues are pods_syev's bit for bit, T within 1e-10 of eigh's scaled vectors (gap rule),
    nm / num_valid the same."""
    from podsgen import engine as E
    pod, s = c3["pod"], c3["s"]
    monkeypatch.setenv("PODS_EIGEN", "split")
    lam, nvalid, nmt, T = E.eigen_modes(c3["gen"].ctx, pod.C, NS, s.nm, 1e-15, False)
    assert np.array_equal(lam, pod.energy)
    assert (nvalid, nmt) == (pod.num_valid, pod.nm)
    lam_t, V = torch.linalg.eigh(pod.C)
    lr = torch.flip(lam_t, (0,)).cpu().numpy()
    Vd = torch.flip(V, (1,))[:, :nmt].cpu().numpy()
    T = T.cpu().numpy()
    for j in range(nmt):
        v = Vd[:, j]
        Tref = v * np.sqrt(lr[j] / (np.sum(v * v) / NS))
        gap = min(abs(lr[j] - lr[j - 1]) if j else np.inf, abs(lr[j] - lr[j + 1]))
        if gap <= 1e-6 * lr[0]:
            continue
        sg = np.sign(np.dot(T[:, j], Tref))
        assert np.max(np.abs(sg * T[:, j] - Tref)) <= 1e-10 * np.max(np.abs(Tref)), j

"""GPU parity: every HIP kernel through the C ABI against the oracle / golden fixtures.

Bit-exact: RNG stream, generated snapshots A (filters + Lund + rotation), mean.
Tolerances (stated here, DESIGN.md 'Parity'):
  C               |dC| <= 1e-12 * max|C|          (MFMA fp64 vs BLAS dsyrk order)
  eigenvalues     |dlambda| <= 1e-12 * lambda_0    (eigh vs dgeev)
  T, Phi          per-mode sign-aligned, <= 1e-10 * scale, for modes with a relative
                  eigen-gap > 1e-6 (near-degenerate pairs are checked by subspace)
  Fourier c       complex64, |dc| <= 2 ulp(f32) of max|c| per mode, given identical T
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import pods_oracle as O  # noqa: E402
import podsgen  # noqa: E402
from podsgen import engine as E
from podsgen import _lib  # noqa: E402

CASES = ["c1_32x32x64", "cli_10x11x5", "odd_12x9x17_aniso", "prf_8x12x9", "rot_6x7x6",
         "dtanh_9x12x7", "circ_11x10x6", "ring_12x13x6", "readprf_case", "prof1d_14x16x8"]


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"))


def setup_from(g):
    kw = dict(jma=int(g["cfg_jma"]), kma=int(g["cfg_kma"]), ns=int(g["cfg_ns"]), seed=int(g["cfg_seed"]))
    if "cfg_dt" in g.files:
        kw["dt"] = float(g["cfg_dt"])
    if "cfg_normal" in g.files:
        kw["normal"] = tuple(g["cfg_normal"])
    if "prf_U" in g.files:
        kw["prf"] = {k[4:]: np.array(g[k]) for k in g.files if k.startswith("prf_")}
    if "cfg_mean_profile" in g.files:
        kw["mean_profile"] = str(g["cfg_mean_profile"])
    if "cfg_inner_d" in g.files:
        kw["inner_d"] = float(g["cfg_inner_d"])
    if "cfg_ln_prf" in g.files:
        kw["ln_prf"] = float(g["cfg_ln_prf"])
    if "cfg_profile_text" in g.files:
        from test_oracle_golden import profile1d_from_text
        kw["profile1d"] = profile1d_from_text(str(g["cfg_profile_text"]), kw["kma"])
    return podsgen.DFSetup(**kw)


@pytest.mark.parametrize("profile", ["double-hyperbolic-tangent", "circular-hyperbolic-tangent",
                                     "ring-hyperbolic-tangent"])
def test_generate_adapt2d_large_vs_oracle(ctx, profile):
    """adapt2d at a non-square 96 x 70 inlet (j-varying Lund table through the fused y/z
    kernel, rotated normal): bit-exact against the oracle's per-point loop."""
    kw = dict(jma=96, kma=70, ns=5, seed=61, mean_profile=profile, normal=(1.0, -0.4, 0.2), inner_d=0.35)
    gen = E.Generator(podsgen.DFSetup(**kw), ctx=ctx)
    A = gen.generate().to_host()
    assert np.array_equal(A, O.generate(O.DFConfig(**kw)))


def test_adapt2d_operator_golden(golden_dir):
    """digitalfilters.adapt2d (drop-in operator, GPU transform) on the reference's fixture."""
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "unit_adapt2d.npz"))
    for tag in ["dtanh", "circ", "circ_odd", "ring", "ring_thin"]:
        J, K, inner = g[tag + "_cfg"]
        y = [np.array(v) for v in g[tag + "_in"]]
        df.adapt2d(y[0], y[1], y[2], *g[tag + "_prof"], int(J), int(K), str(g[tag + "_name"]), float(inner))
        assert np.array_equal(np.stack(y), g[tag + "_out"], equal_nan=True), tag


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    c = E.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("layout", ["default", "long_substreams"])
def test_rng_stream_bit_exact(ctx, monkeypatch, layout):
    """numpy's legacy MT19937 stream bit for bit through the jump-ahead (k_mt_jump3) and the
    generator, with the default substream layout and a different one (PODS_MT_SUBSTREAMS=64:
    twice the blocks per substream)."""
    monkeypatch.delenv("PODS_MT_SUBSTREAMS", raising=False)
    if layout == "long_substreams":
        monkeypatch.setenv("PODS_MT_SUBSTREAMS", "64")
    lib = ctx.lib
    for seed, n in [(12345, 1000), (7, 3_000_001), (2**32 - 1, 25_000_000)]:
        out = torch.empty(n, dtype=torch.float64, device="cuda")
        podsgen.check(lib.pods_rng_uniform(ctx.h, seed, n, -np.sqrt(3.0), 2 * np.sqrt(3.0),
                                           E.ptr(out)), "rng")
        ref = np.random.RandomState(seed).uniform(-np.sqrt(3.0), np.sqrt(3.0), n)
        got = out.cpu().numpy()
        bad = np.nonzero(got != ref)[0]
        assert bad.size == 0, (seed, n, bad[:10])


def test_filter_block_golden(ctx, golden_dir):
    g = np.load(os.path.join(golden_dir, "unit_filter.npz"))
    x = np.ascontiguousarray(g["x"])
    y = np.zeros((7, 5))
    podsgen.check(ctx.lib.pods_filter_block(ctx.h, E.ptr(x), 9, 6, 4, 7, 5, E.ptr(g["taps_9"]),
                                            E.ptr(g["taps_6"]), E.ptr(g["taps_4"]), E.ptr(y)), "filter")
    assert np.array_equal(y, g["y"])


@pytest.mark.parametrize("name", CASES)
def test_generate_bit_exact(ctx, golden_dir, name):
    g = load(golden_dir, name)
    s = setup_from(g)
    gen = E.Generator(s, ctx=ctx)
    A = gen.generate().to_host()
    bad = np.argwhere(A != g["A_raw"])
    assert bad.size == 0, (name, bad[:5], A.flat[:3], g["A_raw"].flat[:3])
    pod = E.run_pod(gen.snapshots(), s.nm, keep_C=True)
    assert np.array_equal(pod.mean.cpu().numpy(), g["mean_field"])
    # correlation
    C = pod.C.cpu().numpy()
    assert np.max(np.abs(C - g["C"])) <= 1e-12 * np.max(np.abs(g["C"]))
    assert np.array_equal(C, C.T)
    # eigenvalues, valid modes
    lam = pod.energy
    ref = g["energy"].real
    assert np.max(np.abs(lam - ref)) <= 1e-12 * ref[0]
    assert pod.num_valid == int(g["num_valid_modes"]) and pod.nm == int(g["nm"])
    _check_modes(pod, g, s)


def _check_modes(pod, g, s):
    nm = pod.nm
    lam = g["energy"].real
    T = pod.T.cpu().numpy()[:, :nm]
    Tg = g["temporal_modes"].real
    Phi = pod.phi.cpu().numpy()
    Pg = g["spatial_modes"]
    for j in range(nm):
        gap = min(abs(lam[j] - lam[j - 1]) if j else np.inf, abs(lam[j] - lam[j + 1]))
        if gap <= 1e-6 * lam[0]:
            continue
        sgn = np.sign(np.dot(T[:, j], Tg[:, j]))
        assert np.max(np.abs(sgn * T[:, j] - Tg[:, j])) <= 1e-10 * np.max(np.abs(Tg[:, j])), j
        assert np.max(np.abs(sgn * Phi[:, j] - Pg[:, j])) <= 1e-10 * np.max(np.abs(Pg[:, j])), j


@pytest.mark.parametrize("name", ["c1_32x32x64", "cli_10x11x5", "odd_12x9x17_aniso"])
def test_fourier_vs_oracle_same_T(ctx, golden_dir, name):
    g = load(golden_dir, name)
    s = setup_from(g)
    gen = E.Generator(s, ctx=ctx)
    snap = gen.generate()
    pod = E.run_pod(snap, s.nm)
    fo = E.run_fourier(ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    T = pod.T.cpu().numpy()
    ref = O.fourier(T, s.ns, s.dt_eff, pod.nm, s.et)
    assert fo.period == ref["period"]
    # bit-exact: the device multiplies by the host's np.exp twiddles in numpy's pairwise order
    assert np.array_equal(fo.c, ref["c"]), np.max(np.abs(fo.c - ref["c"]))
    # the GPU's discrete outputs: ranking, counts and FC rows exactly the oracle's
    assert np.array_equal(fo.c_count, ref["c_count"]), (fo.c_count, ref["c_count"])
    assert np.array_equal(fo.c_ind, ref["c_ind"])
    assert np.array_equal(fo.FC, ref["FC"])


@pytest.mark.parametrize("name", CASES)
def test_fourier_counts_vs_golden(ctx, golden_dir, name):
    """GPU N_FC / FC against the reference's own fourier_coefficients output (golden N_FC, FC
    from PODFS.py:1578-1639): counts and coefficient order exact; values equal up to the
    per-mode eigenvector sign (dgeev's vs ours) within complex64 rounding."""
    g = load(golden_dir, name)
    s = setup_from(g)
    gen = E.Generator(s, ctx=ctx)
    pod = E.run_pod(gen.generate(), s.nm)
    fo = E.run_fourier(ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    assert fo.period == float(g["period"])
    assert np.array_equal(fo.c_count, g["N_FC"]), (fo.c_count, g["N_FC"])
    FC, FCg = fo.FC, g["FC"]
    assert FC.shape == FCg.shape
    assert np.array_equal(FC[:, 0], FCg[:, 0])
    start = 0
    for n in fo.c_count:
        blk, ref = FC[start:start + n, 1:], FCg[start:start + n, 1:]
        sg = np.sign(np.sum(blk * ref))
        scale = np.max(np.abs(ref))
        assert np.max(np.abs(sg * blk - ref)) <= 4 * np.spacing(np.float32(scale)), start
        start += n


def _rank_cases():
    rng = np.random.default_rng(11)
    for ns, nm in [(4096, 20), (17, 3), (64, 20), (1, 1), (5000, 4), (16384, 2), (8, 5)]:
        c = (rng.standard_normal((ns, nm)) + 1j * rng.standard_normal((ns, nm)) *
             rng.random((ns, nm)) ** 3).astype(np.complex64)
        if ns > 8:
            h = ns // 2
            c[h + 1:] = np.conj(c[1:ns - h][::-1])       # exact conjugate pairs -> ties
            c[3] = c[5]                                   # plain ties
            c[7] = 0                                      # zeros
            c[:4, 0] = (rng.standard_normal(4) * 1e-30).astype(np.complex64)
        yield ns, nm, c


@pytest.mark.parametrize("et", [0.9, 0.5, 1.0])
def test_fourier_rank_matches_host(ctx, et):
    """pods_fourier_rank == the host restatement of PODFS.py:1575-1593 (numpy f32 abs,
    lexsort ties, pairwise f32 sum, float64 running count), exactly."""
    for ns, nm, c in _rank_cases():
        cdev = torch.from_numpy(np.ascontiguousarray(c).view(np.float32).reshape(ns, nm, 2)).cuda()
        ind = torch.empty((nm, ns), dtype=torch.int32, device="cuda")
        cnt = torch.empty(nm, dtype=torch.int64, device="cuda")
        podsgen.check(ctx.lib.pods_fourier_rank(ctx.h, E.ptr(cdev), nm, ns, float(et), E.ptr(ind),
                                                E.ptr(cnt)), "pods_fourier_rank")
        ci, cc = ind.cpu().numpy(), cnt.cpu().numpy()
        if np.any(cc < 0):  # et = 1: the f64 running sum can stay below f64(f32 sum)
            with pytest.raises(IndexError):
                E.host_rank_and_count(c, et)
            continue
        ref_ind, ref_cnt, ref_FC = E.host_rank_and_count(c, et)
        assert np.array_equal(cc, ref_cnt), (ns, cc, ref_cnt)
        assert np.array_equal(ci, ref_ind), ns
        assert np.array_equal(E.fc_rows(c, ci, cc), ref_FC), ns


def test_syrk_mfma_layout(ctx):
    """Asymmetric data through pods_set_snapshots: catches row/col swaps in the MFMA C map,
    including a case with several tile rows and K splits."""
    rng = np.random.default_rng(3)
    for ns, rows in [(64, 300), (100, 1000), (130, 77), (1, 5), (300, 5000)]:
        A = rng.standard_normal((rows, ns)) * np.arange(1, ns + 1)[None, :] + np.arange(rows)[:, None]
        snap = E.load_snapshots(A, ctx=ctx)
        mean = torch.empty(rows, dtype=torch.float64, device="cuda")
        podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "mean")
        assert np.array_equal(mean.cpu().numpy(), np.mean(A, 1))
        C = torch.empty((ns, ns), dtype=torch.float64, device="cuda")
        podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1), "corr")
        Ac = A - np.mean(A, 1)[:, None]
        ref = np.dot(Ac.T, Ac) / ns
        assert np.max(np.abs(C.cpu().numpy() - ref)) <= 1e-12 * max(np.max(np.abs(ref)), 1e-300), (ns, rows)
        del snap


def test_prefetched_generation_matches(ctx):
    """The next run's MT19937 jump-ahead enqueued on the gen stream (Generator.prefetch_jump)
    while the main stream still works on this run: the following generate() (planes, x and y/z
    passes) gives the same snapshot matrix bit for bit, and a prefetched pipeline step the same
    POD."""
    s = podsgen.DFSetup(jma=40, kma=27, ns=30, seed=5)
    gen = E.Generator(s, ctx=ctx)
    ref = gen.generate().to_host()
    gen.prefetch_jump()
    mean = torch.empty(gen.rowlen, dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")  # main-stream work meanwhile
    podsgen.check(ctx.lib.pods_center(ctx.h), "pods_center")
    assert np.array_equal(gen.generate().to_host(), ref)
    s2 = podsgen.DFSetup(jma=24, kma=20, ns=64, seed=2024)
    g2 = E.Generator(s2, ctx=ctx)
    _, p1, f1 = E.pipeline(s2, gen=g2, prefetch_next=True)
    _, p2, f2 = E.pipeline(s2, gen=g2)
    assert np.array_equal(p1.energy, p2.energy) and p1.nm == p2.nm
    assert torch.equal(p1.phi, p2.phi) and np.array_equal(f1.c, f2.c)


def test_planes_prefetched_beside_solver(ctx):
    """ns > 2048: the next run's random planes start on the gen stream behind the marker of
    tridiagonalisation range 3 (Generator.prefetch_planes_beside_solver) while the solver's
    late ranges run, and (by default, engine.XPASS_BESIDE) its x pass behind the solver's
    eigenvalues, beside the eigenvectors and back-transformation.  The next step's snapshot
    matrix and POD equal a plain run's bit for bit, and no persistent kernel aborted (no
    fallback warning)."""
    import warnings
    s = podsgen.DFSetup(jma=24, kma=20, ns=2560, seed=31)
    g1 = E.Generator(s, ctx=ctx)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        E.pipeline(s, gen=g1, prefetch_next=True)
        assert g1._ahead_parts == (_lib.PODS_GEN_JUMP | _lib.PODS_GEN_PLANES
                                   | (_lib.PODS_GEN_XPASS if E.XPASS_BESIDE else 0))
        _, p2, f2 = E.pipeline(s, gen=g1)
        A2 = g1.snapshots().to_host()
    assert not [x for x in w if "podsgen" in str(x.message)], [str(x.message) for x in w]
    c2 = E.Context(0)
    g2 = E.Generator(s, ctx=c2)
    _, p3, f3 = E.pipeline(s, gen=g2)
    assert np.array_equal(A2, g2.snapshots().to_host())
    assert np.array_equal(p2.energy, p3.energy) and p2.nm == p3.nm
    assert torch.equal(p2.phi, p3.phi) and np.array_equal(f2.c, f3.c)
    c2.close()


def test_spatial_pass_overlapping_next_generation(ctx):
    """One device, three runs with overlap_spatial (engine.pipeline): the runs alternate between
    the two snapshot banks and each run's spatial-mode pass runs on its own stream beside the next
    run's generation.  Every run's Phi (read after pod.phi_ready), mean, energy and Fourier
    coefficients equal the plain runs' bit for bit, and consecutive runs of different seeds differ
    (so a bank mix-up would show)."""
    s = podsgen.DFSetup(jma=24, kma=20, ns=2560, seed=41)
    g1 = E.Generator(s, ctx=ctx)
    got = []
    for k, seed in enumerate((41, 42, 43)):
        podsgen.check(ctx.lib.pods_df_set_seed(ctx.h, seed), "pods_df_set_seed")
        _, p, f = E.pipeline(s, gen=g1, prefetch_next=False, overlap_spatial=True)
        assert p.phi_ready is not None
        p.phi_ready.synchronize()
        got.append((p.phi.cpu().numpy(), p.mean.cpu().numpy(), p.energy, f.c))
    c2 = E.Context(0)
    g2 = E.Generator(s, ctx=c2)
    for k, seed in enumerate((41, 42, 43)):
        podsgen.check(c2.lib.pods_df_set_seed(c2.h, seed), "pods_df_set_seed")
        _, p, f = E.pipeline(s, gen=g2)
        assert p.phi_ready is None
        phi, mean, energy, c = got[k]
        assert np.array_equal(phi, p.phi.cpu().numpy()), k
        assert np.array_equal(mean, p.mean.cpu().numpy()) and np.array_equal(energy, p.energy), k
        assert np.array_equal(c, f.c), k
    assert not np.array_equal(got[0][0], got[1][0])
    # one seed, the next runs prefetched (the deferred join: a run's Phi completes beside the
    # next run's generation)
    podsgen.check(ctx.lib.pods_df_set_seed(ctx.h, 41), "pods_df_set_seed")
    for k in range(3):
        _, p, f = E.pipeline(s, gen=g1, prefetch_next=k < 2, overlap_spatial=True)
        p.phi_ready.synchronize()
        assert np.array_equal(p.phi.cpu().numpy(), got[0][0]), k
        assert np.array_equal(f.c, got[0][3]), k
    c2.close()


def test_speculative_modes_fallback(ctx):
    """One device: the temporal/spatial modes are enqueued behind pods_syev for nm_trunc = nm
    before the host reads the spectrum.  With fewer valid modes than nm (a rank-6 correlation,
    nm = 10) they are redone on the host path: the result equals the oracle's POD."""
    rng = np.random.default_rng(11)
    A = rng.standard_normal((6, 30)) * np.arange(1, 7)[:, None]
    snap = E.load_snapshots(A, ctx=ctx)
    pod = E.run_pod(snap, 10, tol_CN=1e-6)
    _, Ac = O.mean_and_center(A)
    ref = O.pod(Ac, 30, 10, tol_CN=1e-6)
    assert pod.num_valid == ref["num_valid"] and pod.nm == ref["nm"] and pod.nm < 10, (pod.num_valid, ref["num_valid"])
    lam = ref["energy"].real
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    T, Phi = pod.T.cpu().numpy(), pod.phi.cpu().numpy()
    for j in range(pod.nm):
        sgn = np.sign(np.dot(T[:, j], ref["T"][:, j].real))
        assert np.max(np.abs(sgn * T[:, j] - ref["T"][:, j].real)) <= 1e-10 * np.max(np.abs(ref["T"][:, j])), j
        Pg = ref["spatial"][:, j].real
        assert np.max(np.abs(sgn * Phi[:, j] - Pg)) <= 1e-10 * np.max(np.abs(Pg)), j


def test_row_slabs_match_full(ctx):
    """Multi-GPU sharding on one device: 3 row slabs concatenate to the full generation."""
    s = podsgen.DFSetup(jma=20, kma=17, ns=11, seed=99)
    full = E.Generator(s, ctx=ctx).generate().to_host()
    P = s.P
    parts = []
    for r in range(3):
        c2 = E.Context(0)
        gen = E.Generator(s, rank=r, world=3, ctx=c2)
        parts.append((gen.j0, gen.j1, gen.generate().to_host()))
        c2.close()
    for comp in range(3):
        rows = np.concatenate([a[comp * (j1 - j0) * s.kma:(comp + 1) * (j1 - j0) * s.kma]
                               for j0, j1, a in parts])
        assert np.array_equal(rows, full[comp * P:(comp + 1) * P])


@pytest.mark.parametrize("J,K,ns,world", [(256, 256, 7, 8), (96, 70, 9, 5), (64, 40, 5, 2)])
def test_row_slabs_large(ctx, J, K, ns, world):
    """Row slabs at 256^2 (8 ranks) and odd shapes: the slab generator (twist-only blocks
    outside the slab) reproduces the rows of the single-GPU generation bit for bit."""
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=2718)
    full = E.Generator(s, ctx=ctx).generate().to_host()
    P = s.P
    parts = []
    for r in range(world):
        gen = E.Generator(s, rank=r, world=world, ctx=ctx)
        parts.append((gen.j0, gen.j1, gen.generate().to_host()))
    for comp in range(3):
        rows = np.concatenate([a[comp * (j1 - j0) * K:(comp + 1) * (j1 - j0) * K] for j0, j1, a in parts])
        assert np.array_equal(rows, full[comp * P:(comp + 1) * P]), comp


@pytest.mark.parametrize("J,K,ns,world", [(256, 256, 40, 8), (96, 70, 33, 5), (64, 40, 61, 2), (64, 40, 5, 3)])
def test_mt_state_exchange_bit_exact(J, K, ns, world):
    """The multi-GPU state exchange (pods_df_set_exchange): every rank twists only its 1/world of
    the MT19937 stream, records the segment-start states of every rank, the records move by an
    all_to_all (emulated here on one device: rank r's send chunk for q, concatenated over r),
    and each rank regenerates only its own row segments -- the snapshot rows bit for bit those of
    the slab generator that twists the whole stream (digitalfilters.py:1361-1367, :1454-1467)."""
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=977)
    gens = [E.Generator(s, rank=r, world=world, ctx=E.Context(0), exchange=False) for r in range(world)]
    for g in gens:
        g.enable_exchange()
        podsgen.check(g.ctx.lib.pods_df_generate_parts(g.ctx.h, _lib.PODS_GEN_JUMP | _lib.PODS_GEN_RECORD), "record")
    torch.cuda.synchronize()
    for q, gq in enumerate(gens):
        chunks = []
        for gr in gens:
            sb = gr._xch[0]
            off = sum(sb[:q])
            chunks.append(gr._send[off:off + sb[q]])
        recv = torch.cat(chunks)
        assert recv.numel() == sum(gq._xch[1])
        gq._recv[:recv.numel()].copy_(recv)
        podsgen.check(gq.ctx.lib.pods_df_generate_parts(
            gq.ctx.h, _lib.PODS_GEN_PLANES | _lib.PODS_GEN_XPASS | _lib.PODS_GEN_YZPASS), "segments")
    for q, gq in enumerate(gens):
        got = gq.snapshots().to_host()
        ref = E.Generator(s, rank=q, world=world, ctx=gq.ctx, exchange=False).generate().to_host()
        assert np.array_equal(got, ref), q
    for g in gens:
        g.ctx.close()


def test_center_in_place(ctx):
    """pods_center: A - mean (main() :1493-1495) in place, bit for bit the numpy subtraction;
    the correlation from the centred A equals the one that subtracts inside the SYRK."""
    s = podsgen.DFSetup(jma=40, kma=24, ns=48, seed=8)
    gen = E.Generator(s, ctx=ctx)
    snap = gen.generate()
    A = snap.to_host()
    mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")
    C0 = torch.empty((s.ns, s.ns), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C0), 1), "pods_corr")
    podsgen.check(ctx.lib.pods_center(ctx.h), "pods_center")
    Ac = snap.to_host()
    assert np.array_equal(Ac, A - mean.cpu().numpy()[:, None])
    C1 = torch.empty_like(C0)
    podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C1), 1), "pods_corr")
    assert torch.equal(C0, C1)


@pytest.mark.parametrize("kw", [dict(jma=32, kma=32, ns=64, seed=12345),
                                dict(jma=40, kma=27, ns=30, seed=5, normal=(1.0, -0.4, 0.2))])
def test_generate_ragged_tiles_vs_oracle(ctx, kw):
    """Generation bit-exact against the oracle on full tiles and ragged edge tiles (40 x 27)
    with a rotated normal."""
    A = E.Generator(podsgen.DFSetup(**kw), ctx=ctx).generate().to_host()
    assert np.array_equal(A, O.generate(O.DFConfig(**kw)))


def test_medium_case_vs_oracle(ctx):
    """256 x 256 inlet, 24 steps: generation bit-exact against the oracle."""
    s = podsgen.DFSetup(jma=256, kma=256, ns=24, seed=4242)
    A = E.Generator(s, ctx=ctx).generate().to_host()
    cfg = O.DFConfig(jma=256, kma=256, ns=24, seed=4242)
    ref = O.generate(cfg)
    assert np.array_equal(A, ref)


def test_mid_case_vs_reference(ctx, golden_dir):
    """40 x 40 x 520 against the reference's own outputs (reduced fixture): three 256-row
    SYRK blocks with split K, the spatial-mode pass with its snapshot axis split (ks = 4) and
    the k_spatial_reduce, the eigensolver at n = 520 and the DFT/ranking at ns = 520."""
    from podsgen import engine as E_
    g = load(golden_dir, "mid_40x40x520")
    s = setup_from(g)
    gen = E_.Generator(s, ctx=ctx)
    snap = gen.generate()
    A = snap.to_host()
    for k, i in enumerate(g["A_steps"]):
        assert np.array_equal(A[:, i], g["A_cols"][k]), i
    pod = E_.run_pod(snap, s.nm, keep_C=True)
    assert np.array_equal(pod.mean.cpu().numpy(), g["mean_field"])
    C = pod.C.cpu().numpy()
    assert np.array_equal(C, C.T)
    cmax = float(g["C_max"])
    assert np.max(np.abs(C[g["C_rows_idx"]] - g["C_rows"])) <= 1e-12 * cmax
    assert np.max(np.abs(np.diag(C) - g["C_diag"])) <= 1e-12 * cmax
    assert np.max(np.abs(C.sum(axis=0) - g["C_colsum"])) <= 1e-12 * cmax * s.ns
    lam = g["energy"].real
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    assert pod.num_valid == int(g["num_valid_modes"]) and pod.nm == int(g["nm"])
    _check_modes(pod, g, s)
    fo = E_.run_fourier(ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    assert np.array_equal(fo.c_count, g["N_FC"]), (fo.c_count, g["N_FC"])
    assert np.array_equal(fo.FC[:, 0], g["FC"][:, 0])


@pytest.mark.parametrize("J,K,ns,kw", [
    (9, 1024, 3, {}),                                             # C5 width: four 256-column tiles
    (11, 600, 4, {"dt": 0.05}),                                   # K not a multiple of 16, nfx != nfy
    (37, 530, 3, {}),                                             # ragged row and column tiles
])
def test_generate_wide_inlet_vs_oracle(ctx, J, K, ns, kw):
    """kma up to 1024 (BASELINE config 5's 1024-point span): bit-exact against the oracle."""
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=77, **kw)
    A = E.Generator(s, ctx=ctx).generate().to_host()
    ref = O.generate(O.DFConfig(jma=J, kma=K, ns=ns, seed=77, **kw))
    assert np.array_equal(A, ref)


def test_generate_c5_style_prf_vs_oracle(ctx):
    """The C5 workload (adapt2prf with a synthetic inhomogeneous stress field, anisotropic
    x filter from -t) on a 12 x 640 inlet: bit-exact against the oracle."""
    import bench
    J, K, ns = 12, 640, 4
    prf = bench.c5_profile(J, K)
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=5, dt=0.05, prf=prf)
    assert s.nfx > s.nfy
    A = E.Generator(s, ctx=ctx).generate().to_host()
    ref = O.generate(O.DFConfig(jma=J, kma=K, ns=ns, seed=5, dt=0.05, prf=prf))
    assert np.array_equal(A, ref)

"""GPU: BASELINE config 5 at full size -- 1024 x 1024 inlet x 16384 snapshots, anisotropic
length scales (-t halves dt: lnx = 2 ln, nfx = 12, digitalfilters.py:1315-1322) and an
inhomogeneous Reynolds-stress field through adapt2prf (:180-231) -- run on ONE device as the 8
row slabs the 8-GPU job uses (412 GB of snapshots do not fit one GPU; one slab's 51.5 GB do).

Pass 1, slab by slab through the product's own slab generator (the same code each rank of
the 8-GPU run executes): generate, mean, centre, partial correlation A_g^T A_g (SYRK,
divide = 0), packed lower triangle (pods_pack_lower); the packed partials are summed in rank
order (the RCCL all-reduce's arithmetic) and unpacked / ns into C (pods_unpack_lower).
Eigensolve on the summed C with the product's path for ns = 16384 (pods_syev2).
Pass 2: each slab regenerated and its spatial modes formed (pods_spatial_modes).

Checked: generation of every slab's rows bit-exact against the oracle at steps 0, 1, 2047 (past
the 2^32-word mark of the stream) and 16383 (the last, ~53 G doubles in: oracle.generate_steps
with the independent MT19937 jump-ahead of oracle.mt_jump);
sampled partial-C tiles of two slabs within 1e-12 max|C_g| of torch; C exactly symmetric;
all 16384 eigenvalues within 1e-12 lambda_0 of torch.linalg.eigh on the same C and T
sign-aligned within 1e-10 (gap rule); Phi of two slabs within 1e-10 of torch
A_c,g T Lambda^-1 / ns; the columns of the whole Phi (all slabs) of unit norm.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import pods_oracle as O  # noqa: E402

J, K, NS, SEED, WORLD = 1024, 1024, 16384, 2024, 8
CHECK_SLABS = (0, WORLD - 1)
LATE = (2047, NS - 1)        # stream offsets ~6.7 G and ~52.8 G doubles
FOURIER_MODES = 4            # the oracle DFT at ns = 16384: ~3 s per mode on the host


def snap_block(gen, i0, i1):
    import podsgen
    out = torch.empty((i1 - i0, gen.rowlen), dtype=torch.float64, device="cuda")
    podsgen.check(gen.ctx.lib.pods_copy_snapshots(gen.ctx.h, i0, i1, ctypes.c_void_p(out.data_ptr())),
                  "pods_copy_snapshots")
    return out


def slab_rows(gen):
    """Rows of the full reference A (3P, ns) that a slab's rows are (comp, j, k order)."""
    P = J * K
    return np.concatenate([np.arange(c * P + gen.j0 * K, c * P + gen.j1 * K) for c in range(3)])


@pytest.fixture(scope="module")
def c5():
    import bench
    import podsgen
    from podsgen import engine as E
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    s = bench.make_setup(podsgen, "c5", SEED)
    assert (s.jma, s.kma, s.ns) == (J, K, NS) and s.nfx == 12 and s.nfy == 6
    ctx = E.Context(0)
    lib = ctx.lib
    pack, unpack = E.device_triangle_ops(ctx)
    early, late, tiles, slabs = {}, {}, {}, []
    packed_sum = None
    for r in range(WORLD):
        gen = E.Generator(s, ctx=ctx, rank=r, world=WORLD)
        gen.generate()
        early[r] = snap_block(gen, 0, 2).cpu().numpy()
        late[r] = {i: snap_block(gen, i, i + 1)[0].cpu().numpy() for i in LATE}
        slabs.append((gen.j0, gen.j1))
        podsgen.check(lib.pods_mean(ctx.h, None, 0), "pods_mean")
        podsgen.check(lib.pods_center(ctx.h), "pods_center")
        Cg = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
        podsgen.check(lib.pods_corr(ctx.h, E.ptr(Cg), 0), "pods_corr")   # partial, not divided
        if r in CHECK_SLABS:
            out = []
            cmax = float(Cg.abs().max())
            for bi, bj in [(0, 0), (40, 3), (63, 62)]:
                X = snap_block(gen, bi * 256, (bi + 1) * 256)
                Y = snap_block(gen, bj * 256, (bj + 1) * 256)
                ref = X @ Y.T
                got = Cg[bi * 256:(bi + 1) * 256, bj * 256:(bj + 1) * 256]
                out.append(float((got - ref).abs().max()) / cmax)
                del X, Y
            tiles[r] = out
            assert torch.equal(Cg, Cg.T)
        p = pack(Cg)
        packed_sum = p if packed_sum is None else packed_sum + p   # the all-reduce's sum, rank order
        del Cg, p
    C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
    unpack(packed_sum, C)
    del packed_sum
    lam_desc, nvalid, nmt, T = E.eigen_modes(ctx, C, NS, s.nm, 1.0e-15, False)
    phis, sq = {}, torch.zeros(nmt, dtype=torch.float64, device="cuda")
    phi_ref = {}
    for r in range(WORLD):
        gen = E.Generator(s, ctx=ctx, rank=r, world=WORLD)
        gen.generate()
        podsgen.check(lib.pods_mean(ctx.h, None, 0), "pods_mean")
        podsgen.check(lib.pods_center(ctx.h), "pods_center")
        phi = torch.empty((gen.rowlen, nmt), dtype=torch.float64, device="cuda")
        podsgen.check(lib.pods_spatial_modes(ctx.h, E.ptr(T), T.shape[1], E.ptr(np.ascontiguousarray(lam_desc[:nmt])),
                                             nmt, E.ptr(phi)), "pods_spatial_modes")
        sq += (phi * phi).sum(0)
        if r in CHECK_SLABS:
            acc = torch.zeros_like(phi)
            for i0 in range(0, NS, 512):
                b = snap_block(gen, i0, i0 + 512)
                acc += b.T @ T[i0:i0 + 512, :nmt]
                del b
            lam = torch.from_numpy(np.ascontiguousarray(lam_desc[:nmt])).cuda()
            phi_ref[r] = (acc / lam[None, :] / NS).cpu()
            phis[r] = phi.cpu()
            del acc
        del phi
    fo = E.run_fourier(ctx, T, nmt, NS, s.dt_eff, s.et)
    torch.cuda.synchronize()
    yield dict(s=s, ctx=ctx, C=C, lam=lam_desc, nvalid=nvalid, nm=nmt, T=T, early=early, late=late, tiles=tiles,
               slabs=slabs, phis=phis, phi_ref=phi_ref, sq=sq.cpu().numpy(), fo=fo)
    ctx.close()


@pytest.mark.timeout(900)
def test_c5_generation_every_slab_bit_exact_early_steps(c5):
    import bench
    prf = bench.c5_profile(J, K)
    s = c5["s"]
    cfg = O.DFConfig(jma=J, kma=K, ns=NS, seed=SEED, dt=s.dt, prf=prf)
    assert (cfg.nfx, cfg.nfy, cfg.nfz) == (s.nfx, s.nfy, s.nfz)
    ref = O.generate_steps(cfg, [0, 1])
    P = J * K
    for r, (j0, j1) in enumerate(c5["slabs"]):
        rows = np.concatenate([np.arange(c * P + j0 * K, c * P + j1 * K) for c in range(3)])
        for i in (0, 1):
            got = c5["early"][r][i]
            assert np.array_equal(got, ref[i][rows]), (r, i)


@pytest.mark.timeout(900)
def test_c5_generation_every_slab_bit_exact_late_steps(c5):
    """Steps 2047 and 16383 -- stream offsets past the 2^32-word mark up to the end of C5's
    52.8 G-double stream (SURVEY Appendix A layout: 3 components interleaved per plane from plane
    2nfx+1 on), every slab's rows bit-exact.  The oracle reaches them by the MT19937 jump-ahead of
    oracle.mt_jump (pinned against numpy's sequential draws in test_oracle_golden.py)."""
    import bench
    prf = bench.c5_profile(J, K)
    s = c5["s"]
    cfg = O.DFConfig(jma=J, kma=K, ns=NS, seed=SEED, dt=s.dt, prf=prf)
    P = J * K
    for i in LATE:
        ref = O.generate_steps(cfg, [i], jump=True)[i]
        for r, (j0, j1) in enumerate(c5["slabs"]):
            rows = np.concatenate([np.arange(c * P + j0 * K, c * P + j1 * K) for c in range(3)])
            assert np.array_equal(c5["late"][r][i], ref[rows]), (r, i)
        del ref


@pytest.mark.timeout(900)
def test_c5_mt_state_exchange_every_slab_bit_exact(c5):
    """the 8-GPU generator of BASELINE config 5 (nfx = 12, nfy = nfz = 6,
    adapt2prf; a ~52.8 G-double stream) through the MT state exchange -- each rank twists only its
    1/8 of the stream and regenerates its own rows from the states the one all_to_all brings
    (emulated on this device and context: tests/exchange_emulation.py) -- equals the whole-stream
    slab generator, itself pinned to the oracle above, bit for bit at steps 0, 1, 2047 and 16383
    of every slab (digitalfilters.py:1361-1367, :1454-1467)."""
    from exchange_emulation import emulate_exchange
    s, ctx = c5["s"], c5["ctx"]
    seen = []

    def visit(q, g):
        assert (g.j0, g.j1) == c5["slabs"][q]
        got = snap_block(g, 0, 2).cpu().numpy()
        assert np.array_equal(got, c5["early"][q]), q
        for i in LATE:
            assert np.array_equal(snap_block(g, i, i + 1)[0].cpu().numpy(), c5["late"][q][i]), (q, i)
        seen.append(q)

    emulate_exchange(s, ctx, WORLD, visit)
    assert seen == list(range(WORLD))


@pytest.mark.timeout(900)
def test_c5_fourier_and_ranking(c5):
    """The DFT and ranking at ns = 16384 (PODFS.py:1560-1593) on C5's own temporal modes: c
    bit-exact against the oracle's reference expression for the first FOURIER_MODES modes, and
    c_count / c_ind / the FC rows of those modes exactly the oracle's."""
    s, fo = c5["s"], c5["fo"]
    k = min(FOURIER_MODES, c5["nm"])
    T = c5["T"].cpu().numpy()[:, :k]
    ref = O.fourier(T, NS, s.dt_eff, k, s.et)
    assert fo.period == ref["period"]
    assert np.array_equal(fo.c[:, :k], ref["c"]), int(np.sum(fo.c[:, :k] != ref["c"]))
    assert np.array_equal(fo.c_count[:k], ref["c_count"]), (fo.c_count[:k], ref["c_count"])
    assert np.array_equal(fo.c_ind[:k], ref["c_ind"])
    assert np.array_equal(fo.FC[:int(np.sum(fo.c_count[:k]))], ref["FC"])


def test_c5_partial_correlation_tiles(c5):
    for r, errs in c5["tiles"].items():
        assert max(errs) <= 1e-12, (r, errs)


@pytest.mark.timeout(900)
def test_c5_eigenvalues_and_temporal_modes(c5):
    C, lam_g, nm = c5["C"], c5["lam"], c5["nm"]
    assert torch.equal(C, C.T)
    lam_t, V = torch.linalg.eigh(C)
    lam = torch.flip(lam_t, (0,)).cpu().numpy()
    assert np.max(np.abs(lam_g - lam)) <= 1e-12 * lam[0]
    assert c5["nvalid"] == O.num_valid_modes(lam, NS) and nm == c5["s"].nm
    Vd = torch.flip(V, (1,))[:, :nm].cpu().numpy()
    T = c5["T"].cpu().numpy()[:, :nm]
    checked = 0
    for j in range(nm):
        v = Vd[:, j]
        Tref = v * np.sqrt(lam[j] / (np.sum(v * v) / NS))
        gap = min(abs(lam[j] - lam[j - 1]) if j else np.inf, abs(lam[j] - lam[j + 1]))
        if gap <= 1e-6 * lam[0]:
            continue
        sg = np.sign(np.dot(T[:, j], Tref))
        assert np.max(np.abs(sg * T[:, j] - Tref)) <= 1e-10 * np.max(np.abs(Tref)), j
        checked += 1
    assert checked >= nm // 2


def test_c5_spatial_modes(c5):
    for r in c5["phis"]:
        phi, ref = c5["phis"][r], c5["phi_ref"][r]
        for j in range(c5["nm"]):
            err = float((phi[:, j] - ref[:, j]).abs().max())
            assert err <= 1e-10 * float(ref[:, j].abs().max()), (r, j)
    # the whole field's modes (all 8 slabs) have unit 2-norm (PODFS.py:1330-1333)
    assert np.all(np.abs(np.sqrt(c5["sq"]) - 1.0) <= 1e-9), c5["sq"]

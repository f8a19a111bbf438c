"""GPU parity at BASELINE config 4's size on one device: 512 x 512 inlet x 8192 snapshots.

The production pipeline runs ONCE (module fixture): generation (6.76 G stream doubles), mean,
centring, the split-K SYRK at ns = 8192, the two-stage eigensolver pods_syev2 (the path every
ns > 4096 takes: PODFS.py:1309-1310), temporal scaling and the spatial modes.  Checked against
the oracle and fp64 torch without ever copying the 51.5 GB snapshot matrix whole:

  (i)   generation: steps 0, 1, 4095 and 8191 bit-exact against the oracle (one pass over the
        reference's draw stream, oracle.generate_steps), every sampled block finite; and the
        8-rank MT state exchange (the multi-GPU generator, emulated on this device) giving every
        slab's rows of those steps bit for bit (last test: it reconfigures the context);
  (ii)  the mean bit-exact against numpy's pairwise np.mean on 2048 sampled rows (the pairwise
        sum is per row, so a row sample is exact), and the centred rows == raw - mean;
  (iii) C exactly symmetric; sampled 256 x 256 tiles within 1e-12 max|C| of torch A_c^T A_c/ns;
  (iv)  all 8192 eigenvalues within 1e-12 lambda_0 of torch.linalg.eigh on the same C, T
        sign-aligned within 1e-10 of eigh's scaled vectors (modes with relative gap > 1e-6);
  (v)   Phi within 1e-10 (per mode) of torch's A_c T Lambda^-1 / ns, columns of unit norm;
  (vi)  the DFT and ranking at ns = 8192 (PODFS.py:1560-1593): c bit-exact against the oracle's
        reference expression for all nm modes, c_count / c_ind / FC exactly the oracle's.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import pods_oracle as O  # noqa: E402

J, K, NS, SEED = 512, 512, 8192, 4242
STEPS = [0, 1, NS // 2 - 1, NS - 1]   # stream offsets up to 6.76 G doubles (13.5 G words, past 2^32)
NROWS = 2048


def snap_block(gen, i0, i1):
    """Snapshots [i0, i1) as a (i1-i0, 3P) device tensor (pods_copy_snapshots)."""
    import podsgen
    out = torch.empty((i1 - i0, gen.rowlen), dtype=torch.float64, device="cuda")
    podsgen.check(gen.ctx.lib.pods_copy_snapshots(gen.ctx.h, i0, i1, ctypes.c_void_p(out.data_ptr())),
                  "pods_copy_snapshots")
    return out


def sample_rows(gen, rows, chunk=512):
    """A[rows, :] (the reference layout's rows) gathered chunk by chunk: (len(rows), ns) host."""
    out = np.empty((len(rows), NS))
    idx = torch.from_numpy(rows).cuda()
    for i0 in range(0, NS, chunk):
        b = snap_block(gen, i0, min(NS, i0 + chunk))
        out[:, i0:i0 + b.shape[0]] = b.index_select(1, idx).T.cpu().numpy()
        del b
    return out


@pytest.fixture(scope="module")
def c4():
    import podsgen
    from podsgen import engine as E
    assert torch.cuda.is_available(), "GPU tests need a ROCm device"
    s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=SEED)
    gen = E.Generator(s, device=0)
    snap = gen.generate()
    rows = np.sort(np.random.default_rng(5).choice(gen.rowlen, NROWS, replace=False))
    cols = {i: snap_block(gen, i, i + 1)[0].cpu().numpy() for i in STEPS}
    raw_rows = sample_rows(gen, rows)
    pod = E.run_pod(snap, s.nm, keep_C=True)
    # the default (int8) correlation subtracts the mean while forming its residues and leaves A as
    # generated; centre it in place now (pods_center, main() :1493-1495) for the checks below
    podsgen.check(gen.ctx.lib.pods_center(gen.ctx.h), "pods_center")
    torch.cuda.synchronize()
    cen_rows = sample_rows(gen, rows)
    fo = E.run_fourier(gen.ctx, pod.T, pod.nm, s.ns, s.dt_eff, s.et)
    yield dict(s=s, gen=gen, pod=pod, rows=rows, cols=cols, raw_rows=raw_rows, cen_rows=cen_rows, fo=fo)
    gen.ctx.close()


@pytest.mark.timeout(900)
def test_c4_generation_sampled_steps_bit_exact(c4):
    cfg = O.DFConfig(jma=J, kma=K, ns=NS, seed=SEED)
    ref = O.generate_steps(cfg, STEPS)
    for i in STEPS:
        bad = np.nonzero(c4["cols"][i] != ref[i])[0]
        assert bad.size == 0, (i, bad[:8])
    assert np.all(np.isfinite(c4["raw_rows"]))


@pytest.mark.timeout(600)
def test_c4_mean_and_centring_rows_bit_exact(c4):
    rows, raw = c4["rows"], c4["raw_rows"]
    mean_ref = np.mean(raw, 1)                                  # main() :1492, per row
    mean = c4["pod"].mean.cpu().numpy()[rows]
    assert np.array_equal(mean, mean_ref)
    assert np.array_equal(c4["cen_rows"], raw - mean[:, None])  # :1493-1495


@pytest.mark.timeout(600)
def test_c4_correlation_tiles(c4):
    C = c4["pod"].C
    assert torch.equal(C, C.T)
    cmax = float(C.abs().max())
    b = 256
    for bi, bj in [(0, 0), (1, 0), (13, 7), (31, 0), (31, 30), (31, 31)]:
        X = snap_block(c4["gen"], bi * b, (bi + 1) * b)
        Y = X if bj == bi else snap_block(c4["gen"], bj * b, (bj + 1) * b)
        ref = (X @ Y.T) / NS
        got = C[bi * b:(bi + 1) * b, bj * b:(bj + 1) * b]
        err = float((got - ref).abs().max())
        assert err <= 1e-12 * cmax, (bi, bj, err / cmax)
        del X, Y


@pytest.mark.timeout(600)
def test_c4_eigen_two_stage_vs_eigh(c4):
    pod, s = c4["pod"], c4["s"]
    lam_t, V = torch.linalg.eigh(pod.C)
    lam = torch.flip(lam_t, (0,)).cpu().numpy()
    assert np.max(np.abs(pod.energy - lam)) <= 1e-12 * lam[0]
    assert pod.num_valid == O.num_valid_modes(lam, NS) and pod.nm == s.nm
    nm = pod.nm
    Vd = torch.flip(V, (1,))[:, :nm].cpu().numpy()
    T = pod.T.cpu().numpy()[:, :nm]
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


@pytest.mark.timeout(900)
def test_c4_spatial_modes(c4):
    pod, gen = c4["pod"], c4["gen"]
    nm = pod.nm
    T = pod.T[:, :nm]
    lam = torch.from_numpy(np.ascontiguousarray(pod.energy[:nm])).cuda()
    acc = torch.zeros((gen.rowlen, nm), dtype=torch.float64, device="cuda")
    for i0 in range(0, NS, 512):                   # A_c T, snapshot block by block
        b = snap_block(gen, i0, i0 + 512)
        acc += b.T @ T[i0:i0 + 512]
        del b
    ref = acc / lam[None, :] / NS                  # PODFS.py:1330-1333
    phi = pod.phi
    for j in range(nm):
        err = float((phi[:, j] - ref[:, j]).abs().max())
        assert err <= 1e-10 * float(ref[:, j].abs().max()), j
    norms = torch.linalg.vector_norm(phi, dim=0).cpu().numpy()
    assert np.all(np.abs(norms - 1.0) <= 1e-9), norms


@pytest.mark.timeout(900)
def test_c4_fourier_and_ranking(c4):
    """PODFS.py:1560-1593 at ns = 8192 on C4's temporal modes: every coefficient bit-equal to the
    oracle's reference expression (the device multiplies by the host's np.exp twiddles in numpy's
    pairwise order), so c_count / c_ind / FC are the oracle's for every mode; the GPU ranking
    kernel equals the host restatement on the same c."""
    from podsgen import engine as E
    pod, fo, s = c4["pod"], c4["fo"], c4["s"]
    T = pod.T.cpu().numpy()
    ref = O.fourier(T, NS, s.dt_eff, pod.nm, s.et)
    assert fo.period == ref["period"]
    assert np.array_equal(fo.c, ref["c"]), int(np.sum(fo.c != ref["c"]))
    assert np.array_equal(fo.c_count, ref["c_count"]), (fo.c_count, ref["c_count"])
    assert np.array_equal(fo.c_ind, ref["c_ind"])
    assert np.array_equal(fo.FC, ref["FC"])
    c_ind, c_count, FC = E.host_rank_and_count(fo.c, s.et)
    assert np.array_equal(fo.c_count, c_count) and np.array_equal(fo.c_ind, c_ind)


@pytest.mark.timeout(900)
def test_c4_mt_state_exchange_world8_bit_exact(c4):
    """BASELINE config 4's 8-GPU generator -- each rank twists only its 1/8 of the
    MT19937 stream, records every rank's segment-start states, one all_to_all (emulated on this
    device: tests/exchange_emulation.py) and each rank regenerates its own rows -- at C4's full
    shape, whose 6.76 G-double stream passes 2^32 words: every slab's rows at steps 0, 1, 4095 and
    8191 equal the one-device generation's (pinned to the oracle above) bit for bit
    (digitalfilters.py:1361-1367, :1454-1467).  Runs last: it reconfigures the module's context."""
    from exchange_emulation import emulate_exchange
    s, ctx = c4["s"], c4["gen"].ctx
    P = J * K
    seen = []

    def visit(q, g):
        rows = np.concatenate([np.arange(c * P + g.j0 * K, c * P + g.j1 * K) for c in range(3)])
        for i in STEPS:
            got = snap_block(g, i, i + 1)[0].cpu().numpy()
            bad = np.nonzero(got != c4["cols"][i][rows])[0]
            assert bad.size == 0, (q, i, bad[:8])
        seen.append((g.j0, g.j1))

    emulate_exchange(s, ctx, 8, visit)
    assert [a for a, _ in seen] == [64 * q for q in range(8)] and seen[-1][1] == J

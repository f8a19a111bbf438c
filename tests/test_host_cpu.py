"""CPU tests: host-side setup vs the oracle, library symbols, MT jump math, formats,
CLI, HDF5 layout, and the multi-rank decomposition with gloo (world size 2)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from oracle import pods_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from podsgen import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    hdr = open(os.path.join(ROOT, "include", "podsgen.h")).read()
    names = set(re.findall(r"^\s*(?:int|const char\*)\s+(pods_\w+)\s*\(", hdr, re.M))
    assert len(names) >= 20
    for n in sorted(names):
        assert hasattr(lib, n), n
        assert n in _lib.SIGNATURES, n
    assert _lib.load().pods_abi_version() == 1


DIAG_SWITCHES = ("PODS_SYRK_I8", "PODS_RES_I8", "PODS_CORR_ORDER", "PODS_SYRK_WIDE", "PODS_SYRK_LEAD",
                 "PODS_SYRK_PACE", "PODS_X_NT", "PODS_MEAN", "PODS_CHASE_P")


def test_product_library_has_no_variant_switches():
    """the measurement-only variants (wrong results: PODS_SYRK_I8=9*, the residue
    pass without loads or stores, every item on one tile) and the A/B variants measured equal or
    slower are not in libpodsgen.so -- the product library never reads those switches (no getenv
    of their names: the names are not even in its string table), so setting them cannot change a
    result.  The grid SYRK and its measurement variants build only into the diagnostic library
    (`make -C pods-digital-filter_amd/csrc diag`, -DPODS_DIAG)."""
    from podsgen import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    for name in DIAG_SWITCHES:
        assert name.encode() + b"\0" not in blob, name
    # the switches that select correct alternatives stay (fp64 SYRK, residue budget, K splits)
    for name in ("PODS_CORR", "PODS_CORR_BUDGET_GB", "PODS_CORR_SPLITS"):
        assert name.encode() + b"\0" in blob, name


def test_persistent_grid_rule():
    """The co-residency rule every spin-waiting launch passes first (pods::check_persistent):
    a grid larger than blocks-per-CU x CUs is refused with PODS_ERR_UNSUPPORTED."""
    from podsgen import _lib
    lib = _lib.load()
    assert lib.pods_host_persistent_grid_fits(1, 256, 256) == 0
    assert lib.pods_host_persistent_grid_fits(2, 256, 512) == 0
    assert lib.pods_host_persistent_grid_fits(1, 256, 257) == -6
    assert b"257" in lib.pods_last_error()
    assert lib.pods_host_persistent_grid_fits(0, 256, 1) == -6   # kernel cannot run at all
    assert lib.pods_host_persistent_grid_fits(1, 224, 256) == -6  # CU-masked / partitioned device
    assert lib.pods_host_persistent_grid_fits(-1, 256, 1) == -1


def _i8_plan(ns, rowlen, budget, force=0):
    from podsgen import _lib
    lib = _lib.load()
    out = np.zeros(8, dtype=np.int64)
    rowpad = (rowlen + 15) // 16 * 16
    rc = lib.pods_corr_i8_plan_query(ns, rowlen, rowpad, int(budget), force, out.ctypes.data)
    return rc, dict(zip(("bbits", "nlaunch", "nsplit", "kcs", "chunks", "r_bytes", "p_bytes", "mod_bytes"),
                        (int(v) for v in out)))


@pytest.mark.parametrize("ns,rowlen", [(4096, 196608), (8192, 786432), (2048, 3145728), (16384, 393216),
                                       (72, 140000), (4096, 24576)])
@pytest.mark.parametrize("budget_gib", [0.0001, 16, 64, 200])
def test_corr_i8_plan_offsets_fit_32_bits(ns, rowlen, budget_gib):
    """k_residues addresses one modulus' residues with 32-bit offsets, so no
    launch may hold 2^32 bytes per modulus, whatever PODS_CORR_BUDGET_GB says (a 64 GiB budget
    used to wrap them); the launches cover every K chunk and the plan keeps b = 52 up to C4's K."""
    rc, p = _i8_plan(ns, rowlen, budget_gib * 2 ** 30)
    assert rc == 0, p
    assert p["mod_bytes"] == p["chunks"] * ns * 64 < 2 ** 32
    assert p["nlaunch"] * p["chunks"] >= -(-rowlen // 64)
    assert p["r_bytes"] == 16 * p["mod_bytes"]
    assert 1 <= p["nsplit"] <= 8 and p["nsplit"] * p["kcs"] == p["chunks"]
    if rowlen <= 786432:
        assert p["bbits"] == 52


@pytest.mark.parametrize("force", [1, 3, 8, 9, 300, 100000])
def test_corr_i8_plan_forced_splits_capped(force):
    """a forced split count is capped at 8 (k_crt sums the splits' bytes in
    16-bit fields; 258 or more used to overflow them)."""
    rc, p = _i8_plan(4096, 196608, 16 * 2 ** 30, force)
    assert rc == 0 and p["nsplit"] == min(force, 8)


@pytest.mark.parametrize("ns,dt", [(4096, 0.1), (520, 0.037), (17, 0.05), (64, 0.1), (5, 0.1), (2, 0.3),
                                   (8192, 0.0731)])
def test_dft_twiddles_are_the_reference_expression(ns, dt):
    """podsgen.host.dft_twiddles (the table the GPU DFT multiplies by) equals the reference's
    np.exp(-1j*2*k*np.pi*time/period) (PODFS.py:1566) bit for bit, row by row, and the rows it
    omits (k < 0 except -ns/2) are exact conjugates of stored ones (the kernel writes
    c[h-k] = conj(c[h+k]))."""
    from podsgen.host import dft_rows, dft_twiddles, time_axis
    time_, period = time_axis(ns, dt)
    W = dft_twiddles(ns, time_, period, chunk=7)
    ks = dft_rows(ns)
    assert W.shape == (len(ks), ns, 2)
    pick = range(len(ks)) if ns <= 520 else list(range(0, len(ks), 97)) + [len(ks) - 2, len(ks) - 1]
    for q in pick:
        k = ks[q]
        e = np.exp(-1j * 2 * k * np.pi * time_ / period)
        assert np.array_equal(W[q, :, 0].view(np.uint64), e.real.view(np.uint64)), (ns, k)
        assert np.array_equal(W[q, :, 1].view(np.uint64), e.imag.view(np.uint64)), (ns, k)
        if 0 < k:
            en = np.exp(-1j * 2 * (-k) * np.pi * time_ / period)
            assert np.array_equal(en.real, e.real) and np.array_equal(en.imag, -e.imag), (ns, k)


@pytest.mark.parametrize("seed,nblocks", [(0, 2), (12345, 3), (7, 1000), (2 ** 32 - 1, 65537)])
def test_host_mt_jump_math(seed, nblocks):
    from podsgen import _lib
    lib = _lib.load()
    assert lib.pods_host_mt_charpoly_degree() == 19937
    assert lib.pods_host_mt_jump_check(seed, nblocks) == 0, lib.pods_last_error()


@pytest.mark.parametrize("kw", [dict(jma=12, kma=9, ns=17, seed=3, dt=0.05),
                                dict(jma=10, kma=11, ns=5, seed=7),
                                dict(jma=6, kma=7, ns=6, seed=5, normal=(1.0, 1.0, 0.5)),
                                dict(jma=9, kma=12, ns=7, seed=21, mean_profile="double-hyperbolic-tangent"),
                                dict(jma=11, kma=10, ns=6, seed=22, mean_profile="circular-hyperbolic-tangent"),
                                dict(jma=12, kma=13, ns=6, seed=23, mean_profile="ring-hyperbolic-tangent",
                                     inner_d=0.3),
                                dict(jma=31, kma=40, ns=6, seed=2, mean_profile="circular-hyperbolic-tangent"),
                                dict(jma=64, kma=33, ns=6, seed=2, mean_profile="ring-hyperbolic-tangent")])
def test_setup_matches_oracle(kw):
    import podsgen
    s = podsgen.DFSetup(**kw)
    c = O.DFConfig(**kw)
    assert (s.nfx, s.nfy, s.nfz) == (c.nfx, c.nfy, c.nfz)
    assert s.dt_eff == c.dt_eff and s.lnx == c.lnx
    for a, b in zip(s.taps(), (O.calccoeff(c.nfx, c.lnx), O.calccoeff(c.nfy, c.lny), O.calccoeff(c.nfz, c.lnz))):
        assert np.array_equal(a, b)
    assert np.array_equal(s.lund_rows(), O.lund_point_coeffs(c))
    assert np.array_equal(s.rotation(), O.rotation_matrix(*c.n_unit))


@pytest.mark.parametrize("tag", ["dtanh", "circ", "circ_odd", "ring", "ring_thin"])
def test_adapt2d_host_factor_matches_oracle_loop(golden_dir, tag):
    """podsgen.profiles2d (vectorised, once per run) == the reference's per-point loop."""
    from podsgen.profiles2d import adapt2d_factor
    g = np.load(os.path.join(golden_dir, "unit_adapt2d.npz"))
    J, K, inner = g[tag + "_cfg"]
    name, prof = str(g[tag + "_name"]), g[tag + "_prof"]
    fac = adapt2d_factor(name, float(inner), *prof, int(J), int(K))
    co, um = O.adapt2d_point_coeffs(name, float(inner), *prof, int(J), int(K))
    for a, b in zip(fac, tuple(co) + (um,)):
        assert np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("tag,mdot,den,bulk", [("plain", 0.0, 0.0, 1.0), ("bulk", 0.0, 0.0, 2.5),
                                              ("mdot", 0.7, 1.2, 1.0)])
def test_read_prf_matches_reference(golden_dir, tmp_path, tag, mdot, den, bulk):
    """read_prf (digitalfilters.py:524-1035) on a synthetic CFD plane == the reference's
    output (griddata, gradients, eddy-viscosity stresses, rescaling), bit for bit."""
    from podsgen.prf import read_prf
    g = np.load(os.path.join(golden_dir, "unit_read_prf.npz"))
    path = tmp_path / "inlet.prf"
    path.write_text(str(g["prf_text"]))
    res = read_prf(str(path), 0.1, mdot, den, bulk, False, False)
    for name, v in zip(("U", "V", "W", "uu", "vv", "ww", "uv", "uw", "vw"), res[:9]):
        assert np.array_equal(np.asarray(v), g["%s_%s" % (tag, name)]), name
    assert np.array_equal(np.array([float(x) for x in res[9:]]), g[tag + "_scalars"])


def test_lund_rows_slab():
    import podsgen
    s = podsgen.DFSetup(jma=9, kma=5, ns=3)
    full = s.lund_rows()
    parts = [s.lund_rows(*podsgen.row_slab(9, r, 4)) for r in range(4)]
    assert np.array_equal(np.concatenate([p.reshape(9, -1, 5) for p in parts], axis=1).reshape(9, -1), full)


@pytest.mark.parametrize("J,world", [(256, 1), (256, 8), (10, 3), (7, 7), (512, 8)])
def test_row_slab_partition(J, world):
    import podsgen
    slabs = [podsgen.row_slab(J, r, world) for r in range(world)]
    assert slabs[0][0] == 0 and slabs[-1][1] == J
    assert all(a[1] == b[0] for a, b in zip(slabs, slabs[1:]))
    assert max(b - a for a, b in slabs) - min(b - a for a, b in slabs) <= 1


def test_rank_and_count_matches_oracle():
    import podsgen
    rng = np.random.default_rng(1)
    for ns in (5, 64, 257):
        c = (rng.standard_normal(ns) + 1j * rng.standard_normal(ns)).astype(np.complex64)
        c[ns // 2 + 1:] = np.conj(c[1:ns - ns // 2][::-1])[:len(c[ns // 2 + 1:])]  # conjugate ties
        for et in (0.5, 0.9, 0.99):
            a, n = podsgen.rank_and_count(c, et)
            b, m = O.rank_and_count(c, et)
            assert np.array_equal(a, b) and n == m


def test_num_valid_modes_closed_form():
    import podsgen
    rng = np.random.default_rng(2)
    for ns in (3, 4, 5, 17, 64):
        for _ in range(20):
            lam = np.sort(rng.standard_normal(ns) * 10 ** rng.uniform(-40, 0, ns))[::-1]
            lam[0] = abs(lam[0]) + 1.0
            assert podsgen.num_valid_modes(lam, ns) == O.num_valid_modes(lam, ns)


def test_text_formats_match_oracle(golden_dir):
    import PODFS
    g = np.load(os.path.join(golden_dir, "cli_10x11x5.npz"))
    # PODFS.dat writer on the golden coefficients reproduces the reference's file
    Ac = g["A_raw"] - g["mean_field"][:, None]
    res = O.pod(Ac, 5, 20)
    fo = O.fourier(res["T"], 5, float(g["dt"]), res["nm"], 0.9)
    assert PODFS.podfs_dat_text(res["nm"], fo["period"], fo["c"], fo["c_ind"], fo["c_count"], 5) == str(g["podfs_dat"])


def test_eigenvalue_file_writer(golden_dir, tmp_path):
    import PODFS
    g = np.load(os.path.join(golden_dir, "c1_32x32x64.npz"))
    fn = str(tmp_path / "POD.eigenvalues.dat")
    PODFS.write_eigenvalues(int(g["num_valid_modes"]), 64, g["energy"].real, fn)
    assert open(fn).read() == str(g["eigenvalues_dat"])


def test_read_profile_dropin_matches_reference(golden_dir, tmp_path):
    """digitalfilters.read_profile (drop-in) == the reference's read_profile (:487-522)."""
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "unit_read_profile.npz"))
    path = tmp_path / "profile.dat"
    path.write_text(str(g["text"]))
    for kma in (17, 32, 64):
        assert np.array_equal(np.stack(df.read_profile(str(path), kma)), g["k%d" % kma]), kma


def test_profile_file_setup_matches_oracle(golden_dir, tmp_path):
    """-i profile.dat: the drop-in CLI setup reads the profile, clamps the stresses and skips
    the rotation (:1306-1307, :1344-1350, :1476) exactly as the pinned oracle config does."""
    import digitalfilters as df
    from test_oracle_golden import cfg_from
    g = np.load(os.path.join(golden_dir, "prof1d_14x16x8.npz"))
    path = tmp_path / "profile.dat"
    path.write_text(str(g["cfg_profile_text"]))
    opts = df.make_parser().parse_args(["-j", "14", "-k", "16", "-n", "8", "--seed", "41", "-i", str(path),
                                        "--nx", "1.0", "--ny", "0.3"])[0]
    s = df.setup_from_options(opts)
    cfg = cfg_from(g)
    assert not s.rotated and not cfg.rotated
    assert s.dt_eff == cfg.dt_eff == float(g["dt"])
    for key in ("U", "uu", "vv", "ww", "uw"):
        assert np.array_equal(s.profile[key], cfg.profile[key]), key


def test_save_plane_matches_reference(golden_dir, tmp_path, monkeypatch):
    """save_plane (verbose per-step snapshot .prf, PODFS.py:854-887): file name and text equal
    to the reference's for three planes (default normal, a translation, a tilted plane)."""
    import types
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "unit_save_plane.npz"))
    monkeypatch.chdir(tmp_path)
    for c in range(3):
        i_d = types.SimpleNamespace()
        i_d.grid = types.SimpleNamespace(points=g["plane%d_points" % c])
        i_d.n = [np.float64(v) for v in g["plane%d_n" % c]]
        i_d.t_o = [float(v) for v in g["plane%d_t_o" % c]]
        i_d.time = float(g["plane%d_time" % c])
        df.save_plane(g["plane%d_u" % c], i_d)
        name = str(g["plane%d_name" % c])
        assert os.path.exists(os.path.join("PODFS", name)), name
        assert open(os.path.join("PODFS", name)).read() == str(g["plane%d_text" % c])


def test_sort_eigenvalues_semantics():
    import PODFS
    energy = np.array([1.0, 3.0, np.nan, 3.0, -2.0])
    T = np.arange(25, dtype=np.float64).reshape(5, 5)
    e2, T2 = O.sort_eigen(energy.astype(complex), T.astype(complex))
    PODFS.sort_eigenvalues(5, energy, T)
    assert np.array_equal(energy, e2) and np.array_equal(T, T2)


def test_prf_geometry_doc_row_and_sizes():
    import PODFS
    import nsigproclib as sp
    pts = PODFS.cell_centres(10, 11, 0.1)
    assert pts.shape == (110, 3)
    assert ",".join(sp.str(v) for v in pts[0]) == "0.000000000000,-0.500000000000,0.550000011921"
    assert np.all(pts[:, 0] == 0.0)
    assert np.allclose(pts[-1, 1:], [0.5, -0.55], atol=1e-7)


def test_cli_options_and_aliases():
    import digitalfilters as df
    p = df.make_parser()
    o, _ = p.parse_args(["-j", "8", "-k", "9", "--num_steps", "7", "--udash", "0.05", "--filter_width", "3",
                         "--num_modes", "4", "--seed", "11", "-5"])
    assert (o.jma, o.kma, o.nsteps, o.turbulence_intensity, o.fwidth, o.nm, o.seed, o.hdf5) == \
        (8, 9, 7, 0.05, 3.0, 4, 11, True)
    s = df.setup_from_options(o)
    assert s.nfx == int(np.ceil(3.0 * 3.0)) and s.seed == 11


def _h5py_python():
    import HDF5
    return HDF5._h5py_python()


@pytest.mark.skipif(_h5py_python() is None, reason="no interpreter with h5py")
def test_hdf5_layout(tmp_path):
    import HDF5

    class I:
        pass
    i_d = I()
    i_d.nm, i_d.period, i_d.num_points = 2, 0.5, 3
    i_d.N_FC = np.array([2, 1])
    i_d.FC = np.arange(9, dtype=np.float64).reshape(3, 3)
    i_d.mean = np.arange(18, dtype=np.float64).reshape(3, 6)
    i_d.modes = np.arange(36, dtype=np.float64).reshape(2, 3, 6) * 0.5
    fn = str(tmp_path / "PODFS.hdf5")
    HDF5.write_HDF5(i_d, fn)
    reader = ("import h5py, numpy as np, sys\n"
              "f = h5py.File(sys.argv[1], 'r'); m = f['main']\n"
              "print(int(m.attrs['N_POD']), float(m.attrs['period']), list(m['N_FC'][:]), list(m['FC'][:]))\n"
              "print(list(m['mean'][:]), m['mean'].attrs['Np'], m['mean'].attrs['Nvar'], m['mean'].attrs['Vars'], list(m['mean'].attrs['SF']))\n"
              "print(sorted(m['modes'].keys()), list(m['modes/mode_0002'][:4]))\n")
    out = subprocess.run([_h5py_python(), "-c", reader, fn], capture_output=True, text=True).stdout.splitlines()
    assert out[0] == "2 0.5 [2, 1] %s" % [float(v) for v in i_d.FC.reshape(-1, order="F")]
    assert out[1].startswith(str([float(v) for v in i_d.mean.reshape(-1, order="F")]))
    assert "3 6 b'x,y,z,u,v,w,dummy' [1.0, 1.0, 1.0, 1.0, 1.0, 1.0]" in out[1]
    assert out[2].startswith("['mode_0001', 'mode_0002']")


def test_mode_stack_matches_reference_fill():
    """PODFS.ModeStack gives the array the reference fills (PODFS.py:1671-1672, :1745-1747)."""
    import PODFS
    rng = np.random.default_rng(2)
    P, nm = 7, 3
    points = rng.standard_normal((P, 3))
    spatial = rng.standard_normal((3 * P, nm))
    want = np.zeros((nm, P, 6))
    for i in range(nm):
        want[i, :, 0:3] = points
        want[i, :, 3:] = spatial[:, i].reshape((P, 3), order="F")
    st = PODFS.ModeStack(points, spatial, nm)
    assert len(st) == nm and st.shape == want.shape
    for i in range(nm):
        assert np.array_equal(st[i], want[i])
    assert np.array_equal(st[-1], want[-1]) and np.array_equal(np.asarray(st), want)
    with pytest.raises(IndexError):
        st[nm]


@pytest.mark.skipif(_h5py_python() is None, reason="no interpreter with h5py")
def test_hdf5_streamed_modes_identical(tmp_path):
    """The writer fed a ModeStack (modes rebuilt per mode from points + spatial modes) writes the
    same datasets as from the materialised (nm, P, 6) array."""
    import HDF5
    import PODFS
    rng = np.random.default_rng(4)
    P, nm = 11, 3
    points = rng.standard_normal((P, 3))
    spatial = rng.standard_normal((3 * P, nm))

    class I:
        pass
    files = []
    for lazy in (True, False):
        i_d = I()
        i_d.nm, i_d.period, i_d.num_points = nm, 0.25, P
        i_d.N_FC = np.array([1, 2, 1])
        i_d.FC = rng.standard_normal((4, 3)) if lazy else files_fc
        files_fc = i_d.FC
        i_d.mean = np.arange(6 * P, dtype=np.float64).reshape(P, 6)
        st = PODFS.ModeStack(points, spatial, nm)
        i_d.modes = st if lazy else np.asarray(st)
        fn = str(tmp_path / ("lazy.h5" if lazy else "full.h5"))
        HDF5.write_HDF5(i_d, fn)
        files.append(fn)
    reader = ("import h5py, numpy as np, sys\n"
              "a, b = (h5py.File(x, 'r')['main'] for x in sys.argv[1:3])\n"
              "ok = all(np.array_equal(a['modes'][k][:], b['modes'][k][:]) for k in b['modes'])\n"
              "ok = ok and sorted(a['modes']) == sorted(b['modes']) and np.array_equal(a['FC'][:], b['FC'][:])\n"
              "print('same' if ok else 'differ', len(a['modes']))\n")
    out = subprocess.run([_h5py_python(), "-c", reader] + files, capture_output=True, text=True)
    assert out.stdout.split() == ["same", str(nm)], out.stderr


def _c5_hdf5_worker(rank, world, port, fn, out):
    """One rank of the streamed multi-rank HDF5 write at C5 size: rank 0 writes through a
    ModeStack over digitalfilters.SlabColumns, the others serve their row slabs per mode."""
    import hashlib
    import types
    import torch.distributed as dist
    import HDF5
    import PODFS
    import digitalfilters as df
    import podsgen
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    J = K = 1024
    nm, P = 4, 1024 * 1024
    s = types.SimpleNamespace(jma=J, kma=K, P=P)
    rng = np.random.default_rng(123)
    spatial = rng.standard_normal((3 * P, nm))    # the whole inlet's modes, sliced per rank
    j0, j1 = podsgen.row_slab(J, rank, world)
    rows = np.concatenate([np.arange(c * P + j0 * K, c * P + j1 * K) for c in range(3)])
    local = spatial[rows]
    if rank == 0:
        points = rng.standard_normal((P, 3))
        cols = df.SlabColumns(dist, s, local)
        i_d = types.SimpleNamespace(nm=nm, period=0.5, num_points=P, N_FC=np.array([2, 1, 1, 1]),
                                    FC=np.arange(15, dtype=np.float64).reshape(5, 3),
                                    mean=np.zeros((P, 6)), modes=PODFS.ModeStack(points, cols, nm))
        try:
            HDF5.write_HDF5(i_d, fn)
        finally:
            cols.close()
        want = []
        for i in range(nm):
            m = np.empty((P, 6))
            m[:, 0:3] = points
            m[:, 3:] = spatial[:, i].reshape((P, 3), order="F")
            want.append(hashlib.sha1(m.reshape(P * 6, order="F").tobytes()).hexdigest())
        out[0] = want
    else:
        df.serve_slab_columns(dist, s, local)
    dist.destroy_process_group()


@pytest.mark.skipif(_h5py_python() is None, reason="no interpreter with h5py")
def test_hdf5_c5_size_streamed_two_ranks(tmp_path):
    """BASELINE config 5's streamed HDF5 write at its size (1024 x 1024 inlet, 4 modes of 6 x 1 M
    doubles, 0.2 GB), from two ranks holding row slabs: every mode dataset equals the mode built
    from the whole array (SHA-1 of its bytes), and rank 0 only ever held one mode."""
    import multiprocessing as mp
    fn = str(tmp_path / "PODFS_c5.hdf5")
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    port = 29900 + os.getpid() % 90
    procs = [ctx.Process(target=_c5_hdf5_worker, args=(r, 2, port, fn, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0
    reader = ("import h5py, hashlib, numpy as np, sys\n"
              "f = h5py.File(sys.argv[1], 'r')['main']\n"
              "print(' '.join(hashlib.sha1(f['modes'][k][:].tobytes()).hexdigest() for k in sorted(f['modes'])))\n"
              "print(f['mean'].attrs['Np'], f.attrs['N_POD'])\n")
    r = subprocess.run([_h5py_python(), "-c", reader, fn], capture_output=True, text=True)
    lines = r.stdout.split("\n")
    assert lines[0].split() == list(out[0]), r.stderr
    assert lines[1].split() == [str(1024 * 1024), "4"]


def _gloo_worker(rank, world, port, A, out):
    """One rank of the product's multi-GPU host path on gloo/CPU tensors:
    engine.allreduce_correlation (packed lower-triangle all-reduce, divide, mirror) and
    digitalfilters.gather_row_slabs (row slabs -> rank 0), on the rows host.row_slab gives it."""
    import torch
    import torch.distributed as dist
    import podsgen
    import digitalfilters as df
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    J, K, ns = 13, 5, 9
    j0, j1 = podsgen.row_slab(J, rank, world)
    P = J * K
    rows = np.concatenate([np.arange(c * P + j0 * K, c * P + j1 * K) for c in range(3)])
    Al = A[rows]
    mean = np.mean(Al, 1)
    Ac = Al - mean[:, None]
    C = torch.from_numpy(np.dot(Ac.T, Ac))
    r_, c_ = torch.tril_indices(ns, ns)   # CPU stand-ins for pods_pack_lower / pods_unpack_lower

    def pack(M):
        return M[r_, c_].clone()

    def unpack(packed, M):
        x = torch.from_numpy(packed.numpy() / ns)
        M[r_, c_] = x
        M[c_, r_] = x
    E.allreduce_correlation(dist, C, ns, pack, unpack)
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=1)
    full = df.gather_row_slabs(dist, s, np.concatenate([mean[:, None], Ac], axis=1))
    out[rank] = (C.numpy().tobytes(), None if full is None else full.tobytes())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_multirank_correlation_and_gather(world):
    """The multi-GPU decomposition through the product's host code (gloo transport, world 2
    and 3 with unequal slabs): partial A_g^T A_g, the packed lower-triangle all-reduce, the
    divide by ns, the mirror (C exactly symmetric), and the slab gather to rank 0."""
    import multiprocessing as mp
    rng = np.random.default_rng(0)
    J, K, ns = 13, 5, 9
    A = rng.standard_normal((3 * J * K, ns)) + 1.0
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29500 + (os.getpid() + 17 * world) % 1000
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, A, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    mean = np.mean(A, 1)
    Ac = A - mean[:, None]
    ref = np.dot(Ac.T, Ac) / ns
    for r in range(world):
        C = np.frombuffer(out[r][0]).reshape(ns, ns)
        assert np.array_equal(C, C.T)
        assert np.max(np.abs(C - ref)) <= 1e-13 * np.max(np.abs(ref))
        assert (out[r][1] is None) == (r != 0)
    full = np.frombuffer(out[0][1]).reshape(3 * J * K, ns + 1)
    assert np.array_equal(full[:, 0], mean)
    assert np.array_equal(full[:, 1:], Ac)


def test_num_valid_modes_vectorised_matches_reference_loop():
    """host.num_valid_modes (vectorised, on the step's critical path) against the literal
    PODFS.py:1312-1317 loop: sorted/unsorted spectra, zeros, negatives, energy[0] = 0,
    every ns parity, three tolerances."""
    import warnings
    from podsgen.host import num_valid_modes, num_valid_modes_loop
    rng = np.random.default_rng(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for ns in list(range(1, 12)) + [50, 51, 4096, 4097]:
            for trial in range(120 if ns < 60 else 10):
                e = np.sort(rng.standard_normal(ns) * 10.0 ** rng.uniform(-20, 3, ns))[::-1].copy()
                if trial % 5 == 0:
                    e = np.abs(e)
                if trial % 7 == 0 and ns > 3:
                    e[rng.integers(ns)] = 0.0
                if trial % 11 == 0:
                    e[0] = 0.0
                if trial % 13 == 0:
                    e = np.abs(rng.standard_normal(ns))
                for tol in (1e-15, 1e-3, 0.5):
                    assert num_valid_modes(e, ns, tol) == num_valid_modes_loop(e, ns, tol), (ns, tol, trial)


@pytest.mark.parametrize("ns", [4096, 8192, 16384])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_spectrum_queue_ownership(world, ns):
    """SpectrumQueue's owner sequence (host logic, no device): identical on every rank, shares
    of the spectra proportional to the per-step budgets, rank 0 (which carries the leading-pair
    solve) owning less than the others and none at world 8 (C3 costs).  ns = 8192 / 16384
    (BASELINE configs 4 / 5): the two-stage solver's units (17 / 33: stage-1 panel groups, chase
    ranges, the bisection) are spread the same way -- no owner solves a whole step at once."""
    from podsgen import engine as E

    class _Ctx:
        lib = None

    qs = [E.SpectrumQueue(_Ctx(), ns, r, world) for r in range(world)]
    seq = [qs[0].owner(s) for s in range(400)]
    for q in qs[1:]:
        assert [q.owner(s) for s in range(400)] == seq
    b = qs[0].budgets
    if ns == 4096:
        assert abs(sum(b) - sum(E.SpectrumQueue.UNIT_MS)) < 1e-9
    else:
        assert qs[0].units == {8192: 17, 16384: 33}[ns]
        assert abs(sum(b) - sum(qs[0].cost)) < 1e-9
        # the largest unit is a small share of one spectrum: units interleave with steps
        assert max(qs[0].cost) < 0.2 * sum(qs[0].cost)
    counts = np.bincount(seq, minlength=world)
    for r in range(world):
        assert abs(counts[r] / 400 - b[r] / sum(b)) <= 0.01, (r, counts, b)
    if world > 1:
        assert b[0] < b[1]
    if world == 8 and ns == 4096:
        assert counts[0] == 0

"""The oracle is pinned against fixtures produced by the reference's own code
(tests/golden/make_golden.py).  Everything here is bit-exact unless stated."""
import os

import numpy as np
import pytest

from oracle import pods_oracle as O

CASES = ["c1_32x32x64", "cli_10x11x5", "odd_12x9x17_aniso", "prf_8x12x9", "rot_6x7x6",
         "dtanh_9x12x7", "circ_11x10x6", "ring_12x13x6", "readprf_case", "prof1d_14x16x8"]
UNIT_2D = ["dtanh", "circ", "circ_odd", "ring", "ring_thin"]


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name + ".npz"))


def cfg_from(g):
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
        kw["profile1d"] = profile1d_from_text(str(g["cfg_profile_text"]), kw["kma"])
    return O.DFConfig(**kw)


def profile1d_from_text(text, kma):
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "profile.dat")
        with open(path, "w") as f:
            f.write(text)
        U, uu, vv, ww, uw = O.read_profile(path, kma)
    return dict(U=U, uu=uu, vv=vv, ww=ww, uw=uw)


def test_read_profile_matches_reference(golden_dir, tmp_path):
    """read_profile (digitalfilters.py:487-522) restated == the reference's own output."""
    g = np.load(os.path.join(golden_dir, "unit_read_profile.npz"))
    path = tmp_path / "profile.dat"
    path.write_text(str(g["text"]))
    for kma in (17, 32, 64):
        assert np.array_equal(np.stack(O.read_profile(str(path), kma)), g["k%d" % kma]), kma


def test_mid_case_reduced(golden_dir):
    """40 x 40 x 520 (three 256-row SYRK blocks, split K, spatial split ks=4 on the GPU side):
    the oracle against the reference's sampled columns, C rows, eigenvalues, modes and FC."""
    g = load(golden_dir, "mid_40x40x520")
    cfg = cfg_from(g)
    A = O.generate(cfg)
    for k, i in enumerate(g["A_steps"]):
        assert np.array_equal(A[:, i], g["A_cols"][k]), i
    mean, Ac = O.mean_and_center(A)
    assert np.array_equal(mean, g["mean_field"])
    res = O.pod(Ac, cfg.ns, cfg.nm)
    C = res["C"]
    assert np.array_equal(C[g["C_rows_idx"]], g["C_rows"])
    assert np.array_equal(np.diag(C), g["C_diag"])
    assert np.array_equal(C.sum(axis=0), g["C_colsum"])
    lam = g["energy"].real
    assert np.max(np.abs(res["energy"] - lam)) <= 1e-12 * lam[0]
    assert res["num_valid"] == int(g["num_valid_modes"]) and res["nm"] == int(g["nm"])
    nm = res["nm"]
    T, Tg = res["T"][:, :nm], g["temporal_modes"].real
    Phi, Pg = res["spatial"], g["spatial_modes"]
    for j in range(nm):
        sg = np.sign(np.dot(T[:, j], Tg[:, j]))
        assert np.max(np.abs(sg * T[:, j] - Tg[:, j])) <= 1e-10 * np.max(np.abs(Tg[:, j])), j
        assert np.max(np.abs(sg * Phi[:, j] - Pg[:, j])) <= 1e-10 * np.max(np.abs(Pg[:, j])), j
    fo = O.fourier(res["T"], cfg.ns, cfg.dt_eff, nm, cfg.et)
    assert np.array_equal(fo["c_count"], g["N_FC"])


def unit_2d(golden_dir, tag):
    g = np.load(os.path.join(golden_dir, "unit_adapt2d.npz"))
    J, K, inner = g[tag + "_cfg"]
    return (str(g[tag + "_name"]), int(J), int(K), float(inner), g[tag + "_prof"], g[tag + "_in"],
            g[tag + "_out"])


@pytest.mark.parametrize("tag", UNIT_2D)
def test_unit_adapt2d(golden_dir, tag):
    """adapt2d (digitalfilters.py:233-485) on raw fields: oracle point loop == reference."""
    name, J, K, inner, prof, yin, yout = unit_2d(golden_dir, tag)
    co, um = O.adapt2d_point_coeffs(name, inner, *prof, J, K)
    u, v, w = O.apply_lund(yin[0], yin[1], yin[2], co, um)
    assert np.array_equal(np.stack([u, v, w]), yout, equal_nan=True)


@pytest.mark.parametrize("name", CASES)
def test_generation_bit_exact(golden_dir, name):
    g = load(golden_dir, name)
    cfg = cfg_from(g)
    assert cfg.nfx == int(g["nfx"]) and cfg.nfy == int(g["nfy"])
    assert cfg.dt_eff == float(g["dt"])
    A = O.generate(cfg)
    assert np.array_equal(A, g["A_raw"])
    mean, Ac = O.mean_and_center(A)
    assert np.array_equal(mean, g["mean_field"])


@pytest.mark.parametrize("name", CASES)
def test_pod_and_fourier_bit_exact(golden_dir, name):
    g = load(golden_dir, name)
    cfg = cfg_from(g)
    Ac = g["A_raw"] - g["mean_field"][:, None]
    res = O.pod(Ac, cfg.ns, cfg.nm)
    assert np.array_equal(res["C"], g["C"])
    assert np.array_equal(res["energy"], g["energy"].real)
    assert res["num_valid"] == int(g["num_valid_modes"]) and res["nm"] == int(g["nm"])
    assert np.array_equal(res["T"][:, :res["nm"]], g["temporal_modes"].real)
    assert np.array_equal(res["spatial"], g["spatial_modes"])
    fo = O.fourier(res["T"], cfg.ns, cfg.dt_eff, res["nm"], cfg.et)
    assert fo["period"] == float(g["period"])
    assert np.array_equal(fo["c_count"], g["N_FC"])
    assert np.array_equal(fo["FC"], g["FC"])
    txt = O.podfs_dat_text(res["nm"], fo["period"], fo["c"], fo["c_ind"], fo["c_count"], cfg.ns)
    assert txt == str(g["podfs_dat"])
    assert O.eigenvalues_text(res["num_valid"], cfg.ns, res["energy"]) == str(g["eigenvalues_dat"])


def test_unit_filter_and_taps(golden_dir):
    g = np.load(os.path.join(golden_dir, "unit_filter.npz"))
    for n, l, key in ((9, 4.5, "taps_9"), (6, 3.0, "taps_6"), (4, 2.0, "taps_4"), (12, 6.0, "taps_12")):
        assert np.array_equal(O.calccoeff(n, l), g[key])
    y = O.filter_block(g["x"], g["taps_9"], g["taps_6"], g["taps_4"])
    assert np.array_equal(y, g["y"])
    assert np.array_equal(O.filter_block_scipy(g["x"], g["taps_9"], g["taps_6"], g["taps_4"]), g["y"])


def test_unit_rotation(golden_dir):
    g = np.load(os.path.join(golden_dir, "unit_rotation.npz"))
    for n, R in zip(g["normals"], g["R"]):
        n = n / np.linalg.norm(n)
        assert np.array_equal(O.rotation_matrix(*n), R)


def test_loops_form_matches_vectorised(golden_dir):
    g = load(golden_dir, "cli_10x11x5")
    cfg = cfg_from(g)
    assert np.array_equal(O.generate(cfg, loops=True), g["A_raw"])


@pytest.mark.parametrize("n", [1, 5, 7, 8, 9, 64, 127, 128, 129, 200, 1000, 4096, 4097, 8193, 9000, 16384, 20000, 50000])
def test_pairwise_restatement(n):
    a = np.random.default_rng(n).standard_normal(n) + 1.0
    assert O.pairwise_sum(a) == np.add.reduce(a)
    A = np.stack([a, a[::-1]])
    assert np.array_equal(np.mean(A, 1), np.array([O.pairwise_sum(a), O.pairwise_sum(a[::-1])]) / n)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 63, 64, 65, 100, 129, 1000, 4096, 8193, 9000, 16384, 20000])
def test_complex_pairwise_restatement(n):
    r = np.random.default_rng(n)
    z = r.standard_normal(n) + 1j * r.standard_normal(n)
    sr, si = O.cpairwise_sum(z.real, z.imag)
    assert complex(sr, si) == z.sum()


@pytest.mark.parametrize("ns", [5, 17, 64, 65, 130])
def test_dft_explicit_equals_reference_expression(ns):
    y = np.random.default_rng(ns).standard_normal(ns)
    time, period = O.time_axis(ns, 0.0731)
    assert np.array_equal(O.dft_explicit(y, time, period), O.dft_reference(y, time, period))


def test_dft_conjugate_symmetry():
    ns = 64
    y = np.random.default_rng(0).standard_normal(ns)
    time, period = O.time_axis(ns, 0.05)
    c = O.dft_reference(y, time, period)
    h = ns // 2
    for k in range(1, h):
        assert c[h + k] == np.conj(c[h - k])


def test_prf_row_geometry_doc_example():
    """docs/usage/CFDCodeIntegration.rst:53 -- first .prf data row for the default
    10 x 11 grid at res 0.1 (geometry + '%0.12f')."""
    from nsigproclib import str as fmt  # product helper (sp.str restatement)
    import PODFS
    pts = PODFS.cell_centres(10, 11, 0.1, (1.0, 0.0, 0.0), 0.0, (0.0, 0.0, 0.0))
    row = ",".join(fmt(v) for v in pts[0])
    assert row == "0.000000000000,-0.500000000000,0.550000011921"


def test_verbose_outputs_match_reference(golden_dir, tmp_path):
    """fct_welch (nsigproclib_no_mpi.py:10-68, every window, odd and even
    block sizes) and write_temporal_modes (PODFS.py:1468-1482) against the reference's own
    functions run by tests/golden/make_golden.py: identical arrays, identical file text."""
    import warnings
    import nsigproclib as sp
    import PODFS
    g = np.load(os.path.join(golden_dir, "unit_verbose.npz"))
    ncase = 0
    while "welch%d_cfg" % ncase in g.files:
        n, N, iw, fs = g["welch%d_cfg" % ncase]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            f, Sxx, M = sp.fct_welch(g["welch%d_x" % ncase], float(fs), int(N), int(iw))
        assert M == int(g["welch%d_M" % ncase])
        assert np.array_equal(f, g["welch%d_f" % ncase])
        assert Sxx.dtype == g["welch%d_Sxx" % ncase].dtype
        assert np.array_equal(Sxx, g["welch%d_Sxx" % ncase])
        ncase += 1
    assert ncase == 6
    PODFS.write_temporal_modes(3, 9, 0.0731, g["tmodes_T"], str(tmp_path) + "/")
    names = sorted(os.listdir(tmp_path))
    assert names == [str(s) for s in g["tmodes_names"]]
    for name, text in zip(names, g["tmodes_text"]):
        assert open(os.path.join(tmp_path, name)).read() == str(text)


@pytest.mark.parametrize("seed,offset", [(1, 0), (3, 1), (12345, 1_000_003), (2024, 4_000_001)])
def test_mt_jump_equals_sequential_draws(seed, offset):
    """oracle.mt_jump.stream_at(seed, D) continues np.random.RandomState(seed)'s stream at double
    D (Berlekamp-Massey characteristic polynomial, t^k mod phi, Horner on the word window): its
    next draws equal numpy's own after drawing and discarding D doubles."""
    from oracle import mt_jump
    ref = np.random.RandomState(seed)
    if offset:
        for i in range(0, offset, 1 << 22):
            ref.uniform(-O.SQRT3, O.SQRT3, size=min(1 << 22, offset - i))
    got = mt_jump.stream_at(seed, offset)
    assert np.array_equal(got.uniform(-O.SQRT3, O.SQRT3, size=4099), ref.uniform(-O.SQRT3, O.SQRT3, size=4099))
    assert mt_jump.char_poly().bit_length() - 1 == mt_jump.DEGREE


def test_generate_steps_jump_equals_draw(monkeypatch):
    """generate_steps(jump=True) (gaps skipped by the MT19937 jump-ahead) == the sequential pass,
    on late steps of a run where every gap exceeds the (lowered) jump threshold, with an
    anisotropic x filter (nfx != nfy) as at BASELINE config 5."""
    cfg = O.DFConfig(jma=20, kma=17, ns=400, seed=77, dt=0.5)
    monkeypatch.setattr(O, "JUMP_MIN", 5000)
    steps = [0, 150, 333, 399]
    a = O.generate_steps(cfg, steps)
    b = O.generate_steps(cfg, steps, jump=True)
    for i in steps:
        assert np.array_equal(a[i], b[i]), i

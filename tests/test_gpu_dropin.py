"""GPU: the reference-facing modules (digitalfilters.py / PODFS.py / HDF5.py) end to end,
the per-call operator API, and the sharded (multi-rank) pipeline on one device."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from oracle import pods_oracle as O  # noqa: E402


def _parse_podfs_dat(text):
    lines = text.split("\n")
    nm = int(lines[0])
    period = float(lines[1])
    counts = [int(l.split("\t")[1]) for l in lines[2:2 + nm]]
    rows = np.array([[float(x) for x in l.split("\t")] for l in lines[2 + nm:]]).reshape(-1, 3)
    return nm, period, counts, rows


def test_main_end_to_end_cli_case(golden_dir, tmp_path, monkeypatch):
    """python digitalfilters.py -n 5 --seed 7 (the quickstart example) vs the reference run."""
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "cli_10x11x5.npz"))
    monkeypatch.chdir(tmp_path)
    i_d = df.main(["-n", "5", "--seed", "7", "-5"])
    # PODFS.dat: same counts and ranks; coefficients equal up to the per-mode eigenvector sign
    nm, period, counts, rows = _parse_podfs_dat(open("PODFS/PODFS.dat").read())
    nm_g, period_g, counts_g, rows_g = _parse_podfs_dat(str(g["podfs_dat"]))
    assert (nm, counts) == (nm_g, counts_g) and period == period_g
    assert np.array_equal(rows[:, 0], rows_g[:, 0])
    start = 0
    for c in counts:
        blk, ref = rows[start:start + c, 1:], rows_g[start:start + c, 1:]
        s = np.sign(np.sum(blk * ref))
        assert np.max(np.abs(s * blk - ref)) <= 2e-6 * np.max(np.abs(ref)), start
        start += c
    ev = np.loadtxt("PODFS/POD.eigenvalues.dat")
    ev_g = np.loadtxt(__import__("io").StringIO(str(g["eigenvalues_dat"])))
    assert ev.shape == ev_g.shape
    assert np.max(np.abs(ev[:, 1] - ev_g[:, 1])) <= 1e-12 * ev_g[0, 1]
    # mean field is bit-exact, so PODFS_mean.prf is too
    import PODFS
    import nsigproclib as sp
    pts = PODFS.cell_centres(10, 11, 0.1)
    u = g["mean_field"].reshape((110, 3), order="F")
    body = "".join(",".join(sp.str(v) for v in (*pts[j], *u[j])) + "\n" for j in range(110))
    assert open("PODFS/PODFS_mean.prf").read().endswith(body)
    assert os.path.exists("PODFS/PODFS_mode_0004.prf") and not os.path.exists("PODFS/PODFS_mode_0005.prf")
    import HDF5
    if HDF5._h5py_python() is not None:
        assert os.path.getsize("PODFS/PODFS.hdf5") > 0
    assert i_d.nm == 4


def test_main_prf_inlet(golden_dir, tmp_path, monkeypatch):
    """python digitalfilters.py -i inlet.prf -n 6 --seed 31: read_prf sizes the grid and the
    per-point stresses (adapt2prf, no rotation); the snapshots' mean and the eigenvalues
    match the reference replay of the same file (tests/golden/readprf_case.npz)."""
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "readprf_case.npz"))
    u = np.load(os.path.join(golden_dir, "unit_read_prf.npz"))
    monkeypatch.chdir(tmp_path)
    with open("inlet.prf", "w") as f:
        f.write(str(u["prf_text"]))
    i_d = df.main(["-i", "inlet.prf", "-n", "6", "--seed", "31"])
    assert (i_d.jma, i_d.kma) == (int(g["cfg_jma"]), int(g["cfg_kma"]))
    assert np.array_equal(i_d.mean_field, g["mean_field"])
    lam = i_d.energy
    ref = g["energy"].real
    assert np.max(np.abs(lam - ref)) <= 1e-12 * ref[0]
    assert i_d.nm == int(g["nm"])
    scal = u["plain_scalars"]
    assert np.array_equal(np.array(i_d.n), scal[3:6])


def test_operator_api_bit_exact(golden_dir):
    import digitalfilters as df
    g = np.load(os.path.join(golden_dir, "unit_filter.npz"))
    y = np.zeros((7, 5))
    df.filter3DSciPy1D(g["x"], y, None, 7, 5, 4.5, 3.0, 2.0, 9, 6, 4)
    assert np.array_equal(y, g["y"])
    rng = np.random.default_rng(5)
    J, K = 6, 9
    yu, yv, yw = (rng.standard_normal((J, K)) for _ in range(3))
    U, uu, vv, ww, uw = O.build_profile("hyperbolic-tangent", "top-hat", 1.0, 0.02, K)
    uw = 0.3 * np.sqrt(uu * ww)
    ref = [a.copy() for a in (yu, yv, yw)]
    O.adapt1d_loops(*ref, U, uu, vv, ww, uw, J, K)
    got = [a.copy() for a in (yu, yv, yw)]
    df.adapt1d(*got, U, uu, vv, ww, uw, J, K)
    assert all(np.array_equal(a, b) for a, b in zip(got, ref))
    prf = {k: rng.uniform(0.1, 1.0, (J, K)) for k in ("U", "V", "W", "uu", "vv", "ww")}
    prf.update(uv=0.2 * rng.standard_normal((J, K)), uw=0.1 * rng.standard_normal((J, K)),
               vw=0.1 * rng.standard_normal((J, K)))
    co = O.lundprf_coeffs(prf["uu"], prf["vv"], prf["ww"], prf["uv"], prf["uw"], prf["vw"])
    ref = O.apply_lund(yu, yv, yw, co, prf["U"], prf["V"], prf["W"])
    got = [a.copy() for a in (yu, yv, yw)]
    df.adapt2prf(*got, prf["U"], prf["V"], prf["W"], prf["uu"], prf["vv"], prf["ww"], prf["uv"], prf["uw"],
                 prf["vw"], J, K)
    assert all(np.array_equal(a, b) for a, b in zip(got, ref))
    col = rng.standard_normal(3 * J * K)
    n = np.array([0.3, -0.5, 0.8]) / np.linalg.norm([0.3, -0.5, 0.8])
    assert np.array_equal(df.rotate_velocity(col, *n), O.rotate_velocity(col, O.rotation_matrix(*n)))


def test_pod_on_host_array_matches_reference(golden_dir):
    """PODFS.POD called like the reference (host A, already mean-subtracted)."""
    import PODFS
    g = np.load(os.path.join(golden_dir, "odd_12x9x17_aniso.npz"))
    Ac = g["A_raw"] - g["mean_field"][:, None]

    class I:
        verbose = False
    i_d = I()
    PODFS.POD(Ac, 17, 108, 3, "false", [], "", "false", 1e-15, 20, 0, "false", "false", None, None,
              float(g["dt"]), "velocity", 1, 17, 1, 1, i_d)
    assert i_d.nm == int(g["nm"])
    lam = g["energy"].real
    assert np.max(np.abs(i_d.energy - lam)) <= 1e-12 * lam[0]
    C = np.zeros((17, 17))
    PODFS.calculate_correlation_matrix(17, 108, 3, "false", [], Ac, C)
    assert np.max(np.abs(C - g["C"])) <= 1e-12 * np.max(np.abs(g["C"]))


def _rank_worker(rank, world, port, out):
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = podsgen.DFSetup(jma=40, kma=24, ns=48, seed=31)
    gen, pod, fo = E.pipeline(s, device=0, dist=dist)
    out[rank] = dict(j0=gen.j0, j1=gen.j1, energy=pod.energy, nm=pod.nm, phi=pod.phi.cpu().numpy(),
                     mean=pod.mean.cpu().numpy(), c=None if fo is None else fo.c)
    dist.destroy_process_group()


PIPE_SEEDS = (11, 12, 13)


def _steps_worker(rank, world, port, out):
    """Three steps of different seeds through engine.ShardedSteps, pipelined (step k-1's tail
    after step k's generation and correlation, two snapshot banks, rank 0's solve on its own
    stream) and not; every per-step output kept."""
    import torch
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = podsgen.DFSetup(jma=48, kma=40, ns=1024, seed=PIPE_SEEDS[0])
    res = {}
    for pipelined in (True, False):
        gen = E.Generator(s, device=0, rank=rank, world=world, dist=dist)
        spectrum = E.SpectrumQueue(gen.ctx, s.ns, rank, world)
        backlog = E.FourierBacklog()
        run = E.ShardedSteps(s, gen, dist, spectrum, backlog, pipelined=pipelined)
        for seed in PIPE_SEEDS:
            run.step(seed=seed)
        run.flush()
        spectrum.drain()
        torch.cuda.synchronize()
        res[pipelined] = dict(
            T=[p.T.cpu().numpy() for p in run.results], phi=[p.phi.cpu().numpy() for p in run.results],
            mean=[p.mean.cpu().numpy() for p in run.results], nm=[p.nm for p in run.results],
            spectra=spectrum.results(),
            fc=[None if f is None else (f.c, f.c_count, f.FC) for f in backlog.results])
        gen.ctx.close()
    out[rank] = res
    dist.destroy_process_group()


def test_pipelined_steps_bit_equal_two_ranks_one_device():
    """with several ranks, step k-1's POD tail (rank 0's leading-pair solve on
    its own stream, the broadcasts, the spatial modes from the other snapshot bank, the Fourier
    stage) runs after step k's generation and correlation are enqueued.  On 2 ranks (gloo, one
    GPU), three steps of different seeds: lambda (the spread spectra), T, Phi, the mean, nm and
    the Fourier coefficients / counts / FC rows equal the unpipelined run's bit for bit, and the
    steps differ from each other (so a bank mix-up would show)."""
    import multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29700 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_steps_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0
    for r in range(2):
        a, b = out[r][True], out[r][False]
        assert a["nm"] == b["nm"]
        for key in ("T", "phi", "mean"):
            for k in range(len(PIPE_SEEDS)):
                assert np.array_equal(a[key][k], b[key][k]), (r, key, k)
            assert not np.array_equal(a[key][0], a[key][1]), (r, key)
        assert sorted(a["spectra"]) == sorted(b["spectra"])
        for k in a["spectra"]:
            assert np.array_equal(a["spectra"][k], b["spectra"][k]), (r, k)
        assert len(a["fc"]) == len(b["fc"])
        for fa, fb in zip(a["fc"], b["fc"]):
            assert (fa is None) == (fb is None)
            if fa is not None:
                for x, y in zip(fa, fb):
                    assert np.array_equal(x, y)
    assert sum(len(out[r][True]["spectra"]) for r in range(2)) == len(PIPE_SEEDS)
    assert out[0][True]["fc"][0] is not None


def _prefetch_worker(rank, world, port, out):
    """Three steps of one seed through engine.ShardedSteps with the next step's MT jump-ahead
    prefetched (bench.py's order), the jump enqueued before the generation (PODS_JUMP_EARLY, the
    default) or after it, and without any prefetch."""
    import torch
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = podsgen.DFSetup(jma=48, kma=40, ns=1024, seed=21)
    res = {}
    for name, early, ahead in (("early", "1", True), ("late", "0", True), ("none", "1", False)):
        os.environ["PODS_JUMP_EARLY"] = early
        gen = E.Generator(s, device=0, rank=rank, world=world, dist=dist)
        assert gen._xch is not None   # the MT state exchange is on with several ranks
        spectrum = E.SpectrumQueue(gen.ctx, s.ns, rank, world)
        run = E.ShardedSteps(s, gen, dist, spectrum, E.FourierBacklog())
        for k in range(3):
            run.step(prefetch_next=ahead and k < 2)
        run.flush()
        spectrum.drain()
        torch.cuda.synchronize()
        res[name] = dict(T=[p.T.cpu().numpy() for p in run.results], phi=[p.phi.cpu().numpy() for p in run.results],
                         mean=[p.mean.cpu().numpy() for p in run.results], spectra=spectrum.results())
        gen.ctx.close()
    os.environ.pop("PODS_JUMP_EARLY", None)
    out[rank] = res
    dist.destroy_process_group()


def test_jump_prefetch_early_bit_equal_two_ranks_one_device():
    """The next step's jump-ahead enqueued before this step's generation (beside its planes and
    x / y-z passes; Generator.prefetch_jump_early), after it, or not prefetched at all: on 2 ranks
    with the MT state exchange (gloo, one GPU), every step's mean, T, Phi and spectrum are equal
    bit for bit -- and, one seed for all steps, equal from step to step."""
    import multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29300 + os.getpid() % 500
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_prefetch_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0
    for r in range(2):
        ref = out[r]["none"]
        for name in ("early", "late"):
            got = out[r][name]
            for key in ("T", "phi", "mean"):
                for k in range(3):
                    assert np.array_equal(got[key][k], ref[key][k]), (r, name, key, k)
                    assert np.array_equal(ref[key][k], ref[key][0]), (r, key, k)
            assert sorted(got["spectra"]) == sorted(ref["spectra"])
            for k in got["spectra"]:
                assert np.array_equal(got["spectra"][k], ref["spectra"][k]), (r, name, k)


def _world1_worker(backend, port, out):
    """One rank, three steps of ShardedSteps with the next step's jump prefetched (bench.py's
    order): once through the collective path over a world-1 `backend` group (collectives=True: the
    packed all-reduce issued asynchronously and finished on rank 0's solve stream; the MT state
    exchange, whose all_to_all is issued asynchronously on the gen stream), once without any
    collective or exchange (the reference)."""
    import torch
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    s = podsgen.DFSetup(jma=48, kma=40, ns=1024, seed=23)
    res = {"backend": dist.get_backend()}
    for name, coll in (("coll", True), ("plain", False)):
        d = dist if coll else None
        gen = E.Generator(s, device=0, rank=0, world=1, dist=d, exchange=coll)
        assert (gen._xch is not None) == coll
        spectrum = E.SpectrumQueue(gen.ctx, s.ns, 0, 1)
        backlog = E.FourierBacklog()
        run = E.ShardedSteps(s, gen, d, spectrum, backlog, collectives=coll)
        assert run.collectives == coll
        for k in range(3):
            run.step(prefetch_next=k < 2)
        run.flush()
        backlog.flush()
        spectrum.drain()
        torch.cuda.synchronize()
        res[name] = dict(T=[p.T.cpu().numpy() for p in run.results], phi=[p.phi.cpu().numpy() for p in run.results],
                         mean=[p.mean.cpu().numpy() for p in run.results], nm=[p.nm for p in run.results],
                         spectra=spectrum.results(),
                         fc=[None if f is None else (f.c, f.c_count, f.FC) for f in backlog.results])
        gen.ctx.close()
    out[backend] = res
    dist.destroy_process_group()


def test_world1_collective_paths_rccl_and_gloo_bit_equal():
    """the RCCL branches of the multi-GPU path execute on this one device -- a
    world-1 `nccl` (RCCL) process group drives ShardedSteps with its collectives forced: the MT
    state exchange's all_to_all_single on device buffers (issued asynchronously on the gen stream,
    Generator.exchange_states), the packed correlation's async all_reduce, finished and unpacked on
    rank 0's solve stream (the solve waits for the all-reduce only).  Every step's mean,
    T, Phi, spectrum and Fourier counts / FC rows are bit-equal to the same steps with no
    collective at all, and to the same run over gloo (its host-copy exchange branch)."""
    import multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    for i, backend in enumerate(("nccl", "gloo")):
        p = ctx.Process(target=_world1_worker, args=(backend, 29900 + os.getpid() % 80 + i, out))
        p.start()
        p.join(600)
        assert p.exitcode == 0, backend
    assert out["nccl"]["backend"] == "nccl" and out["gloo"]["backend"] == "gloo"
    ref = out["gloo"]["plain"]
    for run in (out["nccl"]["coll"], out["nccl"]["plain"], out["gloo"]["coll"]):
        assert run["nm"] == ref["nm"]
        for key in ("T", "phi", "mean"):
            assert len(run[key]) == 3
            for k in range(3):
                assert np.array_equal(run[key][k], ref[key][k]), (key, k)
        assert sorted(run["spectra"]) == sorted(ref["spectra"]) == [0, 1, 2]
        for k in ref["spectra"]:
            assert np.array_equal(run["spectra"][k], ref["spectra"][k]), k
        assert len(run["fc"]) == len(ref["fc"]) == 3
        for fa, fb in zip(run["fc"], ref["fc"]):
            assert fa is not None and fb is not None
            for x, y in zip(fa, fb):
                assert np.array_equal(x, y)


def test_one_gpu_pipelined_steps_bit_equal():
    """on ONE device (no process group) the pipelined runner -- step k's
    generation into snapshot bank k % 2, mean and correlation enqueued before step k-1's tail (the
    leading-pair solve on its own stream beside them, the spectrum units and spatial modes of
    step k-1 from the other bank, the Fourier stage) -- gives every step's mean, T, Phi, nm,
    spectrum and Fourier counts / FC rows bit-equal to the same steps run one after the other
    (pipelined=False, bank 0), over three seeds whose results differ."""
    import podsgen
    from podsgen import engine as E
    s = podsgen.DFSetup(jma=48, kma=40, ns=1024, seed=PIPE_SEEDS[0])
    res = {}
    for pipelined in (True, False):
        gen = E.Generator(s, device=0)
        spectrum = E.SpectrumQueue(gen.ctx, s.ns, 0, 1)
        backlog = E.FourierBacklog()
        run = E.ShardedSteps(s, gen, None, spectrum, backlog, pipelined=pipelined)
        assert run.world == 1 and not run.collectives
        for seed in PIPE_SEEDS:
            run.step(seed=seed)
        run.flush()
        backlog.flush()
        spectrum.drain()
        torch.cuda.synchronize()
        res[pipelined] = dict(
            T=[p.T.cpu().numpy() for p in run.results], phi=[p.phi.cpu().numpy() for p in run.results],
            mean=[p.mean.cpu().numpy() for p in run.results], nm=[p.nm for p in run.results],
            spectra=spectrum.results(),
            fc=[None if f is None else (f.c, f.c_count, f.FC) for f in backlog.results])
        gen.ctx.close()
    a, b = res[True], res[False]
    assert a["nm"] == b["nm"]
    for key in ("T", "phi", "mean"):
        assert len(a[key]) == len(PIPE_SEEDS)
        for k in range(len(PIPE_SEEDS)):
            assert np.array_equal(a[key][k], b[key][k]), (key, k)
        assert not np.array_equal(a[key][0], a[key][1]), key
    assert sorted(a["spectra"]) == sorted(b["spectra"]) == list(range(len(PIPE_SEEDS)))
    for k in a["spectra"]:
        assert np.array_equal(a["spectra"][k], b["spectra"][k]), k
    assert len(a["fc"]) == len(b["fc"]) == len(PIPE_SEEDS)
    for fa, fb in zip(a["fc"], b["fc"]):
        assert fa is not None and fb is not None
        for x, y in zip(fa, fb):
            assert np.array_equal(x, y)


def _tiny_worker(rank, world, port, out):
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = podsgen.DFSetup(jma=8, kma=8, ns=16, seed=5, lengthscale=1.0, nm=4)
    gen = E.Generator(s, device=0, rank=rank, world=world, dist=dist)
    xch = gen._xch is not None
    gen, pod, fo = E.pipeline(s, device=0, dist=dist, gen=gen)
    out[rank] = dict(j0=gen.j0, j1=gen.j1, xch=xch, mean=pod.mean.cpu().numpy(), nm=pod.nm)
    dist.destroy_process_group()


def test_tiny_inlet_two_ranks_whole_stream_fallback():
    """an inlet whose random planes are shorter than one 312-word MT19937 block (8 x 8,
    nf = 2: S = 144) has no state-exchange plan (pods_df_set_exchange: PODS_ERR_UNSUPPORTED); a
    multi-rank Generator then falls back to every rank twisting the whole stream instead of
    failing -- 2 ranks (gloo, one GPU): the pipeline runs and every slab's mean equals the
    single-rank run's rows bit for bit."""
    import multiprocessing as mp
    import podsgen
    from podsgen import engine as E
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29150 + os.getpid() % 40
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_tiny_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    s = podsgen.DFSetup(jma=8, kma=8, ns=16, seed=5, lengthscale=1.0, nm=4)
    assert s.nfy == 2 and (s.jma + 2 * s.nfy) * (s.kma + 2 * s.nfz) < 312
    gen, pod, fo = E.pipeline(s, device=0)
    mean = pod.mean.cpu().numpy()
    P, K = s.P, s.kma
    for r in range(2):
        d = out[r]
        assert not d["xch"]
        pl = (d["j1"] - d["j0"]) * K
        for comp in range(3):
            rows = slice(comp * P + d["j0"] * K, comp * P + d["j1"] * K)
            assert np.array_equal(d["mean"][comp * pl:(comp + 1) * pl], mean[rows])
        assert d["nm"] == pod.nm


def test_sharded_pipeline_two_ranks_one_device():
    """Row slabs on 2 ranks (gloo transport, one GPU) == the single-rank pipeline."""
    import multiprocessing as mp
    import podsgen
    from podsgen import engine as E
    mgr = mp.Manager()
    out = mgr.dict()
    port = 29600 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    s = podsgen.DFSetup(jma=40, kma=24, ns=48, seed=31)
    gen, pod, fo = E.pipeline(s, device=0)
    lam = pod.energy
    assert np.max(np.abs(out[0]["energy"] - lam)) <= 1e-12 * lam[0]
    phi = pod.phi.cpu().numpy()
    mean = pod.mean.cpu().numpy()
    P, K = s.P, s.kma
    for r in range(2):
        d = out[r]
        pl = (d["j1"] - d["j0"]) * K
        for comp in range(3):
            rows = slice(comp * P + d["j0"] * K, comp * P + d["j1"] * K)
            assert np.array_equal(d["mean"][comp * pl:(comp + 1) * pl], mean[rows])
    # signed modes: ONE sign per mode for the whole field (the eigenvector's), taken from
    # rank 0's slab; every slab must then agree with that sign -- a per-slab sign error fails
    for m in range(pod.nm):
        d0 = out[0]
        pl0 = (d0["j1"] - d0["j0"]) * K
        rows0 = slice(d0["j0"] * K, d0["j1"] * K)
        sg = np.sign(np.dot(d0["phi"][:pl0, m], phi[rows0, m]))
        assert sg != 0
        for r in range(2):
            d = out[r]
            pl = (d["j1"] - d["j0"]) * K
            for comp in range(3):
                rows = slice(comp * P + d["j0"] * K, comp * P + d["j1"] * K)
                a = d["phi"][comp * pl:(comp + 1) * pl, m]
                assert np.max(np.abs(sg * a - phi[rows, m])) <= 1e-10 * np.max(np.abs(phi[:, m])), (r, comp, m)
        c_sg = sg
        assert np.max(np.abs(c_sg * out[0]["c"][:, m] - fo.c[:, m])) <= 1e-6 * np.max(np.abs(fo.c[:, m]))


def _h5py_ok():
    import HDF5
    return HDF5._h5py_python() is not None


def _verbose_worker(rank, world, port, wdir, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    os.chdir(wdir)
    import digitalfilters as df
    i_d = df.main(["-n", "6", "--seed", "19", "-j", "9", "-k", "8", "-v"] + (["-5"] if _h5py_ok() else []))
    out[rank] = dict(nm=i_d.nm, mean=None if rank else i_d.mean_field)
    dist.destroy_process_group()


def test_verbose_cli_two_ranks_one_device(tmp_path):
    """digitalfilters.py -v under 2 ranks (gloo, one GPU): the per-step snapshot planes are
    gathered to rank 0 and written there byte-identical to the single-rank run (A is
    bit-exact), the temporal-mode files come from rank 0's full T only (no IndexError on the
    ranks holding T[:, :nm]), and the PODFS outputs match the single-rank run."""
    import multiprocessing as mp
    single, multi = tmp_path / "single", tmp_path / "multi"
    single.mkdir()
    multi.mkdir()
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_verbose_worker, args=(0, 1, 29700 + os.getpid() % 500, str(single), out))
    p.start()
    p.join(300)
    assert p.exitcode == 0
    ref = dict(out[0])
    port = 29200 + os.getpid() % 500
    procs = [ctx.Process(target=_verbose_worker, args=(r, 2, port, str(multi), out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    assert out[0]["nm"] == ref["nm"] and out[1]["nm"] == ref["nm"]
    assert np.array_equal(out[0]["mean"], ref["mean"])
    names = sorted(os.listdir(single / "PODFS"))
    assert sorted(os.listdir(multi / "PODFS")) == names
    planes = [n for n in names if n.endswith(".prf") and not n.startswith("PODFS_")]
    assert len(planes) == 6
    for n in planes:
        assert (single / "PODFS" / n).read_text() == (multi / "PODFS" / n).read_text(), n
    tmodes = [n for n in names if n.startswith("POD.temporal_mode_")]
    assert len(tmodes) >= ref["nm"]
    for n in tmodes:
        a = np.loadtxt(single / "PODFS" / n)
        b = np.loadtxt(multi / "PODFS" / n)
        assert np.array_equal(a[:, 0], b[:, 0])
        sg = np.sign(np.dot(a[:, 1], b[:, 1]))
        assert np.max(np.abs(a[:, 1] - sg * b[:, 1])) <= 1e-9 * np.max(np.abs(a[:, 1])), n
    assert (single / "PODFS" / "PODFS_mean.prf").read_text() == (multi / "PODFS" / "PODFS_mean.prf").read_text()
    if _h5py_ok():   # the HDF5 file written from the modes streamed to rank 0 one at a time
        import subprocess
        import HDF5
        reader = ("import h5py, numpy as np, sys\n"
                  "a, b = (h5py.File(x, 'r')['main'] for x in sys.argv[1:3])\n"
                  "assert np.array_equal(a['mean'][:], b['mean'][:]) and sorted(a['modes']) == sorted(b['modes'])\n"
                  "for k in a['modes']:\n"
                  "    x, y = a['modes'][k][:], b['modes'][k][:]\n"
                  "    P = x.size // 6\n"
                  "    assert np.array_equal(x[:3 * P], y[:3 * P])\n"
                  "    sg = np.sign(np.dot(x[3 * P:], y[3 * P:]))\n"
                  "    assert np.max(np.abs(x[3 * P:] - sg * y[3 * P:])) <= 1e-9 * np.max(np.abs(x[3 * P:])), k\n"
                  "print('ok', len(a['modes']))\n")
        r = subprocess.run([HDF5._h5py_python(), "-c", reader, str(single / "PODFS" / "PODFS.hdf5"),
                            str(multi / "PODFS" / "PODFS.hdf5")], capture_output=True, text=True)
        assert r.stdout.split() == ["ok", str(ref["nm"])], r.stderr


def test_pack_unpack_lower_kernels():
    """pods_pack_lower / pods_unpack_lower (the all-reduce's packed triangle): the pack is the
    lower triangle row by row, the unpack writes packed / ns to both triangles -- exactly
    numpy's IEEE division, C exactly symmetric -- at sizes with ragged 64 x 64 edge tiles."""
    import podsgen
    from podsgen import engine as E
    ctx = E.Context(0)
    try:
        pack, unpack = E.device_triangle_ops(ctx)
        for n in (1, 2, 63, 64, 65, 130, 1000):
            C = torch.randn(n, n, dtype=torch.float64, device="cuda")
            packed = pack(C)
            r, c = torch.tril_indices(n, n, device="cuda")
            assert torch.equal(packed, C[r, c]), n
            packed.mul_(3.0)
            out = torch.full((n, n), float("nan"), dtype=torch.float64, device="cuda")
            unpack(packed, out)
            torch.cuda.synchronize()
            # numpy's true division (torch divides by a Python scalar as a multiply by 1/n)
            q = torch.from_numpy(packed.cpu().numpy() / n).cuda()
            ref = torch.zeros_like(out)
            ref[r, c] = q
            ref[c, r] = q
            assert torch.equal(out, ref), n
            assert torch.equal(out, out.T)
        podsgen.check(ctx.lib.pods_synchronize(ctx.h), "sync")
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_bench_launches_its_own_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (torch.distributed.run as a
    child process); with --backend gloo both share this one GPU.  Rank 0's JSON line reports
    the world it observed and the all-reduce stage (PODFS.py:1451-1455 summed over slabs)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--config", "c1", "--steps", "2", "--warmup", "1", "--no-cpu"],
                       capture_output=True, text=True, timeout=540, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["config"]["dist_world_size"] == 2
    assert out["config"]["backend"] == "gloo"
    assert "allreduce" in out["stages_ms"]
    assert out["metric"].startswith("filtered-snapshot Mpoints/s") and "32x32" in out["metric"]
    assert out["value"] > 0


@pytest.mark.timeout(1500)
def test_bench_c3_two_ranks_one_device_no_fallback():
    """`bench.py --gpus 2 --backend gloo` at C3 (ns = 4096: the split eigensolve, the spectrum
    units of engine.SpectrumQueue on both ranks) with both ranks on this one GPU.  The ranks'
    persistent grids take the per-device lock (pods_set_shared_device), so none of them starves
    the other's: the run completes without any fallback (no 'eigvalsh', no 'falling back', no
    unconverged subspace iteration) -- r3's run of the same command aborted its hand-off waits."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONWARNINGS"] = "always::UserWarning"   # inherited by the ranks
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--config", "c3", "--steps", "2", "--warmup", "1", "--no-cpu"],
                       capture_output=True, text=True, timeout=840, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    for bad in ("eigvalsh", "falling back", "did not converge", "aborted"):
        assert bad not in r.stderr, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["ns"] == 4096
    assert out["results"]["eigensolve"].startswith("split")
    assert out["results"]["num_valid"] is not None and out["results"]["nm"] == 20
    assert out["config"]["mt_state_exchange"] and out["config"]["pipelined_tail"]
    # the same job on one rank (fused eigensolve, no exchange, no pipeline) gives
    # the same results: the valid-mode count of the full spectrum and every mode's Fourier count
    r1 = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--config", "c3",
                         "--steps", "2", "--warmup", "1", "--no-cpu"],
                        capture_output=True, text=True, timeout=600, env=env, cwd=root)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][-1])
    assert one["results"]["eigensolve"].startswith("fused")
    assert out["results"]["num_valid"] == one["results"]["num_valid"]
    assert out["results"]["nm"] == one["results"]["nm"]
    assert out["results"]["N_FC"] == one["results"]["N_FC"], (out["results"]["N_FC"], one["results"]["N_FC"])


@pytest.mark.timeout(600)
def test_bench_c2_generation_line():
    """`bench.py --config c2` (BASELINE config 2: the digital filter + Lund transform only): one JSON
    line with the generation-only metric, the per-kernel HIP-event times (jump, planes, x pass, y/z
    pass) summing to about the step, and the y/z kernel's HBM roofline."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", "c2", "--steps", "3",
                        "--warmup", "1", "--no-cpu"], capture_output=True, text=True, timeout=540, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert "generation only" in out["metric"] and out["config"]["ns"] == 4096
    st = out["stages_ms"]
    assert set(st) == {"gen_jump", "gen_planes", "gen_xpass", "gen_yzpass"}
    assert 0.8 * out["ms_per_step"] <= sum(st.values()) <= 1.05 * out["ms_per_step"]
    rl = out["roofline"]
    assert rl["bound"] == "hbm" and 0.0 < rl["frac"] < 1.0 and rl["unit"] == "GB/s"
    assert 0.0 < out["generation_roofline"]["frac"] < 1.0

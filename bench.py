#!/usr/bin/env python3
"""Headline benchmark: filtered-snapshot Mpoints/s of the digital-filter + PODFS path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--no-cpu]

One "step" is the whole hot path over one synthetic problem (BASELINE.json config 3,
256 x 256 inlet x 4096 snapshots): MT19937 random field -> 3 separable Gaussian filter
passes -> Lund transform -> snapshot matrix -> mean -> correlation (exact int8-MFMA
residue SYRKs + CRT to fp64, RCCL all-reduce when N > 1) -> eigensolve -> temporal/spatial modes -> Fourier
coefficients ranked and counted (the arrays PODFS.pod2prf / HDF5.write_HDF5 consume).
File writing is outside the step.  A point is one inlet (j, k) at one step (3 fp64
components); value = J*K*ns*steps / wall(max over ranks) / 1e6.

N > 1 runs one process per GPU under torch.distributed.run; the inlet rows are split
into N slabs (strong scaling: the same 256^2 x 4096 problem at every N).

Extra JSON objects (rank 0):
  roofline      the dominant kernel, k_syrk_i8 (pods_corr's 16 residue SYRKs), int8 MFMA
                bound; achieved = 16 * 3P * ns * (ns+1) algorithmic int ops per launch / mean
                launch time from HIP events the library records around it on its stream
                inside the timed steps (pods_corr_timing); traffic from the committed
                rocprofv3 PMC summary (profiles/) when one exists for this config.  With
                PODS_CORR=f64: the fp64 SYRK, 3P*ns*(ns+1) flops / the corr stage time.
  cpu_baseline  the oracle (faithful numpy/scipy restatement of the reference, incl. its
                Python loops) on a bounded sample of the same workload, extrapolated to the
                full job (N = 1, rank 0 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pods-digital-filter_amd"))

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (J, K, ns, description)
    "c1": (32, 32, 64, "32x32 inlet x 64 snapshots (BASELINE config 1)"),
    "c2": (256, 256, 4096, "256x256 inlet x 4096 snapshots, fp64, digital-filter convolution + Lund transform "
                           "only (BASELINE config 2)"),
    "c3": (256, 256, 4096, "256x256 inlet x 4096 snapshots, digital filter + full PODFS (BASELINE config 3)"),
    "c4": (512, 512, 8192, "512x512 inlet x 8192 snapshots (BASELINE config 4)"),
    # BASELINE config 5: 1024^2 inlet, anisotropic length scales (-t: lnx = 2 ln -> nfx = 12,
    # nfy = nfz = 6) and an inhomogeneous Reynolds-stress field through adapt2prf.  The full
    # 16384-snapshot job needs ~165 GB per GPU on 8 GPUs (A 412 GB in all); c5s is the same
    # workload at 1024 snapshots, which fits one GPU (readiness check, not a BASELINE line).
    "c5": (1024, 1024, 16384, "1024x1024 inlet x 16384 snapshots, anisotropic filter + inhomogeneous R "
                              "(BASELINE config 5)"),
    "c5s": (1024, 1024, 1024, "1024x1024 inlet x 1024 snapshots, anisotropic filter + inhomogeneous R "
                              "(config 5 workload at reduced ns, one GPU)"),
}


# A/B: one device, the spatial-mode pass beside the next step's generation (engine.pipeline overlap_spatial)
OVERLAP_SPATIAL = os.environ.get("PODS_OVERLAP_SPATIAL", "0") == "1"

def c5_profile(J, K):
    """a deterministic inhomogeneous SPD stress field on a tanh jet,
    uu = vv = ww = (0.02 U)^2 scaled, uv/uw/vw = rho sqrt(..) with a smooth rho in (-0.4, 0.4),
    fed through adapt2prf (digitalfilters.py:180-231) like a read_prf profile."""
    y = np.linspace(-0.5, 0.5, J)[:, None]
    z = np.linspace(-0.5, 0.5, K)[None, :]
    U = 0.5 * (1.0 + np.tanh(10.0 * (0.5 - np.sqrt(y ** 2 + z ** 2)))) + 0.05
    V = 0.01 * np.sin(3.0 * y) * np.ones_like(z)
    W = 0.01 * np.cos(2.0 * z) * np.ones_like(y)
    s = (0.02 * U) ** 2
    rho = 0.4 * np.sin(2.0 * y + 3.0 * z) * np.ones_like(U)
    uu, vv, ww = s.copy(), 1.1 * s, 0.9 * s
    uv = rho * np.sqrt(uu * vv)
    uw = -0.5 * rho * np.sqrt(uu * ww)
    vw = 0.3 * rho * np.sqrt(vv * ww)
    return dict(U=U, V=V, W=W, uu=uu, vv=vv, ww=ww, uv=uv, uw=uw, vw=vw)


def make_setup(podsgen, config, seed):
    J, K, ns, _ = CONFIGS[config]
    if config in ("c5", "c5s"):
        prf = c5_profile(J, K)
        U = prf["U"]
        flag = np.where(U ** 2 + prf["V"] ** 2 + prf["W"] ** 2 != 0)
        dt1 = 0.1 / np.mean(U[flag])   # main() :1306-1309 with res = 0.1
        # -t dt1/2 doubles the x length scale (:1310-1317): lnx = 6, nfx = 12
        return podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=seed, dt=dt1 / 2.0, prf=prf)
    return podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=seed)
FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X dense FP64 matrix (spec); measured 70-76 by tools/mfma_bench.hip
# MI355X dense int8 matrix: v_mfma_i32_16x16x64_i8 = 32768 ops per 16 cycles per SIMD
# (MI355X_MICROARCH.md: I8 = 2x BF16 per clock), 1024 SIMDs at 2.4 GHz
I8_MFMA_PEAK_TOPS = 2048 * 1024 * 2.4e9 / 1e12
CORR_NMOD = 16  # residue SYRKs per correlation (podsgen_corr_i8.hip NMOD)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU sampling")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo for "
                         "CPU-transport tests of the multi-rank path, e.g. 2 ranks on one GPU)")
    return ap.parse_args()


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: start N ranks as children through
    torch.distributed.run (before anything here touches the GPU; no exec) and return their
    exit status.  Under torch.distributed.run (WORLD_SIZE set) this is not called."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cpu_baseline(J, K, ns, nm=20, budget=20.0):
    """Time the oracle (test infrastructure, CPU) on the host cores, as BASELINE.md plans it:
    the generation loop on its first 64 steps (x ns/64: per-step cost is constant), the PODFS
    stages in full -- mean + centring of the whole (3P, ns) A, np.dot(A.T, A) on it,
    np.linalg.eig (dgeev, PODFS.py:1309) of the resulting ns x ns C, the spatial modes and the
    direct DFT of all nm modes -- and the plot-only reconstruction loop on a sample (x its
    iteration count).  `budget` only bounds the generation sample at large sizes."""
    from oracle import pods_oracle as O  # only the cpu_baseline leg imports the oracle
    cores = len(os.sched_getaffinity(0))
    blas_threads = None
    try:
        from threadpoolctl import threadpool_info
        blas_threads = max([1] + [int(i.get("num_threads", 1)) for i in threadpool_info()
                                  if i.get("user_api") == "blas"])
    except Exception:
        pass
    t_all = time.perf_counter()
    est, how = {}, {}
    # generation: reference-faithful loop (scipy convolve x3, adapt1d loop, rotate loop)
    cfg = O.DFConfig(jma=J, kma=K, ns=ns, seed=1)
    m = min(64, ns)
    t = time.perf_counter()
    O.generate(cfg, loops=True, steps=2)
    per = (time.perf_counter() - t) / 2
    if per * m > 4 * budget:  # only at sizes beyond C3
        m = max(2, int(4 * budget / per))
    t = time.perf_counter()
    O.generate(cfg, loops=True, steps=m)
    est["generate"] = (time.perf_counter() - t) / m * ns
    how["generate"] = "first %d of %d steps, x ns/%d" % (m, ns, m)
    # the PODFS stages in full on a (3P, ns) matrix of the workload's shape
    P3 = 3 * J * K
    rng = np.random.default_rng(0)
    A = rng.random((P3, ns))
    t = time.perf_counter()
    mean = np.mean(A, 1)
    A -= mean[:, None]
    est["mean"] = time.perf_counter() - t
    t = time.perf_counter()
    C = np.dot(A.T, A) / ns
    est["corr"] = time.perf_counter() - t
    t = time.perf_counter()
    lam, V = np.linalg.eig(C)
    est["eig"] = time.perf_counter() - t
    order = np.argsort(-lam.real)
    T = V[:, order[:nm]].real
    t = time.perf_counter()
    np.dot(np.dot(A, T), np.diag(np.ones(nm) / lam[order[:nm]].real)) / ns
    est["spatial"] = time.perf_counter() - t
    del A
    time_, period = O.time_axis(ns, 0.1)
    t = time.perf_counter()
    for i in range(nm):
        O.dft_reference(T[:, i], time_, period)
    est["dft"] = time.perf_counter() - t
    for k in ("mean", "corr", "eig", "spatial", "dft"):
        how[k] = "full"
    # the y2 reconstruction loop (PODFS.py:1603-1612), c_count ~ 0.3 ns
    c = np.zeros(ns, dtype=np.complex64)
    reps = 2000
    t = time.perf_counter()
    f = 0
    for n in range(reps):
        f += c[n % ns] * np.exp(1j * 2 * 3 * np.pi * 0.5 / period)
    per_it = (time.perf_counter() - t) / reps
    est["reconstruct"] = per_it * ns * (0.3 * ns) * nm
    how["reconstruct"] = "%d iterations, x ns * 0.3 ns * nm" % reps
    total = sum(est.values())
    used = blas_threads or 1
    sample = ("oracle (numpy %s / scipy, reference-faithful Python loops) on %d BLAS threads: generation %s; "
              "mean, SYRK np.dot(A.T, A) (%dx%d), dgeev n=%d, spatial modes, DFT of %d modes in full; "
              "reconstruction loop %s; measured in %.1f s"
              % (np.__version__, used, how["generate"], P3, ns, ns, nm, how["reconstruct"],
                 time.perf_counter() - t_all))
    # `cores` = the threads that actually ran: numpy's BLAS/LAPACK pool (the SYRK, dgeev and spatial
    # stages; OMP_NUM_THREADS caps it at the box's CPU share), the Python loops on one of them
    return {"value": J * K * ns / total / 1e6, "unit": "Mpoints/s", "cores": used, "kind": "port",
            "affinity_cores": cores, "blas_threads": blas_threads,
            "threads_note": "Python loops (generation, reconstruction) run on one core; numpy BLAS/LAPACK "
                            "(SYRK, dgeev, spatial) on its %d-thread pool (%d cores in the affinity mask)"
                            % (used, cores),
            "sample": sample, "seconds_full_job": round(total, 2),
            "stages_s": {k: round(v, 3) for k, v in est.items()}, "stage_basis": how}


def load_traffic(config, corr_mode):
    """HBM bytes per launch of the roofline kernel from the committed PMC summary (profiles/)."""
    path = os.path.join(ROOT, "profiles", ("pmc_corr_i8_%s.json" if corr_mode == 1 else "pmc_syrk_%s.json") % config)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


HBM_PEAK_TBS = 8.0             # MI355X HBM3E (MI355X_MICROARCH.md)
SURVEY_C3_COMBINED = 6130.0    # the C3 combined roofline with the fp64 SYRK floor (Mpoints/s)


def combined_roofline(J, K, ns, ms_per_step, world, corr_mode):
    """The whole step against the floor of the arithmetic it runs, per stage:
    generation 24 B/unit (A written once), mean 24 B (A read), residues 72 B (A read, 16 int8
    residues of 3 components written), spatial modes 24 B (A read) at the HBM peak, and the 16
    residue SYRKs' int8 ops at the int8 MFMA peak (the fp64 SYRK's flops at the fp64 peak with
    PODS_CORR=f64, plus the centring's 48 B).  The eigensolve is latency-bound (a per-column
    cross-CU hop) and has no roofline term; it is excluded, so this floor is optimistic.  A unit is
    one inlet point at one step (3 fp64 components)."""
    units = float(J * K * ns)
    hbm = lambda b: b * units / (HBM_PEAK_TBS * 1e12) * 1e3   # noqa: E731
    floors = {"generate": hbm(24), "mean": hbm(24), "spatial": hbm(24)}
    if corr_mode == 1:
        floors["residues"] = hbm(72)
        floors["syrk_i8"] = 2.0 * CORR_NMOD * 3 * J * K * ns * (ns + 1) / 2 / (I8_MFMA_PEAK_TOPS * 1e12) * 1e3
    else:
        floors["center"] = hbm(48)
        floors["syrk_f64"] = 3.0 * J * K * ns * (ns + 1) / (FP64_MFMA_PEAK_TFLOPS * 1e12) * 1e3
    floor_ms = sum(floors.values()) / world
    value = units / (ms_per_step * 1e-3) / 1e6
    out = {"floor_ms": round(floor_ms, 3), "floor_mpoints_s": round(units / (floor_ms * 1e-3) / 1e6, 1),
           "stage_floors_ms": {k: round(v / world, 3) for k, v in floors.items()},
           "frac": round(floor_ms / ms_per_step, 4),
           "note": "floor of the arithmetic run (excl. the latency-bound eigensolve) / ms_per_step"}
    if (J, K, ns) == (256, 256, 4096):
        out["survey_frac"] = round(value / SURVEY_C3_COMBINED, 4)
        out["survey_note"] = ("value / SURVEY.md 8(d)'s %.0f Mpoints/s C3 roofline (priced with the fp64 SYRK "
                              "floor of 42 ms)" % SURVEY_C3_COMBINED)
    return out


def metric_name(config):
    J, K, ns, _ = CONFIGS[config]
    if config == "c3":  # BASELINE.json's headline metric
        return "filtered-snapshot Mpoints/s (gen+PODFS), 256^2 inlet x 4096 steps, 1/2/4/8 GPU"
    if config == "c2":
        return "filtered-snapshot Mpoints/s (generation only: filter + Lund), 256^2 inlet x 4096 steps (c2)"
    return "filtered-snapshot Mpoints/s (gen+PODFS), %dx%d inlet x %d steps (%s)" % (J, K, ns, config)


# Algorithmic HBM bytes per unit (one inlet point at one step, 3 fp64 components) of the generator
# kernels at C2/C3: the random planes written once (3 S (ns + 2nfx) doubles), the x pass
# reading them and writing T1 (3 S ns), the y/z pass reading T1 and writing A (3 P ns)
def gen_bytes_per_unit(J, K, ns, nfx, nfy, nfz):
    S = (J + 2 * nfy) * (K + 2 * nfz)
    units = float(J * K * ns)
    planes = 3.0 * S * (ns + 2 * nfx) * 8 / units
    t1 = 3.0 * S * ns * 8 / units
    return {"gen_planes": planes, "gen_xpass": planes + t1, "gen_yzpass": t1 + 24.0, "output": 24.0}


def load_gen_traffic(config):
    """Per-kernel L2-miss bytes per launch of the generator kernels (profiles/pmc_gen_<config>.json)."""
    path = os.path.join(ROOT, "profiles", "pmc_gen_%s.json" % config)
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def bench_generation(args, E, gen, setup, world, rank, dist):
    """BASELINE config 2: the digital filter + Lund transform only (digitalfilters.py:1403-1481 without
    the POD).  A step is one whole generation of the 256^2 x 4096 snapshot matrix, every kernel on the
    main stream -- the MT19937 jump-ahead, the random planes, the x pass, the y/z pass (+ Lund) -- each
    bracketed by its own HIP-event pair, so the stage times are the kernels' times."""
    import torch
    J, K, ns = setup.jma, setup.kma, setup.ns
    for _ in range(args.warmup):
        gen.generate()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tm = E.StageTimer()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gen.generate(timer=tm if world == 1 else None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank != 0:
        return
    ms = elapsed / args.steps * 1e3
    units = float(J * K * ns)
    stages = {k: v / args.steps for k, v in tm.summary().items()}
    bpu = gen_bytes_per_unit(J, K, ns, setup.nfx, setup.nfy, setup.nfz)
    pmc = load_gen_traffic(args.config) if world == 1 else None
    kern = {"gen_jump": "k_mt_jump3", "gen_planes": "k_mt_generate_full", "gen_xpass": "k_filter_x2",
            "gen_yzpass": "k_filter_yz"}
    per_kernel = {}
    for st, kname in kern.items():
        if st not in stages:
            continue
        row = {"kernel": kname, "ms": round(stages[st], 3)}
        if st in bpu:
            gbs = bpu[st] * units / (stages[st] * 1e-3) / 1e9
            row.update(algorithmic_bytes_per_unit=round(bpu[st], 2), achieved_GBps=round(gbs, 1),
                       frac=round(gbs / (HBM_PEAK_TBS * 1e3), 4))
        if pmc:
            for k, v in pmc.get("kernels", {}).items():
                if kname in k:
                    row["traffic"] = v["bytes"]
        per_kernel[st] = row
    yz = per_kernel.get("gen_yzpass")
    gen_gbs = 24.0 * units / (ms * 1e-3) / 1e9
    out = {
        "metric": metric_name(args.config), "value": round(units / (ms * 1e-3) / 1e6, 3), "unit": "Mpoints/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded MT19937 random field, built tanh/top-hat profile)",
        "config": {"workload": CONFIGS[args.config][3], "jma": J, "kma": K, "ns": ns,
                   "nf": [setup.nfx, setup.nfy, setup.nfz], "parallelism": "row-slab dp%d" % world},
        "roofline": None if yz is None else {
            "kernel": "k_filter_yz (y/z filter passes + Lund transform + rotation, K-tiled snapshot store)",
            "bound": "hbm", "achieved": yz["achieved_GBps"], "peak": HBM_PEAK_TBS * 1e3, "unit": "GB/s",
            "frac": yz["frac"], "traffic": yz.get("traffic"),
            "algorithmic_bytes_per_launch": round(bpu["gen_yzpass"] * units), "launch_ms": yz["ms"]},
        "generation_roofline": {
            "note": "the whole step against its output: 24 B per unit (A written once) / ms_per_step / 8 TB/s",
            "achieved_GBps": round(gen_gbs, 1), "frac": round(gen_gbs / (HBM_PEAK_TBS * 1e3), 4),
            "floor_ms": round(24.0 * units / (HBM_PEAK_TBS * 1e12) * 1e3, 3),
            "kernel_traffic_GB": None if not pmc else round(sum(r.get("traffic", 0.0) for r in per_kernel.values())
                                                          / 1e9, 2),
            "algorithmic_kernel_GB": round(sum(bpu[k] for k in ("gen_planes", "gen_xpass", "gen_yzpass")) * units
                                           / 1e9, 2)},
        "kernels": per_kernel,
        "stages_ms": {k: round(v, 3) for k, v in stages.items()},
        "stages_note": "per-step means of HIP-event pairs around each generation kernel, main stream",
    }
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_generation(J, K, ns, args.cpu_budget)
    print(json.dumps(out), flush=True)


def cpu_baseline_generation(J, K, ns, budget=20.0):
    """The oracle's reference-faithful generation loop (scipy convolve x3, adapt1d, rotate) on its first
    steps, x ns / steps (per-step cost is constant)."""
    from oracle import pods_oracle as O  # only the cpu_baseline leg imports the oracle
    cfg = O.DFConfig(jma=J, kma=K, ns=ns, seed=1)
    t = time.perf_counter()
    O.generate(cfg, loops=True, steps=2)
    per = (time.perf_counter() - t) / 2
    m = max(2, min(64, int(budget / max(per, 1e-9))))
    t = time.perf_counter()
    O.generate(cfg, loops=True, steps=m)
    sec = (time.perf_counter() - t) / m * ns
    return {"value": J * K * ns / sec / 1e6, "unit": "Mpoints/s", "cores": 1, "kind": "port",
            "sample": "oracle generation (reference-faithful Python loops, one core): first %d of %d steps, x ns/%d"
                      % (m, ns, m), "seconds_full_job": round(sec, 2)}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    import torch
    import torch.distributed as dist
    import podsgen
    from podsgen import engine as E

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr)
    # gloo: the multi-rank path on however many GPUs there are (ranks may share one)
    ndev = max(torch.cuda.device_count(), 1)
    device = local % ndev if args.backend == "gloo" else local
    torch.cuda.set_device(device)
    observed_world = 1
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        observed_world = dist.get_world_size()
    J, K, ns, desc = CONFIGS[args.config]
    setup = make_setup(podsgen, args.config, args.seed)
    # per-run setup, outside the timed steps (it depends only on the configuration): the context,
    # the generator's configuration (Lund table, filter taps, MT19937 jump polynomials on the
    # host) and the DFT's host twiddle table (numpy's own exp, PODFS.py:1564-1566) -- reported
    # as setup_ms, and paid once by a single digitalfilters.py run
    torch.cuda.synchronize()
    t_setup = time.perf_counter()
    gen = E.Generator(setup, device=device, rank=rank, world=world, dist=dist if world > 1 else None)
    torch.cuda.synchronize()
    setup_ms = {"configure": (time.perf_counter() - t_setup) * 1e3}
    t_setup = time.perf_counter()
    if rank == 0:
        time_, period = E.time_axis(ns, setup.dt_eff)
        E.ensure_twiddles(gen.ctx, ns, np.ascontiguousarray(time_, dtype=np.float64), period)
        torch.cuda.synchronize()
    setup_ms["dft_twiddles"] = (time.perf_counter() - t_setup) * 1e3
    d = dist if world > 1 else None
    if args.config == "c2":
        bench_generation(args, E, gen, setup, world, rank, d)
        if world > 1:
            dist.destroy_process_group()
        return
    # several ranks: the nm leading eigenpairs on the critical path (subspace iteration), the
    # rest of the spectrum spread over the ranks' following steps (engine.SpectrumQueue)
    # PODS_N1_PIPELINE=1 (measurement): one GPU through the same pipelined runner as N > 1 (the
    # leading-pair solve of step k-1 beside step k's generation and correlation, the spectrum
    # units behind them) instead of the fused per-step solver
    n1pipe = world == 1 and os.environ.get("PODS_N1_PIPELINE") == "1"
    split = (world > 1 or n1pipe or os.environ.get("PODS_EIGEN") == "split") and ns >= E.SPLIT_MIN_N
    spectrum = E.SpectrumQueue(gen.ctx, ns, rank, world) if split else None

    # several ranks: step k-1's POD tail (rank 0's leading-pair solve, broadcasts, spatial modes)
    # runs while the device has step k's generation and correlation (engine.ShardedSteps, two
    # snapshot banks; PODS_PIPELINE=0 runs each tail right after its own all-reduce)
    runner = E.ShardedSteps(setup, gen, d, spectrum) if world > 1 or n1pipe else None

    def step(timer=None, backlog=None, ahead=False):
        if runner is not None:
            runner.backlog = backlog
            runner.step(timer=timer, prefetch_next=ahead)
            return None, None, None
        return E.pipeline(setup, device=device, dist=d, gen=gen, timer=timer, spectrum=spectrum, backlog=backlog,
                          prefetch_next=ahead, overlap_spatial=OVERLAP_SPATIAL)

    # ahead: the next step's MT19937 jump-ahead runs on a second stream beside this step's mean
    # and centring (Generator.prefetch_jump).  The last warm-up step and the last timed step do
    # not prefetch, so the timed region holds exactly `steps` whole generations.
    for w in range(args.warmup):
        step(ahead=w < args.warmup - 1)
    if runner is not None:
        runner.flush()
    if spectrum is not None:
        spectrum.drain()
        spectrum.results()
        spectrum.finished.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events (torch.cuda.Event = hipEvent_t on the stream the kernels run on) bracket
    # every stage inside the timed steps; they are read only after the timed region
    tm_run = E.StageTimer()
    # each step's host-side Fourier results (copies, FC rows) finish during the next step's
    # SYRK (E.FourierBacklog); the last one, and the last steps' spectra, inside the timed region
    backlog = E.FourierBacklog()
    corr_mode = gen.ctx.corr_mode()
    podsgen.check(gen.ctx.lib.pods_corr_timing(gen.ctx.h, 1), "pods_corr_timing")
    t0 = time.perf_counter()
    for s in range(args.steps):
        _, pod, _ = step(timer=tm_run, backlog=backlog, ahead=s < args.steps - 1)
    if runner is not None:
        runner.flush(tm_run)
        pod = runner.results[-1]
    backlog.flush()
    fo = backlog.results[-1]
    if spectrum is not None:
        with tm_run("eig_full_drain"):
            spectrum.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms = elapsed / args.steps * 1e3
    value = J * K * ns * args.steps / elapsed / 1e6

    # stage split and the roofline of the dominant kernel, from the timed steps' events
    stages = {k: v / args.steps for k, v in tm_run.summary().items()}
    import ctypes
    k_ms, k_n = ctypes.c_double(0.0), ctypes.c_int(0)
    podsgen.check(gen.ctx.lib.pods_corr_kernel_ms(gen.ctx.h, ctypes.byref(k_ms), ctypes.byref(k_n)),
                  "pods_corr_kernel_ms")
    podsgen.check(gen.ctx.lib.pods_corr_timing(gen.ctx.h, 0), "pods_corr_timing")

    # one job on its own (after the timed region): generation to the FC arrays with no
    # cross-step overlap -- no prefetched jump-ahead or planes, the Fourier results finished in
    # the step, the full spectrum computed within it -- i.e. a single digitalfilters.py run's
    # latency once set up (a fresh process adds setup_ms)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    E.pipeline(setup, device=device, dist=d, gen=gen)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    one_shot = time.perf_counter() - t1
    if world > 1:
        tt = torch.tensor([one_shot], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        one_shot = float(tt.item())
    corr_ms = stages["corr"]
    P_local = (gen.j1 - gen.j0) * K
    flops = 3.0 * P_local * ns * (ns + 1)
    # the committed PMC summary is for the one-GPU launch; a rank's launch at N > 1 covers
    # only its row slab, so no measured figure applies there
    traffic = load_traffic(args.config, corr_mode) if world == 1 else None
    if corr_mode == 1 and k_n.value > 0:
        # the int8 SYRK: CORR_NMOD residue SYRKs of the 3 P x ns matrix, timed alone by HIP events
        kern_ms = k_ms.value / k_n.value
        ops = 2.0 * CORR_NMOD * 3 * P_local * ns * (ns + 1) / 2
        achieved = ops / (kern_ms * 1e-3) / 1e12
        roofline = {"kernel": "k_syrk_i8_paced (pods_corr's %d residue SYRKs on int8 MFMA), rank 0" % CORR_NMOD,
                    "bound": "mfma", "dtype": "i8", "achieved": round(achieved, 1), "peak": round(I8_MFMA_PEAK_TOPS, 1),
                    "unit": "TOP/s", "frac": round(achieved / I8_MFMA_PEAK_TOPS, 4), "traffic": traffic,
                    "launch_ms": round(kern_ms, 3), "ops_per_launch": ops, "launches": k_n.value,
                    "corr_stage_ms": round(corr_ms, 3),
                    "corr_fp64_emulated_tflops": round(flops / (corr_ms * 1e-3) / 1e12, 2),
                    "corr_fp64_emulated_note": ("3P ns (ns+1) fp64-equivalent flop / the corr stage time: the "
                                                "rate of an exact integer emulation on the int8 pipe, above the "
                                                "%.1f TFLOP/s fp64 MFMA peak by construction" % FP64_MFMA_PEAK_TFLOPS),
                    "bound_note": ("the int8 pipe is fed by LDS-DMA: 214 GB L2->LDS per launch at C3; measured "
                                   "(DESIGN.md s3): MFMAs alone 16.9 ms (the chip holds ~1.7-1.94 GHz under "
                                   "this load), the kernel with an L2-resident K window 19.3 ms; r6: "
                                   "SQ_VALU_MFMA_BUSY_CYCLES = 16 x the MFMA count, pipe busy 0.645 at the "
                                   "1.66 GHz held under the profiler; MFMAs + fragment reads alone 17.3 ms, "
                                   "operand traffic alone 20.6 ms (profiles/r6/syrk_mfma_calibration.json, "
                                   "syrk_diag_ab.log); one persistent workgroup per CU, the 32 of an XCD paced "
                                   "round by round over the same panels")}
    else:
        achieved = flops / (corr_ms * 1e-3) / 1e12
        roofline = {"kernel": "pods_corr (k_syrk_g128 + k_syrk_reduce), rank 0",
                    "bound": "mfma", "dtype": "f64", "achieved": round(achieved, 3),
                    "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / FP64_MFMA_PEAK_TFLOPS, 4),
                    "traffic": traffic, "launch_ms": round(corr_ms, 3),
                    "flops_per_launch": flops}
    num_valid = pod.num_valid
    if spectrum is not None:   # from the last full spectrum (whichever rank owned it)
        done = spectrum.results()
        last = torch.zeros(2 * world, dtype=torch.float64, device="cuda")
        if done:
            last[2 * rank] = max(done) + 1
            last[2 * rank + 1] = E.num_valid_modes(done[max(done)], ns)
        if world > 1:
            dist.all_reduce(last)
        last = last.view(world, 2).cpu().numpy()
        r = int(np.argmax(last[:, 0]))
        num_valid = int(last[r, 1]) if last[r, 0] > 0 else None
    if world > 1:
        dist.barrier()
    if rank == 0:
        out = {
            "metric": metric_name(args.config),
            "value": round(value, 3),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (seeded MT19937 random field, inhomogeneous SPD stress field via adapt2prf, "
                     "anisotropic x filter)" if args.config in ("c5", "c5s") else
                     "synthetic (seeded MT19937 random field, built tanh/top-hat profile)"),
            "config": {"workload": desc, "jma": J, "kma": K, "ns": ns, "nm": setup.nm,
                       "nf": [setup.nfx, setup.nfy, setup.nfz], "parallelism": "row-slab dp%d" % world,
                       "pipelined_tail": bool(runner is not None and runner.pipelined),
                       "mt_state_exchange": bool(gen._xch is not None),
                       "backend": args.backend if world > 1 else None, "dist_world_size": observed_world},
            "roofline": roofline,
            "combined_roofline": combined_roofline(J, K, ns, ms, world, corr_mode),
            "corr_arithmetic": ("exact: int8-MFMA residue products mod 16 pairwise-coprime moduli + CRT, one "
                                "rounding to f64 (pods_corr mode 1)" if corr_mode == 1 else
                                "fp64 MFMA SYRK (pods_corr mode 0)"),
            "stages_ms": {k: round(v, 3) for k, v in stages.items()},
            "setup_ms": {k: round(v, 1) for k, v in setup_ms.items()},
            "one_shot_ms": round(one_shot * 1e3, 3),
            "one_shot_note": ("one job alone after the timed steps: no cross-step overlap (no prefetched "
                              "jump-ahead / planes, Fourier finished in the step, full spectrum within the job); "
                              "a fresh process adds setup_ms"),
            "stages_note": ("per-step means of HIP-event times on the stream each stage runs on; "
                            "gen_jump_ahead (the next step's MT19937 jump-ahead) runs on a second "
                            "stream beside mean+center, so the stages do not sum to ms_per_step"),
            "results": {"nm": int(pod.nm), "num_valid": None if num_valid is None else int(num_valid),
                        "eigensolve": "split: leading pairs by subspace iteration + full spectrum spread over "
                                      "steps (SpectrumQueue)" if spectrum is not None else "fused (pods_syev)",
                        "N_FC": [int(x) for x in fo.c_count] if fo is not None else None},
        }
        if world == 1 and not args.no_cpu and args.config in ("c1", "c3"):
            out["cpu_baseline"] = cpu_baseline(J, K, ns, setup.nm, args.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

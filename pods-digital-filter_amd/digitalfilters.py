#!/usr/bin/env python3
"""digitalfilters.py -- drop-in for the digital-filter generator of sidbannet/PODS-digital-filter.

    python digitalfilters.py -j 256 -k 256 -n 4096 [options]        (same CLI, Python 3)

Keeps the reference's entry points (digitalfilters.py) and their meaning:
  calccoeff(a, n, ln)                                   :73-89
  coeff3D(a, nfx, nfy, nfz, lnx, lny, lnz)              :46-70
  filter3D(x, y, a, jma, kma, nfx, nfy, nfz)            :91-98
  filter3DSciPy1D(x, y, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz)   :100-140
  adapt1d(yu, yv, yw, uin, uuin, vvin, wwin, uwin, jma, kma)          :143-178
  adapt2prf(yu, yv, yw, uin, vin, win, uuin, vvin, wwin, uvin, uwin, vwin, jma, kma)  :180-231
  adapt2d(yu, yv, yw, uin, uuin, vvin, wwin, uwin, jma, kma, mean_profile, inner_d)  :233-485
  read_profile(profilefile, kma)                        :487-522
  read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad)   :524-1035
  build_profile(...), prof_rotation_matrix(...), rotate_velocity(A, nx, ny, nz)  :1038-1131
  main()                                                :1134-1510

The per-call operators run their arithmetic on the GPU through libpodsgen (bit-identical
to the reference's numpy/scipy results).  main() does not loop over steps in Python: one
fused device pass (MT19937 stream -> x/y/z filters -> Lund -> rotation -> snapshot matrix)
replaces the step loop, then PODFS runs on the device-resident snapshots.

Extensions: --seed (the reference never seeds its RNG; np.random.seed(seed) semantics),
the documentation's long option names as aliases (--udash, --num_steps, --filter_width,
--num_modes), and multi-GPU under torch.distributed.run (one process per GPU, inlet rows
sharded, one RCCL all-reduce of the correlation matrix).
"""
import math
import os
import sys
from optparse import Option, OptionParser

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import HDF5  # noqa: E402
import PODFS as pod  # noqa: E402
import podsgen  # noqa: E402
from podsgen import engine as _E  # noqa: E402
from podsgen import host as _H  # noqa: E402

PROG = "DigitalFilters"
VERSION = "1.1.0-mi355x"
Pi = np.pi

build_profile = _H.build_profile
prof_rotation_matrix = _H.prof_rotation_matrix


class obj(object):
    """The reference's attribute bag i_d (digitalfilters.py:31-32)."""
    a = 0


class MultipleOption(Option):
    ACTIONS = Option.ACTIONS + ("extend",)
    STORE_ACTIONS = Option.STORE_ACTIONS + ("extend",)
    TYPED_ACTIONS = Option.TYPED_ACTIONS + ("extend",)
    ALWAYS_TYPED_ACTIONS = Option.ALWAYS_TYPED_ACTIONS + ("extend",)

    def take_action(self, action, dest, opt, value, values, parser):
        if action == "extend":
            values.ensure_value(dest, []).append(value)
        else:
            Option.take_action(self, action, dest, opt, value, values, parser)


_CTX = None


def _ctx():
    global _CTX
    if _CTX is None:
        _CTX = _E.Context(int(os.environ.get("LOCAL_RANK", "0")))
    return _CTX


# ------------------------------------------------------------------------------------------
# operator API
# ------------------------------------------------------------------------------------------
def calccoeff(a, n, ln):
    """:73-89 -- fills a with the unnormalised taps, returns them normalised."""
    norm = 0.0
    for i in range(n * 2 + 1):
        k = float(i - n)
        a[i] = np.exp(-Pi * k * k / (2.0 * ln * ln))
        norm = norm + a[i] ** 2
    norm = np.sqrt(norm)
    return a / norm


def coeff3D(a, nfx, nfy, nfz, lnx, lny, lnz):
    ax = _H.calccoeff(nfx, lnx)
    ay = _H.calccoeff(nfy, lny)
    az = _H.calccoeff(nfz, lnz)
    a[0, :, :, :] = ax[:, None, None] * ay[None, :, None] * az[None, None, :]


def filter3DSciPy1D(x, y, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz):
    """Three 'valid' 1-D convolutions x -> y -> z on the GPU, scipy's direct-path order."""
    bx, by, bz = _H.calccoeff(nfx, lnx), _H.calccoeff(nfy, lny), _H.calccoeff(nfz, lnz)
    xc = np.ascontiguousarray(x, dtype=np.float64)
    if xc.shape != (2 * nfx + 1, 2 * nfy + jma, 2 * nfz + kma):
        raise ValueError("x has shape %s, expected %s" % (xc.shape, (2 * nfx + 1, 2 * nfy + jma, 2 * nfz + kma)))
    out = np.empty((jma, kma))
    c = _ctx()
    podsgen.check(c.lib.pods_filter_block(c.h, _E.ptr(xc), nfx, nfy, nfz, jma, kma, _E.ptr(bx), _E.ptr(by),
                                          _E.ptr(bz), _E.ptr(out)), "pods_filter_block")
    y[:, :] = out


def filter3D(x, y, a, jma, kma, nfx, nfy, nfz):
    """The reference's brute-force 3-D filter (:91-98) is dead code kept for its accuracy
    check; it is the same linear operator as filter3DSciPy1D with the 3-D product taps, so
    it is served by the separable GPU filter (equal to rounding, which is what the
    reference's own L2-norm comparison at :1434-1436 checks)."""
    lnx = _infer_ln(a[0, :, nfy, nfz], nfx)
    lny = _infer_ln(a[0, nfx, :, nfz], nfy)
    lnz = _infer_ln(a[0, nfx, nfy, :], nfz)
    filter3DSciPy1D(x, y, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz)


def _infer_ln(tap_line, n):
    if n == 0:
        return 1.0
    r = tap_line[n + 1] / tap_line[n]
    return math.sqrt(-Pi / (2.0 * math.log(r)))


def _lund_rows_1d(uin, uuin, vvin, wwin, uwin, jma, kma):
    K = kma
    fac = _H.lund1d_factor(*(np.broadcast_to(np.asarray(v, dtype=np.float64), (K,)) for v in (uuin, vvin, wwin, uwin)))
    rows = np.zeros((9, jma, kma))
    for r, v in enumerate(fac):
        rows[r] = np.broadcast_to(np.asarray(v, dtype=np.float64), (K,))[None, :]
    rows[6] = np.asarray(uin, dtype=np.float64)[None, :]
    return rows.reshape(9, jma * kma)


def _apply(yu, yv, yw, rows, mode, rot):
    P = yu.size
    bufs = [np.ascontiguousarray(v, dtype=np.float64).reshape(P).copy() for v in (yu, yv, yw)]
    c = _ctx()
    podsgen.check(c.lib.pods_lund_apply(c.h, _E.ptr(bufs[0]), _E.ptr(bufs[1]), _E.ptr(bufs[2]), P,
                                        _E.ptr(rows) if rows is not None else None, mode,
                                        _E.ptr(rot) if rot is not None else None), "pods_lund_apply")
    for dst, src in zip((yu, yv, yw), bufs):
        dst[...] = src.reshape(dst.shape)


def adapt1d(yu, yv, yw, uin, uuin, vvin, wwin, uwin, jma, kma):
    rows = np.ascontiguousarray(_lund_rows_1d(uin, uuin, vvin, wwin, uwin, jma, kma))
    _apply(yu, yv, yw, rows, 0, None)


def adapt2prf(yu, yv, yw, uin, vin, win, uuin, vvin, wwin, uvin, uwin, vwin, jma, kma):
    fac = _H.lundprf_factor(uuin, vvin, wwin, uvin, uwin, vwin)
    rows = np.stack(list(fac) + [np.asarray(uin), np.asarray(vin), np.asarray(win)]).astype(np.float64)
    _apply(yu, yv, yw, np.ascontiguousarray(rows.reshape(9, jma * kma)), 1, None)


def adapt2d(yu, yv, yw, uin, uuin, vvin, wwin, uwin, jma, kma, mean_profile, inner_d):
    """:233-485 -- double/circular/ring hyperbolic-tangent profiles: the per-point factor and
    mean velocity are evaluated on the host (podsgen.profiles2d), the transform on the GPU."""
    from podsgen.profiles2d import adapt2d_factor
    fac = adapt2d_factor(mean_profile, inner_d, uin, uuin, vvin, wwin, uwin, jma, kma)
    rows = np.zeros((9, jma * kma))
    for r in range(7):
        rows[r] = np.asarray(fac[r], dtype=np.float64).reshape(jma * kma)
    _apply(yu, yv, yw, np.ascontiguousarray(rows), 0, None)


def rotate_velocity(A, nx, ny, nz):
    """rotate_velocity (:1119-1131): R.dot(V) per point, in OpenBLAS dgemv's fma order."""
    A = np.asarray(A, dtype=np.float64)
    pts = len(A) // 3
    R = np.ascontiguousarray(_H.prof_rotation_matrix(nx, ny, nz), dtype=np.float64)
    u, v, w = (np.array(A[c * pts:(c + 1) * pts]) for c in range(3))
    _apply(u, v, w, None, -1, R)
    return np.concatenate([u, v, w])


def read_profile(profilefile, kma):
    """1-D text profile with columns y, U, uu, vv, ww, uv (:487-522); mirrored about y=1,
    spline-interpolated to kma points, zero at both walls."""
    from scipy import interpolate
    d = np.genfromtxt(profilefile, names=True, autostrip=True, comments="#")
    npoints = d.shape[0]
    for i in reversed(d[0:npoints - 2]):
        d = np.append(d, i)
    d["y"][npoints:] = (-(d["y"][npoints:] - 1.0) + 1)
    d["uv"][npoints:] = -d["uv"][npoints:]
    z = d["y"]
    z = (z - np.min(z)) / (np.max(z) - np.min(z))
    zi = np.linspace(np.min(z), np.max(z), kma)
    out = []
    for name in ("U", "uu", "vv", "ww", "uv"):
        v = interpolate.splev(zi, interpolate.splrep(z, d[name], s=0), der=0)
        v[0] = v[-1] = 0.
        out.append(v)
    return tuple(out)


def save_plane(u, i_d):
    """Verbose per-step snapshot .prf (PODFS.py:854-887) with the analytic cell centres."""
    import nsigproclib as sp
    points = i_d.grid.points
    npt = points.shape[0]
    os.makedirs("./PODFS", exist_ok=True)
    fn = "./PODFS/" + ("%.5E" % i_d.time) + ".prf"
    rhs = i_d.t_o[0] * i_d.n[0] + i_d.t_o[1] * i_d.n[1] + i_d.t_o[2] * i_d.n[2]
    with open(fn, "w") as f:
        f.write("# Generated using the digital filter method # name of the profile\n")
        f.write("# turbulence model, none\n")
        f.write("# plane normal and translation " + str(i_d.n[0]) + "\t" + str(i_d.n[1]) + "\t" + str(i_d.n[2]) +
                "\t" + str(rhs) + "\n")
        f.write("type, xyz # type of profile (rad or xyz)\n")
        f.write("localcs,origin,0,0,0 # origin of local coordinate system\n")
        f.write("localcs,xaxis,1,0,0 # x axis direction of local coordinate system\n")
        f.write("localcs,yaxis,0,1,0 # y axis direction of local coordinate system\n")
        f.write("localcs,zaxis,0,0,1 # z axis direction of local coordinate system\n")
        f.write("tolerance, 1.00E-08 # tolerance\n")
        f.write("scale,1,1,1,1,1,1 # scaling factors\n")
        f.write("data,x,y,z,u,v,w\n")
        for i in range(npt):
            f.write(sp.str(points[i, 0]) + "," + sp.str(points[i, 1]) + "," + sp.str(points[i, 2]) + "," +
                    sp.str(u[i]) + "," + sp.str(u[i + npt]) + "," + sp.str(u[i + 2 * npt]) + "\n")


# ------------------------------------------------------------------------------------------
# CLI
# ------------------------------------------------------------------------------------------
def make_parser():
    parser = OptionParser(option_class=MultipleOption, usage="usage: %prog [options]",
                          version="%s %s" % (PROG, VERSION),
                          description=" LES Inflow Generator after Klein et.al. (MI355X build) ")
    a = parser.add_option
    a("-i", "--inputfile", dest="profilefile", default="none", help="1d turbulent profile file", metavar="FILE")
    a("-p", "--mean_profile", dest="mean_profile", default="hyperbolic-tangent",
      help="hyperbolic-tangent, double-hyperbolic-tangent, circular-hyperbolic-tangent, ring-hyperbolic-tangent",
      metavar="STRING")
    a("--turb_profile", dest="turb_profile", default="top-hat", help="top-hat, none", metavar="STRING")
    a("--U0", "--bulk_velocity", type="float", dest="bulk_velocity", default=1.0, metavar="NUM")
    a("--u_dash", "--udash", type="float", dest="turbulence_intensity", default="0.02", metavar="NUM")
    a("-n", "--nsteps", "--num_steps", type="int", dest="nsteps", default=20, metavar="INT")
    a("-l", "--lengthscale", type="float", dest="lengthscale", default=3.0, metavar="NUM")
    a("-f", "--fwidth", "--filter_width", type="float", dest="fwidth", default=2.0, metavar="NUM")
    a("-k", "--nk", type="int", dest="kma", default=11, metavar="INT")
    a("-j", "--nj", type="int", dest="jma", default=10, metavar="INT")
    a("-t", "--dt", type="float", dest="dt", default=0.0, metavar="NUM")
    a("-m", "--nm", "--num_modes", type="int", dest="nm", default=20, metavar="INT")
    a("-e", "--et", type="float", dest="et", default=0.9, metavar="NUM")
    a("-v", "--verbose", dest="verbose", default=False, action="store_true")
    a("--non_dim", dest="non_dim", default=False, action="store_true")
    a("-r", "--resolution", type="float", dest="res", default=0.1, metavar="NUM")
    a("--nx", type="float", dest="nx", default=1.0, metavar="NUM")
    a("--ny", type="float", dest="ny", default=0.0, metavar="NUM")
    a("--nz", type="float", dest="nz", default=0.0, metavar="NUM")
    a("--ox", type="float", dest="ox", default=0.0, metavar="NUM")
    a("--oy", type="float", dest="oy", default=0.0, metavar="NUM")
    a("--oz", type="float", dest="oz", default=0.0, metavar="NUM")
    a("--rotate", type="float", dest="rot", default=0.0, metavar="NUM")
    a("--ring", type="float", dest="ring", default=0.5, metavar="NUM")
    a("--massflow", type="float", dest="mdot", default=0.0, metavar="NUM")
    a("--density", type="float", dest="den", default=0.0, metavar="NUM")
    a("-5", "--hdf5", dest="hdf5", default=False, action="store_true")
    a("--test_gradients", dest="TestGrad", default=False, action="store_true")
    a("--seed", type="int", dest="seed", default=None,
      help="seed numpy's legacy RandomState (np.random.seed); default: a random seed", metavar="INT")
    return parser


def setup_from_options(options):
    profilefile = options.profilefile
    seed = options.seed
    if seed is None:
        seed = int.from_bytes(os.urandom(4), "little")
    kw = dict(jma=options.jma, kma=options.kma, ns=options.nsteps, seed=seed, lengthscale=options.lengthscale,
              fwidth=options.fwidth, dt=options.dt, res=options.res, bulk_velocity=options.bulk_velocity,
              u_dash=options.turbulence_intensity, nm=options.nm, et=options.et,
              normal=(options.nx, options.ny, options.nz), mean_profile=options.mean_profile,
              turb_profile=options.turb_profile, inner_d=options.ring)
    if profilefile != "none" and os.path.isfile(profilefile):
        if profilefile.endswith(".prf"):  # :1299-1305 -- plane, grid and stresses from the file
            (U, V, W, uu, vv, ww, uv, uw, vw, lnx, kma, jma, nx, ny, nz, ox, oy, oz) = read_prf(
                profilefile, options.res, options.mdot, options.den, options.bulk_velocity,
                options.non_dim, options.TestGrad)
            kw.update(jma=jma, kma=kma, ln_prf=lnx, normal=(nx, ny, nz),
                      prf=dict(U=U, V=V, W=W, uu=uu, vv=vv, ww=ww, uv=uv, uw=uw, vw=vw))
            options.nx, options.ny, options.nz = nx, ny, nz      # the plane of the file
            options.ox, options.oy, options.oz = ox, oy, oz
        else:
            U, uu, vv, ww, uw = read_profile(profilefile, options.kma)
            kw["profile1d"] = dict(U=U, uu=uu, vv=vv, ww=ww, uw=uw)
    return _H.DFSetup(**kw)


def read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad):
    """:524-1035 -- see podsgen/prf.py (host setup; the contour plots are not drawn)."""
    from podsgen.prf import read_prf as _read_prf
    return _read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad)


def main(argv=None):
    parser = make_parser()
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) == 0:
        parser.parse_args(["--help"])
    options, args = parser.parse_args(argv)
    s = setup_from_options(options)
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        import torch
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if rank == 0:
        os.makedirs("PODFS", exist_ok=True)
        if options.dt == 0.:
            print("timestep set to: ", s.dt_eff, " seconds")
        else:
            print("Lengthscale in x-direction set to: ", s.lnx, "grid points")
            print("Filter width in x-direction set to: ", s.nfx, "grid points")
    if s.prf is not None and options.profilefile.endswith(".prf"):
        nx, ny, nz = options.nx, options.ny, options.nz          # read_prf's unit normal (:1301)
    else:
        n1 = np.array([options.nx, options.ny, options.nz], dtype=np.float64)
        nx, ny, nz = (n1 / np.sqrt(np.sum(n1 ** 2))).tolist()
    i_d = obj()
    i_d.kma, i_d.jma, i_d.ns, i_d.dt, i_d.nm, i_d.et = s.kma, s.jma, s.ns, s.dt_eff, s.nm, s.et
    i_d.rot = options.rot
    i_d.t_o = [options.ox, options.oy, options.oz]
    i_d.res = options.res
    i_d.n = [nx, ny, nz]
    i_d.num_points = s.P
    i_d.is_POD_var_vec = False
    i_d.grid = pod.make_inflow_plane(i_d)
    i_d.hdf5 = options.hdf5
    i_d.verbose = options.verbose
    i_d.seed = s.seed
    gen = _E.Generator(s, device=local, rank=rank, world=world, dist=dist if world > 1 else None)
    i_d._pods_ctx = gen.ctx
    snap = gen.generate()  # main() step loop :1403-1477 as one device pass
    if options.verbose:  # per-step snapshot planes (:1479-1481), written by rank 0
        A = snap.to_host()
        if world > 1:
            A = gather_row_slabs(dist, s, A)
        if rank == 0:
            for i in range(s.ns):
                i_d.time = i * s.dt_eff
                save_plane(A[:, i], i_d)
        del A
    nmw = s.nm if options.verbose else 0
    pod_res = pod.POD(snap, s.ns, s.P, 3, "false", [], "PODFS/", "false", 1.0e-15, s.nm, nmw, "false",
                      "false", i_d.grid, None, s.dt_eff, "velocity", 1, s.ns, 1, 1, i_d,
                      dist=dist if world > 1 else None)
    mean_local = pod_res.mean.cpu().numpy()
    local_modes = i_d.spatial_modes
    if world > 1:
        # the mean in one gather; the spatial modes streamed to rank 0 one mode at a time as its
        # .prf / HDF5 writers ask for them (SlabColumns), so no host holds all nm modes of the
        # whole inlet (C5: 20 x 3 x 1 M doubles = 0.5 GB) -- the other ranks serve the requests
        mean_field = gather_row_slabs(dist, s, mean_local)
        spatial = SlabColumns(dist, s, local_modes) if rank == 0 else None
    else:
        mean_field, spatial = mean_local, local_modes
    i_d.mean_field = mean_field
    i_d.spatial_modes = spatial
    if rank == 0:
        try:
            pod.fourier_coefficients(i_d)
            pod.pod2prf(i_d)
            if options.hdf5:
                HDF5.write_HDF5(i_d)
        finally:
            if world > 1:
                spatial.close()
    elif world > 1:
        serve_slab_columns(dist, s, local_modes)
    if world > 1:
        dist.barrier()
    return i_d


def _bcast_int(dist, v):
    """Rank 0's integer to every rank (nccl: a device tensor, gloo: a host one)."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([0 if v is None else int(v)], dtype=torch.int64, device=dev)
    dist.broadcast(t, src=0)
    return int(t.item())


class SlabColumns:
    """Rank 0's view of a (3P, m) array whose rows lie in the ranks' row slabs (the spatial modes
    after a multi-rank POD), gathered one column at a time: a[:, i] broadcasts i and gathers that
    column's slabs (gather_row_slabs) while every other rank sits in serve_slab_columns; close()
    releases them.  Only the last column is kept.  np.asarray(a) gathers every column (the whole
    array, as the reference holds it)."""
    streamed = True

    def __init__(self, dist, s, local):
        self.dist, self.s = dist, s
        self.local = np.asarray(local, dtype=np.float64)
        self.shape = (3 * s.P, self.local.shape[1])
        self.ndim = 2
        self._last = (None, None)
        self._open = True

    def column(self, i):
        i = int(i)
        if not -self.shape[1] <= i < self.shape[1]:
            raise IndexError(i)
        i %= self.shape[1]
        if self._last[0] == i:
            return self._last[1]
        if not self._open:
            raise RuntimeError("SlabColumns: the other ranks were released (close())")
        _bcast_int(self.dist, i)
        col = gather_row_slabs(self.dist, self.s, self.local[:, i])
        self._last = (i, col)
        return col

    def __getitem__(self, idx):
        if (isinstance(idx, tuple) and len(idx) == 2 and isinstance(idx[0], slice) and idx[0] == slice(None)
                and isinstance(idx[1], (int, np.integer))):
            return self.column(idx[1])
        return np.asarray(self)[idx]

    def __array__(self, dtype=None, copy=None):
        out = np.empty(self.shape, dtype=np.float64)
        for i in range(self.shape[1]):
            out[:, i] = self.column(i)
        return out if dtype is None else out.astype(dtype)

    def close(self):
        if self._open:
            _bcast_int(self.dist, -1)
            self._open = False


def serve_slab_columns(dist, s, local):
    """The ranks other than 0 while rank 0 reads a SlabColumns: send this rank's slab of each
    requested column until rank 0 closes it."""
    local = np.asarray(local, dtype=np.float64)
    while True:
        i = _bcast_int(dist, None)
        if i < 0:
            return
        gather_row_slabs(dist, s, local[:, i])


def gather_row_slabs(dist, s, local):
    """Reassemble rows [u(P); v(P); w(P)] of a per-rank array from the row slabs of every rank
    onto rank 0 (one tensor gather; other ranks get None).

    local: (3*(j1-j0)*kma, m) rows of this rank's slab (host).  Slabs are sized by
    host.row_slab, so every rank knows every slab's row count; they are zero-padded to the
    largest for the gather.  nccl gathers device tensors, gloo host tensors."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    K, P = s.kma, s.P
    local = np.asarray(local, dtype=np.float64)
    squeeze = local.ndim == 1
    if squeeze:
        local = local[:, None]
    m = local.shape[1]
    slabs = [_H.row_slab(s.jma, r, world) for r in range(world)]
    rows = [3 * (j1 - j0) * K for j0, j1 in slabs]
    if local.shape[0] != rows[rank]:
        raise ValueError("rank %d holds %d rows, its slab has %d" % (rank, local.shape[0], rows[rank]))
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    buf = torch.zeros((max(rows), m), dtype=torch.float64, device=dev)
    buf[:rows[rank]] = torch.from_numpy(local).to(dev)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    if rank != 0:
        return None
    out = np.zeros((3 * P, m))
    for (j0, j1), n, t in zip(slabs, rows, parts):
        f = t[:n].cpu().numpy()
        pl = (j1 - j0) * K
        for c in range(3):
            out[c * P + j0 * K:c * P + j1 * K] = f[c * pl:(c + 1) * pl]
    return out[:, 0] if squeeze else out


if __name__ == "__main__":
    main()

"""PODFS.py -- drop-in for the POD / Fourier-series half of sidbannet/PODS-digital-filter.

Same entry points and i_d contract as the reference's PODFS.py (Python 3):

  POD(A, num_snapshots, num_points, num_components, correct_for_cell_volumes, cell_volume,
      restart_dir, restart_flag, tol_CN, num_modes_trunc, num_modes_to_write,
      test_POD_orthogonality, write_matrices, grid, mean_field, dt, var_name, ifig, N,
      iwindow, stride, i_d)                                        PODFS.py:1294-1393
  calculate_correlation_matrix(...)                               PODFS.py:1451-1464
  sort_eigenvalues(num_snapshots, energy, temporal_modes)         PODFS.py:1430-1447
  write_eigenvalues(num_valid_modes, num_snapshots, energy, fn)   PODFS.py:1409-1427
  write_temporal_modes(...)                                       PODFS.py:1468-1482
  fourier_coefficients(i_d)                                       PODFS.py:1523-1659
  pod2prf(i_d)                                                    PODFS.py:1662-1800
  make_inflow_plane(i_d)                                          PODFS.py:1243-1290

The arithmetic runs on the MI355X through libpodsgen (podsgen/): the correlation matrix
as exact integer products on the int8 matrix cores (residues of the scaled A - mean modulo 16
coprime moduli, one int8 SYRK each, the Chinese remainder theorem back to fp64 with one
rounding; the fp64 MFMA SYRK with PODS_CORR=f64), the eigensolve with pods_syev (all eigenvalues + the nm leading vectors;
torch.linalg.eigh when the full temporal-mode matrix is requested), the spatial modes and
the shifted DFT in HIP kernels.  `A` may be the reference's host array (3P, ns) or the
device-resident snapshots handed over by digitalfilters.main() (podsgen.DeviceSnapshots).
There is no CPU fallback: without the GPU library these functions raise.

Differences from the reference, by design:
  * a symmetric eigensolver replaces dgeev: eigenvalues agree to ~1e-12 of
    lambda_0, eigenvectors up to a per-mode sign (the PODFS reconstruction is invariant);
  * VTK is not used: the inlet geometry is computed analytically with VTK's float32
    rounding chain (make_inflow_plane / cell_centres), and the VTK visualisation writers
    (write_mean_field2, write_spatial_POD_modes_i_d) are not part of this path.
"""
import math
import os

import numpy as np

import nsigproclib as sp
import podsgen
from podsgen import engine as _E
from podsgen.host import num_valid_modes as _num_valid_modes
from podsgen.host import time_axis as _time_axis


# =======================================================================================
# inlet geometry (PODFS.py:1243-1290 without VTK)
# =======================================================================================
def _rotate_wxyz(angle_deg, x, y, z):
    """vtkTransform::RotateWXYZ matrix (quaternion form, double)."""
    if angle_deg == 0.0 or (x == 0.0 and y == 0.0 and z == 0.0):
        return np.eye(4)
    a = math.radians(angle_deg)
    w = math.cos(0.5 * a)
    f = math.sin(0.5 * a) / math.sqrt(x * x + y * y + z * z)
    x, y, z = x * f, y * f, z * f
    ww, wx, wy, wz = w * w, w * x, w * y, w * z
    xx, yy, zz, xy, xz, yz = x * x, y * y, z * z, x * y, x * z, y * z
    m = np.eye(4)
    m[0, 0] = ww + xx - yy - zz
    m[1, 0] = 2.0 * (xy + wz)
    m[2, 0] = 2.0 * (xz - wy)
    m[0, 1] = 2.0 * (xy - wz)
    m[1, 1] = ww - xx + yy - zz
    m[2, 1] = 2.0 * (yz + wx)
    m[0, 2] = 2.0 * (xz + wy)
    m[1, 2] = 2.0 * (yz - wx)
    m[2, 2] = ww - xx - yy + zz
    return m


def _apply(m, pts):
    """A vtkTransformPolyDataFilter pass: float32 points -> double affine -> float32."""
    p = pts.astype(np.float64)
    out = np.empty_like(p)
    for r in range(3):
        out[:, r] = ((m[r, 0] * p[:, 0] + m[r, 1] * p[:, 1]) + m[r, 2] * p[:, 2]) + m[r, 3]
    return out.astype(np.float32)


def plane_points(jma, kma, res, n, rot, t_o):
    """Corner points of the inlet plane as VTK builds them (PODFS.py:1244-1290)."""
    J, K = int(jma), int(kma)
    nx, ny, nz = (float(v) for v in n)
    # vtkPlaneSource defaults, SetResolution(K, J), then SetNormal(1,0,0): a 90 degree
    # rotation about (0,0,1)x(1,0,0) = +y of Origin/Point1/Point2 about the centre (0,0,0)
    R = _rotate_wxyz(90.0, 0.0, 1.0, 0.0)
    O, P1, P2 = (np.array(v, dtype=np.float64) for v in ((-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (-0.5, 0.5, 0.0)))
    O, P1, P2 = (R[:3, :3] @ v + R[:3, 3] for v in (O, P1, P2))
    v1, v2 = P1 - O, P2 - O
    i = np.arange(J + 1, dtype=np.float64)[:, None]
    j = np.arange(K + 1, dtype=np.float64)[None, :]
    t0 = j / K
    t1 = i / J
    pts = np.empty((J + 1, K + 1, 3), dtype=np.float64)
    for r in range(3):
        pts[:, :, r] = (O[r] + t0 * v1[r]) + t1 * v2[r]
    pts = pts.reshape(-1, 3).astype(np.float32)
    s1 = 0.0
    s2 = res * float(J) * float(J) / (float(J) - 1)
    s3 = res * float(K) * float(K) / (float(K) - 1)
    pts = _apply(np.diag([s1, s2, s3, 1.0]), pts)
    alpha = np.arccos(nx) * 180 / np.pi
    beta = np.arctan2(nz, ny) * 180 / np.pi
    pts = _apply(_rotate_wxyz(alpha, 0, -nz, ny), pts)
    pts = _apply(_rotate_wxyz(beta + rot, nx, ny, nz), pts)
    T = np.eye(4)
    T[:3, 3] = t_o
    return _apply(T, pts)


def cell_centres(jma, kma, res, n=(1.0, 0.0, 0.0), rot=0.0, t_o=(0.0, 0.0, 0.0)):
    """vtkCellCenters of the plane: quad (i, j) -> point id i*(K+1)+j, +1, +K+2, +K+1,
    parametric centre = sum of 0.25*corner in that order (double), stored float32.
    Returns (J*K, 3) float64 holding the float32 values (cell id = j*K + k)."""
    J, K = int(jma), int(kma)
    pts = plane_points(J, K, res, n, rot, t_o).astype(np.float64).reshape(J + 1, K + 1, 3)
    c = np.zeros((J, K, 3))
    for corner in (pts[:-1, :-1], pts[:-1, 1:], pts[1:, 1:], pts[1:, :-1]):
        c = c + corner * 0.25
    return c.astype(np.float32).reshape(J * K, 3).astype(np.float64)


class InletGrid(object):
    """Stand-in for the vtkPolyData the reference passes around as `grid`: the cell
    centres are all the PODFS path reads from it (PODFS.py:1699-1704)."""

    def __init__(self, points):
        self.points = points

    def GetNumberOfCells(self):
        return self.points.shape[0]


def make_inflow_plane(i_d):
    return InletGrid(cell_centres(i_d.jma, i_d.kma, i_d.res, i_d.n, getattr(i_d, "rot", 0.0),
                                  getattr(i_d, "t_o", (0.0, 0.0, 0.0))))


# =======================================================================================
# POD
# =======================================================================================
def _ctx_for(A, i_d=None):
    if isinstance(A, _E.DeviceSnapshots):
        return A
    ctx = getattr(i_d, "_pods_ctx", None) if i_d is not None else None
    return _E.load_snapshots(A, ctx=ctx)


def sort_eigenvalues(num_snapshots, energy, temporal_modes):
    """PODFS.py:1430-1447 (in place): NaN -> -1e10 with the mode zeroed; sort
    (value, index) descending; columns permuted from a .real copy."""
    energy_sorted = np.zeros(num_snapshots, dtype=np.float64)
    idx = np.arange(num_snapshots)
    for k in range(num_snapshots):
        if math.isnan(energy[k].real) or math.isnan(energy[k].imag):
            energy_sorted[k] = -1.0e10
            temporal_modes[:, k] = 0.0
        else:
            energy_sorted[k] = energy[k].real
    order = sorted(zip(energy_sorted, idx), reverse=True)
    energy[0:num_snapshots] = [o[0] for o in order]
    t0 = np.array(temporal_modes[0:num_snapshots, 0:num_snapshots].real, copy=True)
    for k in range(num_snapshots):
        temporal_modes[0:num_snapshots, k] = t0[0:num_snapshots, order[k][1]]


def calculate_correlation_matrix(num_snapshots, num_points, num_components, correct_for_cell_volumes,
                                 cell_volume, A, C):
    """C = A^T A / ns on the GPU (A already mean-subtracted, PODFS.py:1451-1464).
    The cell-volume-weighted branch scales each row by sqrt(volume) (same sum, fp64)."""
    A = np.asarray(A, dtype=np.float64)[:, 0:num_snapshots]
    if correct_for_cell_volumes == "true":
        w = np.sqrt(np.tile(np.asarray(cell_volume, dtype=np.float64), num_components))
        A = A * w[:, None]
    elif correct_for_cell_volumes != "false":
        raise ValueError("correct_for_cell_volumes must be 'true' or 'false'")
    snap = _E.load_snapshots(A)
    ctx = snap.ctx
    podsgen.check(ctx.lib.pods_set_mean(ctx.h, None), "pods_set_mean")
    import torch
    Cd = torch.empty((num_snapshots, num_snapshots), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_corr(ctx.h, _E.ptr(Cd), 1), "pods_corr")
    C[:, :] = Cd.cpu().numpy()


def write_eigenvalues(num_valid_modes, num_snapshots, energy, filename):
    """PODFS.py:1409-1427."""
    energy = np.asarray(energy).real
    cum = np.zeros(num_valid_modes, dtype=np.float64)
    cum[0] = energy[0]
    for i in range(1, num_valid_modes):
        cum[i] = cum[i - 1] + energy[i]
    total = cum[num_valid_modes - 1]
    with open(filename, "w") as f:
        f.write("#\n")
        f.write("# mode, energy, cumulative, percenterage energy, percentage cumulative, condition number (absolute value if negative)\n")
        f.write("#\t\tNote: cummulative energies are set to zero after first negative energy")
        f.write("#\n")
        for i in range(num_valid_modes):
            f.write("%4.1d %18.10e %18.10e %18.10e %18.10e %18.10e\n" % (
                i + 1, energy[i], cum[i], energy[i] / total * 100.0, cum[i] / total * 100.0,
                math.sqrt(energy[i] / energy[0])))
        for i in range(num_valid_modes, num_snapshots):
            f.write("%4.1d %18.10e %18.10e %18.10e %18.10e %18.10e\n" % (
                i + 1, energy[i], 0.0, energy[i] / total * 100.0, 0.0, math.sqrt(abs(energy[i] / energy[0]))))


def write_temporal_modes(num_valid_modes, num_snapshots, dt, temporal_modes, rdir):
    """PODFS.py:1468-1482 (verbose output)."""
    for j in range(num_valid_modes):
        fn = rdir + "POD.temporal_mode_" + "%04d" % (j + 1) + ".dat"
        with open(fn, "w") as f:
            f.write("#\n# time, amplitude\n#\n")
            for i in range(num_snapshots):
                f.write("%18.10e %18.10e\n" % (i * dt, temporal_modes[i, j].real))


def POD(A, num_snapshots, num_points, num_components, correct_for_cell_volumes, cell_volume,
        restart_dir, restart_flag, tol_CN, num_modes_trunc, num_modes_to_write,
        test_POD_orthogonality, write_matrices, grid, mean_field, dt, var_name, ifig, N,
        iwindow, stride, i_d, dist=None):
    """PODFS.py:1294-1393.  `A` is mean-subtracted in the reference call (digitalfilters.py
    :1492-1500); a DeviceSnapshots handle carries the uncentred device matrix, which run_pod
    centres in place (pods_center, the same subtraction) after the bit-exact mean."""
    if correct_for_cell_volumes != "false":
        raise NotImplementedError("the GPU POD path implements correct_for_cell_volumes='false' "
                                  "(the only value digitalfilters.main passes); use "
                                  "calculate_correlation_matrix for the weighted form")
    snap = _ctx_for(A, i_d)
    # The full (ns x ns) temporal-mode matrix is only consumed by the verbose outputs
    # (write_temporal_modes, PSD plots); the compressed PODFS output needs T[:, :nm].
    full = getattr(i_d, "full_temporal_modes", bool(getattr(i_d, "verbose", False)))
    if isinstance(A, _E.DeviceSnapshots):
        res = _E.run_pod(snap, num_modes_trunc, tol_CN=tol_CN, dist=dist, full_temporal=full)
    else:
        # A is already centred by the caller: zero mean, then the same kernels
        ctx = snap.ctx
        res = _run_pod_centred(snap, num_modes_trunc, tol_CN, full)
    i_d._pods = res
    i_d._pods_ctx = snap.ctx
    if restart_dir and (dist is None or not dist.is_initialized() or dist.get_rank() == 0):
        os.makedirs(restart_dir, exist_ok=True)
        write_eigenvalues(res.num_valid, num_snapshots, res.energy, restart_dir + "POD.eigenvalues.dat")
    T = res.T.cpu().numpy() if res.T is not None else None
    rank0 = dist is None or not dist.is_initialized() or dist.get_rank() == 0
    # verbose temporal modes (:1352-1356): rank 0 holds the full (ns, ns) T; the others only
    # the broadcast T[:, :nm]
    if getattr(i_d, "verbose", False) and T is not None and restart_dir and rank0:
        write_temporal_modes(res.num_valid, num_snapshots, dt, T, restart_dir)
    i_d.temporal_modes = T
    i_d.spatial_modes = res.phi.cpu().numpy()
    i_d.nm = res.nm
    i_d.energy = res.energy
    i_d.num_valid_modes = res.num_valid
    return res


def _run_pod_centred(snap, nm, tol_CN, full):
    ctx = snap.ctx
    podsgen.check(ctx.lib.pods_set_mean(ctx.h, None), "pods_set_mean")
    # run_pod recomputes the (zero-mean) mean via pods_mean; for an already-centred A the
    # pairwise mean is ~0 but not exactly 0, so use the zero mean explicitly here
    import torch
    ns = snap.ns
    C = torch.empty((ns, ns), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_corr(ctx.h, _E.ptr(C), 1), "pods_corr")
    lam_desc, nvalid, nmt, T = _E.eigen_modes(ctx, C, ns, nm, tol_CN, full)
    ncols = T.shape[1]
    phi = torch.empty((snap.rowlen, max(nmt, 1)), dtype=torch.float64, device="cuda")
    if nmt > 0:
        podsgen.check(ctx.lib.pods_spatial_modes(ctx.h, _E.ptr(T), ncols,
                                                 _E.ptr(np.ascontiguousarray(lam_desc[:nmt])), nmt,
                                                 _E.ptr(phi)), "pods_spatial_modes")
    mean = torch.zeros(snap.rowlen, dtype=torch.float64, device="cuda")
    return _E.PODResult(energy=lam_desc, num_valid=nvalid, nm=nmt, mean=mean, T=T, phi=phi[:, :nmt])


# =======================================================================================
# Fourier-series compression
# =======================================================================================
def podfs_dat_text(num_modes, period, c, c_ind, c_count, num_fcs):
    s = [str(num_modes), "\n" + str(period)]
    for i in range(num_modes):
        s.append("\n" + str(i + 1) + "\t" + str(c_count[i]))
    for i in range(num_modes):
        for j in range(c_count[i]):
            n = c_ind[i, j]
            s.append("\n" + str(n - num_fcs // 2) + "\t" + str(c[n, i].real) + "\t" + str(c[n, i].imag))
    return "".join(s)


def fourier_coefficients(i_d):
    """PODFS.py:1523-1659: shifted DFT of every kept temporal mode (GPU), ranking by |c|
    and energy count (host), i_d.period / N_FC / FC, and ./PODFS/PODFS.dat."""
    ns = i_d.ns
    nm = i_d.nm
    res = getattr(i_d, "_pods", None)
    ctx = getattr(i_d, "_pods_ctx", None)
    import torch
    if res is not None and res.T is not None:
        T = res.T
    else:
        T = torch.from_numpy(np.ascontiguousarray(np.asarray(i_d.temporal_modes, dtype=np.float64)[:, :nm])).cuda()
        ctx = ctx or _E.Context(0)
    fo = _E.run_fourier(ctx, T, nm, ns, i_d.dt, i_d.et)
    i_d.c = fo.c
    i_d.c_ind = fo.c_ind
    if i_d.hdf5:
        i_d.period = fo.period
        i_d.N_FC = fo.c_count
        i_d.FC = fo.FC
    rdir = "./PODFS/"
    os.makedirs(rdir, exist_ok=True)
    with open(rdir + "PODFS.dat", "w") as f:
        f.write(podfs_dat_text(nm, fo.period, fo.c, fo.c_ind, fo.c_count, ns))
    i_d.period = fo.period
    return fo


# =======================================================================================
# .prf output (PODFS.py:1662-1800)
# =======================================================================================
def _prf_header(name, n, rhs):
    return ("# " + name + " # name of the profile\n"
            "# turbulence model, none\n"
            "# plane normal and translation " + str(n[0]) + "\t" + str(n[1]) + "\t" + str(n[2]) + "\t" + str(rhs) + "\n"
            "type, xyz # type of profile (rad or xyz)\n"
            "localcs,origin,0,0,0 # origin of local coordinate system\n"
            "localcs,xaxis,1,0,0 # x axis direction of local coordinate system\n"
            "localcs,yaxis,0,1,0 # y axis direction of local coordinate system\n"
            "localcs,zaxis,0,0,1 # z axis direction of local coordinate system\n"
            "tolerance, 1.00E-08 # tolerance\n"
            "scale,1,1,1,1,1,1 # scaling factors\n"
            "data,x,y,z,u,v,w\n")


def _prf_rows(points, u):
    return "".join(sp.str(points[j, 0]) + "," + sp.str(points[j, 1]) + "," + sp.str(points[j, 2]) + "," +
                   sp.str(u[j, 0]) + "," + sp.str(u[j, 1]) + "," + sp.str(u[j, 2]) + "\n"
                   for j in range(points.shape[0]))


class ModeStack:
    """i_d.modes of the reference (mode i = [x y z | u v w] per point, PODFS.py:1745-1747) without
    the (nm, P, 6) array: mode i is built from the grid points and column i of the spatial modes
    when asked for.  np.asarray(stack) still gives the whole array."""

    def __init__(self, points, spatial_modes, nm):
        self.points = np.asarray(points, dtype=np.float64)
        self.spatial = spatial_modes
        self.nm = int(nm)

    def __len__(self):
        return self.nm

    @property
    def shape(self):
        return (self.nm, self.points.shape[0], 6)

    def __getitem__(self, i):
        if not isinstance(i, (int, np.integer)):
            return np.asarray(self)[i]
        if not -self.nm <= i < self.nm:
            raise IndexError(i)
        i = int(i) % self.nm
        P = self.points.shape[0]
        m = np.empty((P, 6), dtype=np.float64)
        m[:, 0:3] = self.points
        m[:, 3:] = np.asarray(self.spatial[:, i]).reshape((P, 3), order="F")
        return m

    def __array__(self, dtype=None, copy=None):
        a = np.stack([self[i] for i in range(self.nm)]) if self.nm else np.zeros(self.shape)
        return a if dtype is None else a.astype(dtype, copy=False)


def pod2prf(i_d):
    """PODFS_mean.prf and PODFS_mode_####.prf; i_d.mean / i_d.modes for the HDF5 writer."""
    rdir = "./PODFS/"
    os.makedirs(rdir, exist_ok=True)
    num_modes = i_d.nm
    num_points = i_d.num_points
    i_d.turbulence_model = "none"
    n = i_d.n
    points = i_d.grid.points
    if i_d.hdf5:
        i_d.mean = np.zeros((num_points, 6), dtype=np.float64)
        # the reference fills a (nm, P, 6) array here (PODFS.py:1671-1672, 1 GB at C5); the
        # writer only ever needs one mode at a time, so the modes are assembled on demand
        i_d.modes = ModeStack(points, i_d.spatial_modes, num_modes)
    u = np.asarray(i_d.mean_field).reshape((num_points, 3), order="F")
    if i_d.hdf5:
        i_d.mean[:, 0:3] = points
        i_d.mean[:, 3:] = u
    # the reference resets the translation before writing (PODFS.py:1669), so the plane
    # rhs of PODFS_mean.prf is (0+0)*n1 + (0+0)*n2 + (0+0)*n3 (:1717) whatever --ox/--oy/--oz
    i_d.t_o = np.array([0, 0, 0])
    rhs = (0 + i_d.t_o[0]) * n[0] + (0 + i_d.t_o[1]) * n[1] + (0 + i_d.t_o[2]) * n[2]
    with open(rdir + "PODFS_mean.prf", "w") as f:
        f.write(_prf_header("PODFS_mean", n, rhs))
        f.write(_prf_rows(points, u))
    for i in range(num_modes):
        counter = "%4.4i" % (i + 1)
        um = i_d.spatial_modes[:, i].reshape((num_points, 3), order="F")
        with open(rdir + "PODFS_mode_" + counter + ".prf", "w") as f:
            f.write(_prf_header("PODFS_mode_" + counter, n, 0 * n[0] + 0 * n[1] + 0 * n[2]))
            f.write(_prf_rows(points, um))

#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by RUNNING THE REFERENCE'S OWN CODE.

This script is test infrastructure.  It runs only in the build container (it needs
/root/reference, which never exists on the GPU box) and its outputs are plain data
(.npz arrays and the reference's own text output files).  Nothing from the reference
is copied into the repository: the source text is read at run time, translated in
memory and discarded.

How the reference is executed
-----------------------------
The reference (sidbannet/PODS-digital-filter) is Python 2 and cannot be imported by
this interpreter (mixed tabs, print statements).  We therefore

  1. read digitalfilters.py / PODFS.py as text and apply Python 2's tab rule
     (tabs -> next multiple of 8) to the leading indentation only, so tabs inside
     string literals survive (PODFS.py:1421 writes '#\\t\\tNote');
  2. run lib2to3 over the module text (print/except/zip/... fixers);
  3. parse the result with `ast` and pull out ONLY the pure numpy/scipy functions on
     the hot path -- no module-level imports of vtk/h5py/matplotlib are executed, and
     no stand-ins for those libraries are written;
  4. apply the Python-2 / numpy-1.x semantic patches listed in SEMANTIC_PATCHES
     (integer division, np.int, numpy-1.x float32->float64 promotion);
  5. exec those functions in a namespace holding numpy, scipy.signal and math.

Functions executed from the reference (file:line):
  digitalfilters.py:73-89    calccoeff
  digitalfilters.py:100-140  filter3DSciPy1D
  digitalfilters.py:143-178  adapt1d
  digitalfilters.py:180-231  adapt2prf
  digitalfilters.py:233-485  adapt2d (needs scipy.interpolate in the namespace)
  digitalfilters.py:524-1035 read_prf (plots dropped, see DROP_LINES)
  digitalfilters.py:1038-1062 build_profile
  digitalfilters.py:1064-1131 prof_rotation_matrix / rotate_velocity
  PODFS.py:1409-1427          write_eigenvalues
  PODFS.py:1430-1447          sort_eigenvalues
  PODFS.py:1451-1464          calculate_correlation_matrix
  PODFS.py:1523-1659          fourier_coefficients (writes PODFS/PODFS.dat)
  PODFS.py:1468-1482          write_temporal_modes (verbose output)
  nsigproclib_no_mpi.py:10-68 fct_welch (verbose PSD of a temporal mode)

main() (digitalfilters.py:1134-1510) and POD() (PODFS.py:1294-1393) are monolithic and
reach VTK (make_inflow_plane, write_mean_field2); their glue lines (RNG draws, roll,
snapshot assembly, mean subtraction, valid-mode count, temporal scaling, spatial modes)
are replayed below line by line with the same numpy calls, each citing its line.

Run:  python tests/golden/make_golden.py      (writes tests/golden/*.npz, *.dat)
"""
import ast
import contextlib
import io
import math
import os
import re
import shutil
import sys
import tempfile
import warnings

import numpy as np
import scipy.signal as scSig

REF = os.environ.get("PODS_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

# (function name) -> list of (old, new) text patches, each must apply exactly as listed.
SEMANTIC_PATCHES = {
    # Python 2 integer division (PODFS.py:1565,1607,1636,1657)
    "fourier_coefficients": [
        ("num_fcs/2", "num_fcs//2"),
        # numpy-1.x promotion: np.float32 (*|+) python float -> float64 (PODFS.py:1588-1593)
        ("energy_sum = np.sum(np.abs(c[:,i]))", "energy_sum = np.float64(np.sum(np.abs(c[:,i])))"),
        ("energy += np.abs(c[c_ind[i,c_count[i]],i])", "energy += np.float64(np.abs(c[c_ind[i,c_count[i]],i]))"),
    ],
    # np.int was removed in numpy 1.24 (PODFS.py:1432)
    "sort_eigenvalues": [("dtype=np.int)", "dtype=int)")],
    # Python 2 integer division (digitalfilters.py:1121)
    "rotate_velocity": [("len(A)/3", "len(A)//3")],
}

DF_FUNCS = ["calccoeff", "filter3DSciPy1D", "adapt1d", "adapt2prf", "adapt2d", "build_profile",
            "prof_rotation_matrix", "rotate_velocity", "read_prf", "read_profile"]
# read_prf (digitalfilters.py:524-1035): Python 2 `3/2 == 1` (:758, :767, :779, :788), and its
# nplotlib contour plots (:851-872, :1011-1022; VTK/matplotlib, side effects only) dropped
# line by line (regex below) -- nothing they draw feeds the returned profile.
SEMANTIC_PATCHES["read_prf"] = [("(3/2)", "(3//2)")]
DROP_LINES = {"read_prf": r"^(\s*)plt\.(contourf|close)\(.*$"}
PROFILES_2D = ("double-hyperbolic-tangent", "circular-hyperbolic-tangent", "ring-hyperbolic-tangent")
POD_FUNCS = ["write_eigenvalues", "sort_eigenvalues", "calculate_correlation_matrix",
             "fourier_coefficients", "write_temporal_modes", "save_plane"]
# save_plane (PODFS.py:854-887): its VTK cell-centre lookup (:856-861) is the only VTK use;
# the points are handed in instead (VTK geometry -> given/analytic points).
SEMANTIC_PATCHES["save_plane"] = [
    ("cc = vtk.vtkCellCenters()", "pass"),
    ("cc.SetInputData(i_d.grid)", "pass"),
    ("cc.VertexCellsOn()", "pass"),
    ("cc.Update()", "pass"),
    ("points = VN.vtk_to_numpy(cc.GetOutput().GetPoints().GetData())", "points = i_d.grid_points"),
    ("npt = cc.GetOutput().GetNumberOfPoints()", "npt = points.shape[0]"),
]
SIG_FUNCS = ["fct_welch"]
# nsigproclib_no_mpi.str (:880-882, '%0.12f') -- kept in its own namespace `sp` (PODFS.py
# imports the module as sp), so the builtin str the writers also call is not shadowed.
SP_FUNCS = ["str"]
# Python 2 integer division in the frequency axis (nsigproclib_no_mpi.py:53): -N/2 == (-N)//2
SEMANTIC_PATCHES["fct_welch"] = [("np.linspace(-N/2,N/2-1,N)", "np.linspace(-N//2,N//2-1,N)")]


def _expand_indentation(text):
    """Python 2's tab rule (tabs to the next multiple of 8) applied to the leading
    indentation of each logical line only.  Tabs inside string literals (e.g. the
    '#\\t\\tNote' header of PODFS.py:1421) and inside triple-quoted blocks are kept."""
    out = []
    in_triple = None
    for line in text.splitlines(keepends=True):
        if in_triple is None:
            m = re.match(r"[ \t]*", line)
            line = m.group(0).expandtabs(8) + line[m.end():]
        # track triple-quoted blocks opened/closed on this line (the reference's docstrings)
        pos = 0
        while True:
            if in_triple is None:
                hits = [(line.find(q, pos), q) for q in ('"""', "'''")]
                hits = [h for h in hits if h[0] >= 0]
                if not hits:
                    break
                at, q = min(hits)
                in_triple, pos = q, at + 3
            else:
                at = line.find(in_triple, pos)
                if at < 0:
                    break
                in_triple, pos = None, at + 3
        out.append(line)
    return "".join(out)


def _translate(path):
    from lib2to3 import refactor
    with open(path, "r") as f:
        src = _expand_indentation(f.read())
    if not src.endswith("\n"):
        src += "\n"
    fixers = refactor.get_fixers_from_package("lib2to3.fixes")
    tool = refactor.RefactoringTool(fixers)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return str(tool.refactor_string(src, os.path.basename(path)))


def _extract(src, names):
    tree = ast.parse(src)
    lines = src.splitlines(keepends=True)
    out = {}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            out[node.name] = "".join(lines[node.lineno - 1:node.end_lineno])
    missing = set(names) - set(out)
    assert not missing, missing
    return out


def load_reference():
    from scipy import interpolate
    ns = {"np": np, "scSig": scSig, "math": math, "Pi": np.pi, "linalg": np.linalg,
          "interpolate": interpolate, "sys": sys}
    sp_ns = {"np": np}
    ns["sp"] = type("sp", (), {})
    for name, text in _extract(_translate(os.path.join(REF, "nsigproclib_no_mpi.py")), SP_FUNCS).items():
        exec(compile(text, "<reference:sp.%s>" % name, "exec"), sp_ns)
        setattr(ns["sp"], name, staticmethod(sp_ns[name]))
    for path, names in ((os.path.join(REF, "digitalfilters.py"), DF_FUNCS),
                        (os.path.join(REF, "PODFS.py"), POD_FUNCS),
                        (os.path.join(REF, "nsigproclib_no_mpi.py"), SIG_FUNCS)):
        funcs = _extract(_translate(path), names)
        for name, text in funcs.items():
            for old, new in SEMANTIC_PATCHES.get(name, []):
                assert old in text, (name, old)
                text = text.replace(old, new)
            if name in DROP_LINES:
                import re
                text, ndrop = re.subn(DROP_LINES[name], r"\1pass", text, flags=re.M)
                assert ndrop == 34, ndrop
            exec(compile(text, "<reference:%s>" % name, "exec"), ns)
    return ns


class Obj(object):
    pass


def run_reference_pipeline(ref, *, jma, kma, ns, seed, lengthscale=3.0, fwidth=2.0, dt=0.0,
                           res=0.1, bulk_velocity=1.0, u_dash=0.02, nm=20, et=0.9,
                           normal=(1.0, 0.0, 0.0), prf=None, workdir=None,
                           mean_profile="hyperbolic-tangent", inner_d=0.5, ln_prf=None,
                           profile_text=None):
    """Replay digitalfilters.py main() (:1244-1510) + PODFS.POD (:1294-1393) with the
    reference's own functions.  prf=None -> built profile (adapt1d, or adapt2d for the 2-D
    mean profiles, + rotation); prf=dict(U,V,W,uu,vv,ww,uv,uw,vw) of (jma,kma) arrays ->
    adapt2prf path (no rotation)."""
    out = {}
    np.random.seed(seed)                                  # extension: reference never seeds
    lnx = lny = lnz = lengthscale                         # :1262-1264
    nf = int(math.ceil(fwidth * lengthscale))             # :1267
    nfx = nfy = nfz = nf
    if ln_prf is not None:                                # :1301-1305 (read_prf's lnx)
        lnx = lny = lnz = ln_prf
    n1 = np.asarray(normal, dtype=np.float64)
    nx = n1[0] / np.sqrt(n1[0]**2 + n1[1]**2 + n1[2]**2)  # :1276-1278
    ny = n1[1] / np.sqrt(n1[0]**2 + n1[1]**2 + n1[2]**2)
    nz = n1[2] / np.sqrt(n1[0]**2 + n1[1]**2 + n1[2]**2)
    V = W = 0
    if profile_text is not None:                          # :1306-1307 (-P profile.dat)
        pdir = tempfile.mkdtemp(prefix="pods_profile_")
        try:
            with open(os.path.join(pdir, "profile.dat"), "w") as f:
                f.write(profile_text)
            with contextlib.redirect_stdout(io.StringIO()):
                U, uu, vv, ww, uw = ref["read_profile"](os.path.join(pdir, "profile.dat"), kma)
        finally:
            shutil.rmtree(pdir)
    elif prf is None:
        U, uu, vv, ww, uw = ref["build_profile"](mean_profile, "top-hat",
                                                 bulk_velocity, u_dash, kma)      # :1305
    else:
        U, V, W = prf["U"], prf["V"], prf["W"]
        uu, vv, ww, uv, uw, vw = (prf[k] for k in ("uu", "vv", "ww", "uv", "uw", "vw"))
    if dt == 0.:                                          # :1306-1309
        flag = np.where(U**2 + V**2 + W**2 != 0)
        dt = res / np.mean(U[flag])
    else:                                                 # :1310-1317
        flag = np.where(U**2 + V**2 + W**2 != 0)
        dt1 = res / np.mean(U[flag])
        factor = dt1 / dt
        lnx = factor * lnx
        nfx = int(math.ceil(float(fwidth) * lnx))
    pdfr = np.sqrt(3.0)                                   # :1340
    if prf is None:                                       # :1343-1350
        for k in range(0, kma):
            if uu[k] < 0.0: uu[k] = 0.0
            if vv[k] < 0.0: vv[k] = 0.0
            if ww[k] < 0.0: ww[k] = 0.0
    a = np.zeros((1, nfx * 2 + 1, nfy * 2 + 1, nfz * 2 + 1))
    xu = np.random.uniform(low=-pdfr, high=pdfr, size=(nfx*2+1, nfy*2+jma, nfz*2+kma))  # :1361
    xv = np.random.uniform(low=-pdfr, high=pdfr, size=(nfx*2+1, nfy*2+jma, nfz*2+kma))
    xw = np.random.uniform(low=-pdfr, high=pdfr, size=(nfx*2+1, nfy*2+jma, nfz*2+kma))
    yu = np.zeros((jma, kma)); yv = np.zeros((jma, kma)); yw = np.zeros((jma, kma))
    A = np.zeros((jma * kma * 3, ns), dtype=np.float64)   # :1397
    filt = []
    for i in range(ns):                                   # :1403
        ref["filter3DSciPy1D"](xu, yu, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz)   # :1440
        ref["filter3DSciPy1D"](xv, yv, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz)
        ref["filter3DSciPy1D"](xw, yw, a, jma, kma, lnx, lny, lnz, nfx, nfy, nfz)
        if i < 3:
            filt.append(np.stack([yu.copy(), yv.copy(), yw.copy()]))
        if prf is not None:                               # :1445-1451
            ref["adapt2prf"](yu, yv, yw, U, V, W, uu, vv, ww, uv, uw, vw, jma, kma)
        elif mean_profile in PROFILES_2D:
            ref["adapt2d"](yu, yv, yw, U, uu, vv, ww, uw, jma, kma, mean_profile, inner_d)
        else:
            ref["adapt1d"](yu, yv, yw, U, uu, vv, ww, uw, jma, kma)
        xu = np.roll(xu, -1, axis=0); xv = np.roll(xv, -1, axis=0); xw = np.roll(xw, -1, axis=0)
        xu[nfx*2, :, :] = np.random.uniform(low=-pdfr, high=pdfr, size=(nfy*2+jma, nfz*2+kma))
        xv[nfx*2, :, :] = np.random.uniform(low=-pdfr, high=pdfr, size=(nfy*2+jma, nfz*2+kma))
        xw[nfx*2, :, :] = np.random.uniform(low=-pdfr, high=pdfr, size=(nfy*2+jma, nfz*2+kma))
        A[0:jma*kma, i] = yu.reshape(jma*kma)             # :1471-1473
        A[jma*kma:2*jma*kma, i] = yv.reshape(jma*kma)
        A[2*jma*kma:3*jma*kma, i] = yw.reshape(jma*kma)
        if prf is None and profile_text is None:          # :1476-1477 (profilefile == 'none')
            A[:, i] = ref["rotate_velocity"](A[:, i], nx, ny, nz)
    out["A_raw"] = A.copy()
    out["filtered_first_steps"] = np.stack(filt)
    mean_field = np.mean(A, 1)                            # :1492
    for j in range(0, ns):
        A[:, j] = A[:, j] - mean_field[:]
    out["mean_field"] = mean_field
    # ---- PODFS.POD (:1294-1393), correct_for_cell_volumes='false', tol_CN=1e-15 --------------
    num_points = jma * kma
    C = np.array(np.zeros((ns, ns), dtype=np.float64))
    ref["calculate_correlation_matrix"](ns, num_points, 3, "false", [], A, C)    # :1303
    out["C"] = C.copy()
    energy, temporal_modes = np.linalg.eig(C)             # :1309
    out["eig_is_real"] = np.array(np.isrealobj(energy))
    ref["sort_eigenvalues"](ns, energy, temporal_modes)   # :1310
    tol_CN = 1.0e-15
    num_valid_modes = 0                                   # :1312-1317
    while ((energy[num_valid_modes].real / energy[0].real > pow(tol_CN, 2.0)) and
           (num_valid_modes < ns - 2) and (energy[num_valid_modes].real > 0.0)):
        num_valid_modes += 1
        if ((energy[num_valid_modes].real / energy[0].real > pow(tol_CN, 2.0)) and
                (energy[num_valid_modes].real > 0.0)):
            num_valid_modes += 1
    num_modes_trunc = nm
    if (num_modes_trunc < 0) or (num_modes_trunc > num_valid_modes):           # :1319
        num_modes_trunc = num_valid_modes
    for j in range(0, num_valid_modes):                   # :1323-1325
        temporal_mode_mag = sum(temporal_modes[:, j].real * temporal_modes[:, j].real) / ns
        temporal_modes[:, j] = temporal_modes[:, j] * np.sqrt(energy[j].real / temporal_mode_mag)
    energy_trunc_inv = np.diag(np.ones(num_modes_trunc) / energy[0:num_modes_trunc].real, 0)   # :1331
    spatial = np.dot(np.dot(A[:, 0:ns], temporal_modes[:, 0:num_modes_trunc].real),
                     energy_trunc_inv) / ns              # :1333
    out.update(energy=np.asarray(energy), num_valid_modes=np.array(num_valid_modes),
               nm=np.array(num_modes_trunc), temporal_modes=np.asarray(temporal_modes)[:, :num_modes_trunc],
               spatial_modes=spatial, dt=np.array(dt), nfx=np.array(nfx), nfy=np.array(nfy),
               nfz=np.array(nfz), lnx=np.array(lnx), lny=np.array(lny), lnz=np.array(lnz),
               taps_x=ref["calccoeff"](np.zeros(2*nfx+1), nfx, lnx),
               taps_y=ref["calccoeff"](np.zeros(2*nfy+1), nfy, lny),
               taps_z=ref["calccoeff"](np.zeros(2*nfz+1), nfz, lnz))
    # ---- fourier_coefficients (:1523-1659), run in a scratch dir (writes ./PODFS/PODFS.dat) ----
    i_d = Obj()
    i_d.hdf5 = True; i_d.ns = ns; i_d.dt = dt; i_d.nm = num_modes_trunc; i_d.et = et
    i_d.temporal_modes = temporal_modes; i_d.verbose = False
    cwd = os.getcwd()
    tmp = workdir or tempfile.mkdtemp(prefix="pods_golden_")
    os.makedirs(os.path.join(tmp, "PODFS"), exist_ok=True)
    try:
        os.chdir(tmp)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            _stdout = sys.stdout
            sys.stdout = io.StringIO()
            try:
                ref["fourier_coefficients"](i_d)
                ref["write_eigenvalues"](num_valid_modes, ns, energy, "PODFS/POD.eigenvalues.dat")
            finally:
                sys.stdout = _stdout
        with open("PODFS/PODFS.dat") as f:
            out["podfs_dat"] = np.array(f.read())
        with open("PODFS/POD.eigenvalues.dat") as f:
            out["eigenvalues_dat"] = np.array(f.read())
    finally:
        os.chdir(cwd)
        if workdir is None:
            shutil.rmtree(tmp, ignore_errors=True)
    out.update(period=np.array(i_d.period), N_FC=np.asarray(i_d.N_FC), FC=np.asarray(i_d.FC))
    return out


def synthetic_prf(jma, kma, seed):
    """Deterministic inhomogeneous profile for the adapt2prf path (SURVEY.md 8(d) C5 style)."""
    r = np.random.RandomState(seed)
    y = np.linspace(-0.5, 0.5, jma)[:, None]
    z = np.linspace(-0.5, 0.5, kma)[None, :]
    U = 0.5 * (1.0 + np.tanh(10.0 * (0.5 - np.sqrt(y**2 + z**2)))) + 0.05
    V = 0.01 * np.sin(3.0 * y) * np.ones_like(z)
    W = 0.01 * np.cos(2.0 * z) * np.ones_like(y)
    s = (0.02 * U)**2
    rho = 0.4 * np.sin(2.0 * y + 3.0 * z) * np.ones_like(U)
    uu = s.copy(); vv = 1.1 * s; ww = 0.9 * s
    uv = rho * np.sqrt(uu * vv); uw = -0.5 * rho * np.sqrt(uu * ww); vw = 0.3 * rho * np.sqrt(vv * ww)
    uu[0, 0] = 0.0                                        # exercise the a00<=0 guard
    vv[1, 1] = 0.25 * uv[1, 1] ** 2 / max(uu[1, 1], 1e-300)  # exercise a10^2>R11 clamp
    del r
    return dict(U=U, V=V, W=W, uu=uu, vv=vv, ww=ww, uv=uv, uw=uw, vw=vw)


CASES = {
    # name: kwargs                                                            (why)
    "c1_32x32x64": dict(jma=32, kma=32, ns=64, seed=12345),                  # BASELINE config 1
    "cli_10x11x5": dict(jma=10, kma=11, ns=5, seed=7),                       # quickstart -n 5, CLI default grid
    "odd_12x9x17_aniso": dict(jma=12, kma=9, ns=17, seed=3, dt=0.05),        # odd ns, -t => nfx != nfy
    "prf_8x12x9": dict(jma=8, kma=12, ns=9, seed=11, prf="synthetic"),       # adapt2prf path
    "rot_6x7x6": dict(jma=6, kma=7, ns=6, seed=5, normal=(1.0, 1.0, 0.5)),   # non-identity rotation
    # adapt2d paths (digitalfilters.py:233-485), built profile + rotation as main() does
    "dtanh_9x12x7": dict(jma=9, kma=12, ns=7, seed=21, mean_profile="double-hyperbolic-tangent"),
    "circ_11x10x6": dict(jma=11, kma=10, ns=6, seed=22, mean_profile="circular-hyperbolic-tangent",
                         normal=(1.0, 0.5, -0.25)),
    "ring_12x13x6": dict(jma=12, kma=13, ns=6, seed=23, mean_profile="ring-hyperbolic-tangent", inner_d=0.3),
    # -P profile.dat: read_profile (:487-522) -> adapt1d, no rotation (:1476), clamps (:1344-1350)
    "prof1d_14x16x8": dict(jma=14, kma=16, ns=8, seed=41, normal=(1.0, 0.3, 0.0), profile_text="synthetic"),
    # mid-size: three 256-row SYRK blocks with split K, the split snapshot axis of the
    # spatial-mode pass (ks = 4), DFT/ranking at ns = 520.  Stored reduced (no A_raw / full C).
    "mid_40x40x520": dict(jma=40, kma=40, ns=520, seed=97, reduced=True),
}
MID_STEPS = [0, 1, 255, 256, 518, 519]          # A_raw columns kept for the reduced case
MID_C_ROWS = [0, 1, 255, 256, 257, 300, 511, 512, 519]


def write_synthetic_prf(path, seed=5):
    """A CFD-style .prf plane (CFDCodeIntegration.rst format): 25 x 19 points on a tilted
    rectangle, smooth u, v, w, k, e (k = e = 0 on one edge)."""
    r = np.random.RandomState(seed)
    e1 = np.array([0.2, 0.9, 0.1]); e1 /= np.linalg.norm(e1)
    e2 = np.cross(np.array([0.95, 0.1, 0.3]), e1); e2 /= np.linalg.norm(e2)
    o = np.array([0.3, -0.4, 0.25])
    rows = []
    for a in np.linspace(0.0, 1.2, 25):
        for b in np.linspace(0.0, 0.9, 19):
            x = o + a * e1 + b * e2
            u = 1.0 + 0.2 * np.sin(3 * a) * np.cos(2 * b)
            v, w = 0.05 * a, -0.03 * b
            k = 0.0 if b == 0.0 else 0.01 * (1 + 0.5 * a * b) * (1 + 0.01 * r.rand())
            e = 0.0 if b == 0.0 else 0.05 * (1 + a)
            rows.append((x[0], x[1], x[2], u, v, w, k, e))
    with open(path, "w") as f:
        f.write("# synthetic inlet # name of the profile\n# turbulence model, k-e\n")
        f.write("type, xyz # type of profile (rad or xyz)\n")
        f.write("data,x,y,z,u,v,w,k,e\n")
        for row in rows:
            f.write(",".join("%0.12f" % v for v in row) + "\n")


def unit_read_prf(ref):
    """read_prf on the synthetic plane: plain, bulk-velocity rescaled, mass-flow rescaled."""
    out = {}
    tmp = tempfile.mkdtemp(prefix="pods_prf_")
    try:
        path = os.path.join(tmp, "inlet.prf")
        write_synthetic_prf(path)
        with open(path) as f:
            out["prf_text"] = np.array(f.read())
        for tag, (mdot, den, bulk) in {"plain": (0.0, 0.0, 1.0), "bulk": (0.0, 0.0, 2.5),
                                       "mdot": (0.7, 1.2, 1.0)}.items():
            _stdout = sys.stdout
            sys.stdout = io.StringIO()
            try:
                res = ref["read_prf"](path, 0.1, mdot, den, bulk, False, False)
            finally:
                sys.stdout = _stdout
            for name, v in zip(("U", "V", "W", "uu", "vv", "ww", "uv", "uw", "vw"), res[:9]):
                out["%s_%s" % (tag, name)] = np.asarray(v)
            out[tag + "_scalars"] = np.array([float(x) for x in res[9:]])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def prf_case(ref, ns=6, seed=31):
    """End-to-end main() on the read_prf path: profile from the file, adapt2prf, no rotation."""
    u = unit_read_prf(ref)
    prf = {k: u["plain_" + k] for k in ("U", "V", "W", "uu", "vv", "ww", "uv", "uw", "vw")}
    lnx, kma, jma = u["plain_scalars"][:3]
    kw = dict(jma=int(jma), kma=int(kma), ns=ns, seed=seed, prf=prf, ln_prf=float(lnx))
    res = run_reference_pipeline(ref, **kw)
    res.update({"cfg_jma": np.array(int(jma)), "cfg_kma": np.array(int(kma)), "cfg_ns": np.array(ns),
                "cfg_seed": np.array(seed), "cfg_ln_prf": np.array(float(lnx))})
    res.update({"prf_" + k: v for k, v in prf.items()})
    return res


def unit_adapt2d(ref):
    """adapt2d on raw random fields for each 2-D profile, odd/even/non-square grids."""
    rs = np.random.RandomState(77)
    out = {}
    for tag, (prof, J, K, inner) in {
            "dtanh": ("double-hyperbolic-tangent", 17, 14, 0.5),
            "circ": ("circular-hyperbolic-tangent", 15, 16, 0.5),
            "circ_odd": ("circular-hyperbolic-tangent", 13, 13, 0.5),
            "ring": ("ring-hyperbolic-tangent", 16, 15, 0.5),
            "ring_thin": ("ring-hyperbolic-tangent", 14, 18, 0.8)}.items():
        U, uu, vv, ww, uw = ref["build_profile"](prof, "top-hat", 1.3, 0.05, K)
        uw = 0.3 * np.sqrt(uu * ww) * np.sin(np.linspace(0.0, 3.0, K))      # exercise R20 != 0
        y = [rs.uniform(-2.0, 2.0, (J, K)) for _ in range(3)]
        out[tag + "_in"] = np.stack(y)
        out[tag + "_prof"] = np.stack([U, uu, vv, ww, uw])
        out[tag + "_cfg"] = np.array([J, K, inner])
        out[tag + "_name"] = np.array(prof)
        ref["adapt2d"](y[0], y[1], y[2], U, uu, vv, ww, uw, J, K, prof, inner)
        out[tag + "_out"] = np.stack(y)
    return out


def synthetic_profile_text(npts=15):
    """A 1-D channel profile file for read_profile (digitalfilters.py:487-522): columns
    y U uu vv ww uv over the lower half channel y in [0, 1] (mirrored by the reader).  The
    wall-normal stresses are steep at the wall so the spline overshoots below zero and
    main()'s clamps (:1344-1350) are exercised."""
    y = np.linspace(0.0, 1.0, npts)
    U = np.tanh(6.0 * y) * (1.0 + 0.1 * y)
    uu = 4e-3 * np.exp(-4.0 * y) * np.tanh(30.0 * y) ** 2
    vv = 1e-3 * (1.0 - np.exp(-8.0 * y)) * (1.2 - y)
    ww = 2e-3 * np.tanh(12.0 * y) * (1.1 - 0.5 * y)
    uv = -1.5e-3 * np.tanh(9.0 * y) * (1.0 - y)
    lines = ["# y U uu vv ww uv"]
    for r in zip(y, U, uu, vv, ww, uv):
        lines.append(" ".join("%.10e" % v for v in r))
    return "\n".join(lines) + "\n"


def unit_read_profile(ref):
    """read_profile (digitalfilters.py:487-522) on the synthetic file at a few kma."""
    out = {"text": np.array(synthetic_profile_text())}
    d = tempfile.mkdtemp(prefix="pods_profile_")
    try:
        path = os.path.join(d, "profile.dat")
        with open(path, "w") as f:
            f.write(str(out["text"]))
        for kma in (17, 32, 64):
            with contextlib.redirect_stdout(io.StringIO()):
                res = ref["read_profile"](path, kma)
            out["k%d" % kma] = np.stack(res)
    finally:
        shutil.rmtree(d)
    return out


def unit_save_plane(ref):
    """save_plane (PODFS.py:854-887), the verbose per-step snapshot .prf: file name from
    i_d.time ('%.5E'), header with the plane normal and rhs, rows '%0.12f'."""
    rs = np.random.RandomState(17)
    out = {}
    cases = [((1.0, 0.0, 0.0), (0.0, 0.0, 0.0), 0.0), ((1.0, 0.0, 0.0), (0.5, 0.0, 0.0), 0.0731),
             ((0.6, -0.48, 0.64), (0.25, -1.5, 2.0), 12.5)]
    for c, (n, t_o, tm) in enumerate(cases):
        npt = 7 + 3 * c
        pts = rs.standard_normal((npt, 3)).astype(np.float32).astype(np.float64)
        u = rs.standard_normal(3 * npt) * 10.0 ** rs.randint(-3, 2, 3 * npt)
        i_d = Obj()
        i_d.grid_points = pts
        i_d.n = [np.float64(v) for v in n]
        i_d.t_o = [float(v) for v in t_o]
        i_d.time = tm
        d = tempfile.mkdtemp(prefix="pods_plane_")
        cwd = os.getcwd()
        try:
            os.chdir(d)
            os.makedirs("PODFS")
            ref["save_plane"](u, i_d)
            names = os.listdir("PODFS")
            assert len(names) == 1
            out["plane%d_name" % c] = np.array(names[0])
            out["plane%d_text" % c] = np.array(open(os.path.join("PODFS", names[0])).read())
        finally:
            os.chdir(cwd)
            shutil.rmtree(d)
        out["plane%d_points" % c] = pts
        out["plane%d_u" % c] = u
        out["plane%d_n" % c] = np.array(n)
        out["plane%d_t_o" % c] = np.array(t_o)
        out["plane%d_time" % c] = np.array(tm)
    return out


def unit_verbose(ref):
    """The verbose outputs: fct_welch on temporal-mode-like signals for
    each window and odd/even block sizes, and write_temporal_modes' text for a small T."""
    import contextlib
    rs = np.random.RandomState(91)
    out = {}
    cases = [(64, 16, 1, 100.0), (64, 16, 2, 100.0), (64, 16, 3, 100.0), (101, 15, 2, 37.5),
             (50, 50, 3, 2.0), (33, 8, 1, 10.0)]
    with open(os.devnull, "w") as dn, contextlib.redirect_stdout(dn), warnings.catch_warnings():
        warnings.simplefilter("ignore")                 # complex -> float64 in Sxxsum[:] = ...
        for c, (n, N, iw, fs) in enumerate(cases):
            x = rs.standard_normal(n) * np.sin(np.linspace(0.0, 7.0, n))
            f, Sxx, M = ref["fct_welch"](x, fs, N, iw)
            out["welch%d_cfg" % c] = np.array([n, N, iw, fs])
            out["welch%d_x" % c] = x
            out["welch%d_f" % c] = f
            out["welch%d_Sxx" % c] = Sxx
            out["welch%d_M" % c] = np.array(M)
        T = rs.standard_normal((9, 4)) * np.array([3.0, 1.0, 1e-3, 1e5])
        tmp = tempfile.mkdtemp()
        try:
            ref["write_temporal_modes"](3, 9, 0.0731, T, tmp + "/")
            names = sorted(os.listdir(tmp))
            out["tmodes_T"] = T
            out["tmodes_names"] = np.array(names)
            out["tmodes_text"] = np.array([open(os.path.join(tmp, n)).read() for n in names])
        finally:
            shutil.rmtree(tmp)
    return out


def main():
    only = set(sys.argv[1:])
    ref = load_reference()
    if only:
        if "unit_read_profile" in only:
            np.savez_compressed(os.path.join(HERE, "unit_read_profile.npz"), **unit_read_profile(ref))
        if "unit_save_plane" in only:
            np.savez_compressed(os.path.join(HERE, "unit_save_plane.npz"), **unit_save_plane(ref))
        if "unit_verbose" in only:
            np.savez_compressed(os.path.join(HERE, "unit_verbose.npz"), **unit_verbose(ref))
        if "unit_adapt2d" in only:
            np.savez_compressed(os.path.join(HERE, "unit_adapt2d.npz"), **unit_adapt2d(ref))
        if "unit_read_prf" in only:
            np.savez_compressed(os.path.join(HERE, "unit_read_prf.npz"), **unit_read_prf(ref))
        if "readprf_case" in only:
            np.savez_compressed(os.path.join(HERE, "readprf_case.npz"), **prf_case(ref))
        for name, kw in CASES.items():
            if name in only:
                _write_case(ref, name, kw)
        return
    # unit fixtures for the filter on a raw random block (anisotropic taps) -----------------------
    rs = np.random.RandomState(2024)
    x = rs.uniform(-np.sqrt(3), np.sqrt(3), (2*9+1, 2*6+7, 2*4+5))
    y = np.zeros((7, 5))
    ref["filter3DSciPy1D"](x, y, None, 7, 5, 4.5, 3.0, 2.0, 9, 6, 4)
    taps = [ref["calccoeff"](np.zeros(2*n+1), n, l) for n, l in ((9, 4.5), (6, 3.0), (4, 2.0), (12, 6.0))]
    np.savez_compressed(os.path.join(HERE, "unit_filter.npz"), x=x, y=y, taps_9=taps[0],
                        taps_6=taps[1], taps_4=taps[2], taps_12=taps[3])
    # rotation matrices for a few normals
    normals = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0], [-1, 0, 0], [0.3, -0.5, 0.8]], float)
    Rs = []
    for n in normals:
        n = n / np.linalg.norm(n)
        Rs.append(ref["prof_rotation_matrix"](n[0], n[1], n[2]))
    np.savez_compressed(os.path.join(HERE, "unit_rotation.npz"), normals=normals, R=np.array(Rs))
    np.savez_compressed(os.path.join(HERE, "unit_adapt2d.npz"), **unit_adapt2d(ref))
    np.savez_compressed(os.path.join(HERE, "unit_read_prf.npz"), **unit_read_prf(ref))
    np.savez_compressed(os.path.join(HERE, "readprf_case.npz"), **prf_case(ref))
    np.savez_compressed(os.path.join(HERE, "unit_verbose.npz"), **unit_verbose(ref))
    np.savez_compressed(os.path.join(HERE, "unit_read_profile.npz"), **unit_read_profile(ref))
    np.savez_compressed(os.path.join(HERE, "unit_save_plane.npz"), **unit_save_plane(ref))
    for name, kw in CASES.items():
        _write_case(ref, name, kw)


def _write_case(ref, name, kw):
    kw = dict(kw)
    reduced = kw.pop("reduced", False)
    if kw.get("prf") == "synthetic":
        kw["prf"] = synthetic_prf(kw["jma"], kw["kma"], kw["seed"])
        extra = {"prf_" + k: v for k, v in kw["prf"].items()}
    else:
        extra = {}
    if kw.get("profile_text") == "synthetic":
        kw["profile_text"] = synthetic_profile_text()
    res = run_reference_pipeline(ref, **kw)
    if reduced:  # keep the fixture small: sampled columns/rows plus checksums
        A, C = res.pop("A_raw"), res.pop("C")
        res.pop("filtered_first_steps")
        res["A_steps"] = np.array(MID_STEPS)
        res["A_cols"] = A[:, MID_STEPS].T.copy()
        res["C_rows_idx"] = np.array(MID_C_ROWS)
        res["C_rows"] = C[MID_C_ROWS].copy()
        res["C_diag"] = np.diag(C).copy()
        res["C_max"] = np.array(np.max(np.abs(C)))
        res["C_colsum"] = C.sum(axis=0)
    meta = {k: np.array(v) for k, v in kw.items() if k != "prf"}
    res.update({"cfg_" + k: v for k, v in meta.items()})
    res.update(extra)
    path = os.path.join(HERE, "%s.npz" % name)
    np.savez_compressed(path, **res)
    print("wrote", path, "nm=%d valid=%d" % (res["nm"], res["num_valid_modes"]))


if __name__ == "__main__":
    main()

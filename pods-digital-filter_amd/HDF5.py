"""HDF5.py -- PODFS/PODFS.hdf5 writer, kept as the reference's HDF5.py:11-64.

Layout (CFDCodeIntegration.rst:59-74):
  main              attrs N_POD (int), period (f64)
  main/N_FC         int32 (nm,)
  main/FC           f64 (3*sum N_FC,)  = FC(sum N_FC, 3) flattened in F order
  main/mean         f64 (6P,)          = mean(P, 6) in F order; attrs Np, Nvar, Vars, SF
  main/modes/mode_%04d  same layout and attrs as mean

Python 3 port of the same h5py calls (np.string_ -> np.bytes_, removed in numpy 2).
This interpreter may not have h5py (the build image does not); then the identical h5py
program runs in a Python that does (PODS_H5PY_PYTHON, or /opt/conda/bin/python3*),
fed per dataset through .npy files it memory-maps.  Without any h5py the call raises.
"""
import glob
import os
import subprocess
import sys
import tempfile

import numpy as np

_WRITER = r'''
import os
import sys
import numpy as np
import h5py


def write(f, arrays, nm, period, num_points):
    # HDF5.py:13-62, one dataset at a time (the modes are read one by one)
    main = f.create_group("main")
    main.attrs["N_POD"] = int(nm)
    main.attrs["period"] = float(period)
    N_FC = main.create_dataset("N_FC", (int(nm),), dtype="i")
    N_FC[:] = arrays("N_FC")
    n_fc = arrays("N_FC")
    n = int(np.sum(n_fc))
    FC = main.create_dataset("FC", (n * 3,), dtype=np.float64)
    FC[:] = arrays("FC").reshape(n * 3, order="F")
    P = int(num_points)

    def put(grp, name, a):
        data = grp.create_dataset(name, (P * 6,), dtype=np.float64)
        data[:] = np.asarray(a).reshape(P * 6, order="F")
        data.attrs["Np"] = P
        data.attrs["Nvar"] = 6
        data.attrs["Vars"] = np.bytes_("x,y,z,u,v,w,dummy")
        data.attrs["SF"] = [1., 1., 1., 1., 1., 1.]
    put(main, "mean", arrays("mean"))
    modes = main.create_group("modes")
    for i in range(int(nm)):
        put(modes, "mode_" + "%4.4i" % (i + 1), arrays("mode", i))


if __name__ == "__main__":
    src, dst = sys.argv[1], sys.argv[2]
    meta = np.load(os.path.join(src, "meta.npy"))
    lazy = os.path.exists(os.path.join(src, "spatial.npy"))
    if lazy:  # modes assembled one at a time from the grid points and the spatial modes
        points = np.load(os.path.join(src, "points.npy"), mmap_mode="r")
        spatial = np.load(os.path.join(src, "spatial.npy"), mmap_mode="r")

    def arrays(name, i=None):
        if name == "mode" and lazy:
            P = points.shape[0]
            m = np.empty((P, 6), dtype=np.float64)
            m[:, 0:3] = points
            m[:, 3:] = np.asarray(spatial[:, i]).reshape((P, 3), order="F")
            return m
        fn = name + ("_%04d" % i if i is not None else "") + ".npy"
        return np.load(os.path.join(src, fn), mmap_mode="r")
    with h5py.File(dst, "w") as f:
        write(f, arrays, meta[0], meta[1], meta[2])
'''


def _h5py_python():
    env = os.environ.get("PODS_H5PY_PYTHON")
    cands = ([env] if env else []) + sorted(glob.glob("/opt/conda/bin/python3*")) + ["python3"]
    for exe in cands:
        if not exe or not os.path.exists(exe) and os.sep in exe:
            continue
        try:
            r = subprocess.run([exe, "-c", "import h5py"], capture_output=True, timeout=60)
        except Exception:
            continue
        if r.returncode == 0:
            return exe
    return None


def write_HDF5(i_d, filename="PODFS/PODFS.hdf5"):
    """HDF5.py:11-64.  With h5py in this interpreter the datasets are written directly, one
    after the other; otherwise each array goes to its own .npy file and a Python with h5py
    memory-maps them and writes dataset by dataset.  The modes stream through one at a time:
    i_d.modes (PODFS.ModeStack) builds mode i from the grid points and the spatial modes on
    demand, and the writer does the same from points.npy + spatial.npy, so neither side holds
    the (nm, P, 6) array (1 GB at config 5: 20 modes of 6 x 1 M doubles)."""
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    nm, P = int(i_d.nm), int(i_d.num_points)
    modes = i_d.modes  # indexed one mode at a time: a PODFS.ModeStack is never materialised whole
    try:
        import h5py
    except ImportError:
        h5py = None
    if h5py is not None:
        ns_ = {}
        exec(compile(_WRITER, "<HDF5 writer>", "exec"), ns_)
        src = dict(N_FC=np.asarray(i_d.N_FC), FC=np.asarray(i_d.FC, dtype=np.float64),
                   mean=np.asarray(i_d.mean, dtype=np.float64))
        with h5py.File(filename, "w") as f:
            ns_["write"](f, lambda name, i=None: np.asarray(modes[i], dtype=np.float64) if name == "mode" else src[name],
                         nm, i_d.period, P)
        return filename
    exe = _h5py_python()
    if exe is None:
        raise ImportError("HDF5 output needs h5py (none in this interpreter and no "
                          "PODS_H5PY_PYTHON / conda python with h5py found)")
    with tempfile.TemporaryDirectory() as tmp:
        np.save(os.path.join(tmp, "meta.npy"), np.array([nm, float(i_d.period), P], dtype=np.float64))
        np.save(os.path.join(tmp, "N_FC.npy"), np.asarray(i_d.N_FC))
        np.save(os.path.join(tmp, "FC.npy"), np.asarray(i_d.FC, dtype=np.float64))
        np.save(os.path.join(tmp, "mean.npy"), np.asarray(i_d.mean, dtype=np.float64))
        if hasattr(modes, "spatial") and hasattr(modes, "points") and not getattr(modes.spatial, "streamed", False):
            # the writer assembles each mode from these two (no (nm, P, 6) copy on either side)
            np.save(os.path.join(tmp, "points.npy"), modes.points)
            np.save(os.path.join(tmp, "spatial.npy"), np.asarray(modes.spatial, dtype=np.float64))
        else:
            # one mode at a time (a multi-rank run's modes arrive per mode: digitalfilters.SlabColumns)
            for i in range(nm):
                np.save(os.path.join(tmp, "mode_%04d.npy" % i), np.asarray(modes[i], dtype=np.float64))
        script = os.path.join(tmp, "writer.py")
        with open(script, "w") as f:
            f.write(_WRITER)
        r = subprocess.run([exe, script, tmp, filename], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("HDF5 writer failed: " + r.stderr[-2000:])
    return filename

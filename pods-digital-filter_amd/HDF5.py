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
fed through a temporary .npz.  Without any h5py the call raises.
"""
import glob
import os
import subprocess
import sys
import tempfile

import numpy as np

_WRITER = r'''
import sys
import numpy as np
import h5py
d = np.load(sys.argv[1])
f = h5py.File(sys.argv[2], "w")
main = f.create_group("main")
main.attrs["N_POD"] = int(d["nm"])
main.attrs["period"] = float(d["period"])
N_FC = main.create_dataset("N_FC", (int(d["nm"]),), dtype="i")
N_FC[:] = d["N_FC"]
n = int(np.sum(d["N_FC"]))
FC = main.create_dataset("FC", (n * 3,), dtype=np.float64)
FC[:] = d["FC"].reshape(n * 3, order="F")
P = int(d["num_points"])
data = main.create_dataset("mean", (P * 6,), dtype=np.float64)
data[:] = d["mean"].reshape(P * 6, order="F")
data.attrs["Np"] = P
data.attrs["Nvar"] = 6
data.attrs["Vars"] = np.bytes_("x,y,z,u,v,w,dummy")
data.attrs["SF"] = [1., 1., 1., 1., 1., 1.]
modes = main.create_group("modes")
for i in range(int(d["nm"])):
    counter = "%4.4i" % (i + 1)
    data = modes.create_dataset("mode_" + counter, (P * 6,), dtype=np.float64)
    data[:] = d["modes"][i, :, :].reshape(P * 6, order="F")
    data.attrs["Np"] = P
    data.attrs["Nvar"] = 6
    data.attrs["Vars"] = np.bytes_("x,y,z,u,v,w,dummy")
    data.attrs["SF"] = [1., 1., 1., 1., 1., 1.]
f.close()
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
    payload = dict(nm=np.array(i_d.nm), period=np.array(i_d.period), N_FC=np.asarray(i_d.N_FC),
                   FC=np.asarray(i_d.FC, dtype=np.float64), num_points=np.array(i_d.num_points),
                   mean=np.asarray(i_d.mean, dtype=np.float64), modes=np.asarray(i_d.modes, dtype=np.float64))
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    try:
        import h5py  # noqa: F401
        have = True
    except ImportError:
        have = False
    with tempfile.TemporaryDirectory() as tmp:
        npz = os.path.join(tmp, "podfs_payload.npz")
        np.savez(npz, **payload)
        if have:
            exe = sys.executable
        else:
            exe = _h5py_python()
            if exe is None:
                raise ImportError("HDF5 output needs h5py (none in this interpreter and no "
                                  "PODS_H5PY_PYTHON / conda python with h5py found)")
        r = subprocess.run([exe, "-c", _WRITER, npz, filename], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("HDF5 writer failed: " + r.stderr[-2000:])
    return filename

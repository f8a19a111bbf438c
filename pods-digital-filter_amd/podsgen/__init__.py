"""podsgen -- MI355X-native engine of the digital-filter + PODFS hot path.

Layers:
  _lib.py    ctypes binding of libpodsgen.so (include/podsgen.h)
  host.py    per-run host setup (taps, profiles, Lund factors, rotation, slabs)
  engine.py  device-resident pipeline: generation -> mean -> correlation (+ RCCL
             all-reduce) -> eigensolve -> temporal/spatial modes -> Fourier coefficients
The reference-facing modules (digitalfilters.py, PODFS.py, HDF5.py) sit one level up.
"""
from ._lib import load, check, DFParams  # noqa: F401
from .host import DFSetup, row_slab, time_axis, num_valid_modes, rank_and_count  # noqa: F401
from .engine import (Context, Generator, DeviceSnapshots, PODResult, FourierResult,  # noqa: F401
                     StageTimer, load_snapshots, run_pod, run_fourier, host_rank_and_count, pipeline)

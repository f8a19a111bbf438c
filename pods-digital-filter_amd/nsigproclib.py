"""nsigproclib.py -- the signal helpers of nsigproclib_no_mpi.py the PODFS path uses.

  str(val)          "%0.12f" formatter of every .prf value     nsigproclib_no_mpi.py:880-882
  fct_welch(...)    Welch PSD of a temporal mode (verbose)     nsigproclib_no_mpi.py:10-68

The MPI helpers of the reference file are dead code there (mpi4py is never imported)
and are not carried over; multi-GPU runs use torch.distributed (RCCL) instead.
"""
import builtins

import numpy as np


def str(val):  # noqa: A001 -- the reference's name, shadowing builtins.str on purpose
    return "%0.12f" % val


def fct_welch(x, fs, N, iwindow):
    """Welch PSD with 50 % overlap, returned fftshift-ed (rectangular/Hanning/Blackman)."""
    x = np.asarray(x)
    if N > x.size:
        raise ValueError("Block size N should not be larger than the signal size.")
    if iwindow == 1:
        w = np.ones(N, dtype=np.float64)
    elif iwindow == 2:
        w = np.hanning(N)
    elif iwindow == 3:
        w = np.blackman(N)
    else:
        raise ValueError("iwindow must be 1, 2 or 3")
    Cw = N / np.sum(w ** 2)
    noverlap = int(np.floor(N / 2))
    M = 1
    n_end_block = N
    while True:
        n_end_block = n_end_block + noverlap
        if n_end_block <= x.size:
            M += 1
        else:
            break
    f = np.linspace(-N // 2, N // 2 - 1, N) / N * fs   # Py2 int division: -N/2 == (-N)//2
    Sxx = np.zeros(N, dtype=np.complex64)
    Sxxsum = np.zeros(N, dtype=np.float64)
    for j in range(1, M + 1):
        Sxx[:] = np.fft.fft(x[(j - 1) * noverlap:(j - 1) * noverlap + N] * w)
        Sxx[:] = np.fft.fftshift(Sxx)
        Sxxsum[:] = Sxxsum + (Cw / N / fs * Sxx * np.conj(Sxx)).real
    Sxx[:] = Sxxsum / M
    return f, Sxx, M


__all__ = ["str", "fct_welch", "builtins"]

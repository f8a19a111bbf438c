"""Host cost of the Rayleigh-Ritz round trip pieces: a 2 x 64 x 64 device -> host copy and a
64 x 64 symmetric eigensolve by several host routes (threads matter for so small a problem).

usage: python tools/host_eigh_probe.py
"""
import time

import numpy as np
import torch


def t_us(f, n=200):
    f()
    t = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t) / n * 1e6


def main():
    rng = np.random.default_rng(0)
    A = rng.standard_normal((64, 64))
    A = A + A.T
    out = {}
    out["np.linalg.eigh"] = t_us(lambda: np.linalg.eigh(A))
    try:
        from threadpoolctl import threadpool_limits
        with threadpool_limits(1):
            out["np.linalg.eigh (1 thread)"] = t_us(lambda: np.linalg.eigh(A))
        out["np.linalg.eigh (limits per call)"] = t_us(lambda: (threadpool_limits(1).__enter__(), np.linalg.eigh(A)))
    except Exception as e:  # pragma: no cover
        out["threadpoolctl"] = str(e)
    import scipy.linalg as sl
    from scipy.linalg import lapack
    out["scipy dsyevd"] = t_us(lambda: lapack.dsyevd(A))
    out["scipy dsyev"] = t_us(lambda: lapack.dsyev(A))
    At = torch.from_numpy(A)
    out["torch cpu eigh"] = t_us(lambda: torch.linalg.eigh(At))
    if torch.cuda.is_available():
        D = torch.randn(2, 64, 64, dtype=torch.float64, device="cuda")
        out["device->host 2x64x64 (.cpu())"] = t_us(lambda: D.cpu())
        pin = torch.empty((2, 64, 64), dtype=torch.float64).pin_memory()
        def cp():
            pin.copy_(D, non_blocking=True)
            torch.cuda.current_stream().synchronize()
        out["device->pinned + sync"] = t_us(cp)
        V = torch.empty((64, 64), dtype=torch.float64, device="cuda")
        Vh = np.ascontiguousarray(A)
        out["host->device 64x64"] = t_us(lambda: V.copy_(torch.from_numpy(Vh)))
    for k, v in out.items():
        print("%-36s %s" % (k, ("%.1f us" % v) if isinstance(v, float) else v))


if __name__ == "__main__":
    main()

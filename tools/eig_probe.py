"""GPU probe of pods_syev / pods_sytrd against torch.linalg.eigh (rocSOLVER) on POD-like
correlation matrices C = B^T B / m with a decaying spectrum.

usage: python tools/eig_probe.py [n ...]        (prints one line per size, then timings)
"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))

from podsgen import _lib  # noqa: E402
from podsgen._lib import check, ptr  # noqa: E402
from podsgen.engine import Context  # noqa: E402


def corr_like(n, seed=0, dev="cuda"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    m = max(n + n // 2, 8)
    B = torch.randn(m, n, generator=g, dtype=torch.float64)
    # temporal correlation: smooth the columns so the spectrum decays like a POD's
    k = torch.exp(-0.5 * (torch.arange(-12, 13, dtype=torch.float64) / 4.0) ** 2)
    Bs = torch.nn.functional.conv1d(B.unsqueeze(1), k.view(1, 1, -1), padding=12).squeeze(1)
    Bs = Bs + 0.05 * B
    Bd = Bs.to(dev)
    C = Bd.T @ Bd / m
    return 0.5 * (C + C.T)


def main(sizes):
    ctx = Context(0)
    lib = ctx.lib
    dev = torch.device("cuda", 0)
    nvec = 20
    for n in sizes:
        C = corr_like(n).contiguous()
        lam_ref, V_ref = torch.linalg.eigh(C)
        lam_ref = torch.flip(lam_ref, (0,)).cpu().numpy()
        V_ref = torch.flip(V_ref, (1,)).cpu().numpy()
        d = np.zeros(n)
        e = np.zeros(max(n - 1, 1))
        check(lib.pods_sytrd(ctx.h, ptr(C), n, ptr(d), ptr(e)), "pods_sytrd")
        try:
            from scipy.linalg import eigvalsh_tridiagonal
            lt = np.sort(eigvalsh_tridiagonal(d, e[: n - 1]) if n > 1 else d)[::-1]
            err_t = np.max(np.abs(lt - lam_ref)) / abs(lam_ref[0])
        except Exception as ex:  # pragma: no cover
            err_t = float("nan")
            print("scipy tridiagonal failed:", ex)
        nv = min(nvec, n)
        lam = torch.empty(n, dtype=torch.float64, device=dev)
        Y = torch.empty((n, max(nv, 1)), dtype=torch.float64, device=dev)
        check(lib.pods_syev(ctx.h, ptr(C), n, nv, ptr(lam), ptr(Y)), "pods_syev")
        check(lib.pods_syev_status(ctx.h), "pods_syev_status")
        torch.cuda.synchronize()
        lam_h = lam.cpu().numpy()
        err_l = np.max(np.abs(lam_h - lam_ref)) / abs(lam_ref[0])
        Yh = Y.cpu().numpy()[:, :nv]
        res = np.linalg.norm(C.cpu().numpy() @ Yh - Yh * lam_h[:nv], axis=0) / abs(lam_ref[0])
        orth = np.max(np.abs(Yh.T @ Yh - np.eye(nv)), initial=0.0)
        gl = np.abs(np.diff(lam_ref)) / abs(lam_ref[0])          # gap to the next eigenvalue
        gap = np.minimum(np.r_[gl, np.inf][:nv], np.r_[np.inf, gl][:nv])
        align = np.abs(np.sum(Yh * V_ref[:, :nv], axis=0))
        worst_align = np.max(np.abs(1 - align)[gap > 1e-6], initial=0.0)
        print(f"n={n:5d}  T-eigs err {err_t:.2e}  lam err {err_l:.2e}  resid {res.max():.2e}  "
              f"orth {orth:.2e}  1-|align| (gapped) {worst_align:.2e}", flush=True)

    # timing at the largest size
    n = max(sizes)
    C = corr_like(n).contiguous()
    lam = torch.empty(n, dtype=torch.float64, device=dev)
    Y = torch.empty((n, nvec), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream()
    for it in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        check(lib.pods_syev(ctx.h, ptr(C), n, nvec, ptr(lam), ptr(Y)), "pods_syev")
        e1.record(st)
        torch.cuda.synchronize()
        check(lib.pods_syev_status(ctx.h), "pods_syev_status")
        print(f"pods_syev n={n} nvec={nvec}: {e0.elapsed_time(e1):.2f} ms", flush=True)
    d = np.zeros(n)
    e = np.zeros(n)
    t0 = time.perf_counter()
    check(lib.pods_sytrd(ctx.h, ptr(C), n, ptr(d), ptr(e)), "pods_sytrd")
    print(f"pods_sytrd n={n}: {(time.perf_counter() - t0) * 1e3:.2f} ms (host wall)", flush=True)
    for it in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        torch.linalg.eigh(C)
        e1.record(st)
        torch.cuda.synchronize()
        print(f"torch.linalg.eigh n={n}: {e0.elapsed_time(e1):.2f} ms", flush=True)


if __name__ == "__main__":
    sizes = [int(a) for a in sys.argv[1:]] or [1, 2, 3, 64, 100, 300, 513, 1000, 1500, 2048, 2500, 4096]
    main(sizes)

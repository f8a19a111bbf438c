"""GPU probe: the top-nm eigenpairs of the real C3 correlation matrix by Chebyshev-filtered
subspace iteration (torch fp64 GEMMs), against pods_syev / eigh.  Dumps the C3 spectrum.

usage: python tools/subspace_probe.py [out_dir]
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402


def c3_matrix(J=256, K=256, ns=4096):
    s = podsgen.DFSetup(jma=J, kma=K, ns=ns, seed=12345)
    gen = E.Generator(s, device=0)
    snap = gen.generate()
    lib, ctx = gen.ctx.lib, gen.ctx
    mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
    podsgen.check(lib.pods_mean(ctx.h, E.ptr(mean), 1), "mean")
    podsgen.check(lib.pods_center(ctx.h), "center")
    C = torch.empty((ns, ns), dtype=torch.float64, device="cuda")
    podsgen.check(lib.pods_corr(ctx.h, E.ptr(C), 1), "corr")
    torch.cuda.synchronize()
    return gen, C


def fourier_basis(n, m, dev):
    t = torch.arange(n, dtype=torch.float64, device=dev)
    cols = [torch.ones(n, dtype=torch.float64, device=dev)]
    f = 1
    while len(cols) < m:
        cols.append(torch.cos(2 * np.pi * f * t / n))
        if len(cols) < m:
            cols.append(torch.sin(2 * np.pi * f * t / n))
        f += 1
    return torch.stack(cols, 1)


def orth(Y):
    # Cholesky QR, twice
    for _ in range(2):
        G = Y.T @ Y
        R = torch.linalg.cholesky(G, upper=True)
        Y = torch.linalg.solve_triangular(R, Y, upper=True, left=False)
    return Y


def chfsi(C, k, m, deg, X0, tol, max_outer=30, lmax=None):
    n = C.shape[0]
    X = orth(X0)
    # Rayleigh-Ritz start
    H = X.T @ (C @ X)
    th, V = torch.linalg.eigh(0.5 * (H + H.T))
    th, V = torch.flip(th, (0,)), torch.flip(V, (1,))
    X = X @ V
    if lmax is None:
        lmax = float(th[0]) * 1.01
    ngemm = 1
    hist = []
    for it in range(max_outer):
        cut = float(th[-1])
        a = 0.0
        e = (cut - a) / 2
        c = (cut + a) / 2
        sigma = e / (lmax - c)
        tau = 2 / sigma
        Xp = X
        Y = (C @ X - c * X) * (sigma / e)
        ngemm += 1
        for _ in range(2, deg + 1):
            sn = 1.0 / (tau - sigma)
            Yn = (C @ Y - c * Y) * (2 * sn / e) - (sigma * sn) * Xp
            ngemm += 1
            Xp, Y, sigma = Y, Yn, sn
        Q = orth(Y)
        CQ = C @ Q
        ngemm += 1
        H = Q.T @ CQ
        th, V = torch.linalg.eigh(0.5 * (H + H.T))
        th, V = torch.flip(th, (0,)), torch.flip(V, (1,))
        X = Q @ V
        R = CQ @ V[:, :k] - X[:, :k] * th[:k]
        res = float(torch.linalg.vector_norm(R, dim=0).max()) / float(th[0])
        hist.append(res)
        if res <= tol:
            return X[:, :k], th[:k], it + 1, ngemm, hist
    return X[:, :k], th[:k], max_outer, ngemm, hist


def main(out):
    os.makedirs(out, exist_ok=True)
    gen, C = c3_matrix()
    n = C.shape[0]
    t = time.time()
    lr, Vr = torch.linalg.eigh(C)
    torch.cuda.synchronize()
    t_eigh = time.time() - t
    lr, Vr = torch.flip(lr, (0,)), torch.flip(Vr, (1,))
    lam = lr.cpu().numpy()
    np.save(os.path.join(out, "c3_spectrum.npy"), lam)
    k = 20
    res = {"eigh_s": t_eigh, "lam_head": lam[:80].tolist(), "lam_tail": lam[-8:].tolist()}
    # GEMM speed
    X = torch.randn(n, 64, dtype=torch.float64, device="cuda")
    for w in (32, 64, 128):
        Xw = torch.randn(n, w, dtype=torch.float64, device="cuda")
        for _ in range(3):
            C @ Xw
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(20):
            C @ Xw
        torch.cuda.synchronize()
        res["gemm_us_w%d" % w] = (time.time() - t) / 20 * 1e6
    from podsgen.subspace import leading_eigenpairs, Subspace
    prod = []
    Vh = Vr[:, :k].cpu().numpy()
    ws = Subspace(gen.ctx, n, 64)
    # raw kernel speed: pods_cheb_step at m = 64
    Y = torch.randn(n, 64, dtype=torch.float64, device="cuda")
    Z = torch.randn(n, 64, dtype=torch.float64, device="cuda")
    O_ = torch.empty_like(Y)
    ws.step(C, Y, Z, 1.0, 0.5, 0.25, O_)
    ref = (C @ Y) + 0.5 * Y + 0.25 * Z
    torch.cuda.synchronize()
    res["cheb_err"] = float((O_ - ref).abs().max() / ref.abs().max())
    t = time.time()
    for _ in range(50):
        ws.step(C, Y, Z, 1.0, 0.5, 0.25, O_)
    torch.cuda.synchronize()
    res["cheb_us"] = (time.time() - t) / 50 * 1e6
    print(json.dumps(dict(cheb_us=res["cheb_us"], cheb_err=res["cheb_err"])), flush=True)
    for deg, ch in ((12, 4), (12, 5), (10, 5), (16, 3), (8, 6), (14, 4)):
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.time()
            th, Xk, info = leading_eigenpairs(gen.ctx, C, k, m=64, degree=deg, chunks=ch, tol=3e-14, ws=ws)
            torch.cuda.synchronize()
            dt = time.time() - t
        Xh = Xk.cpu().numpy()
        err = [float(np.max(np.abs(np.sign(np.dot(Xh[:, j], Vh[:, j])) * Xh[:, j] - Vh[:, j]))) for j in range(k)]
        prod.append(dict(deg=deg, chunks=ch, s=dt, vec_err=max(err),
                         lam_err=float(np.max(np.abs(th - lam[:k])) / lam[0]), **info))
        print(json.dumps(prod[-1]), flush=True)
    res["product"] = prod
    trials = []
    for init in ("fourier", "random"):
        for m, deg in ((64, 12),):
            X0 = fourier_basis(n, m, "cuda") if init == "fourier" else torch.randn(n, m, dtype=torch.float64,
                                                                                    device="cuda")
            torch.cuda.synchronize()
            t = time.time()
            Xk, th, its, ngemm, hist = chfsi(C, k, m, deg, X0, tol=1e-14, max_outer=15)
            torch.cuda.synchronize()
            dt = time.time() - t
            Xh = Xk.cpu().numpy()
            Vh = Vr[:, :k].cpu().numpy()
            err = []
            for j in range(k):
                sg = np.sign(np.dot(Xh[:, j], Vh[:, j]))
                err.append(float(np.max(np.abs(sg * Xh[:, j] - Vh[:, j]))))
            lerr = float(np.max(np.abs(th.cpu().numpy() - lam[:k]))) / lam[0]
            trials.append(dict(init=init, m=m, deg=deg, outer=its, gemms=ngemm, s=dt, vec_err=max(err),
                               lam_err=lerr, hist=hist))
            print(json.dumps(trials[-1]), flush=True)
    res["trials"] = trials
    with open(os.path.join(out, "subspace_probe.json"), "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/subspace")

"""The nm leading eigenpairs of the POD correlation matrix without a full tridiagonalisation.

PODFS.py:1309-1333 consumes only lambda_0..lambda_{nm-1} and the nm leading eigenvectors of C
(the temporal modes); the other eigenvalues reach POD.eigenvalues.dat and the printed valid-mode
count only (:1312-1320, :1339), and are computed apart (pods_eigvals_*).  This module finds the
leading block by Chebyshev-filtered subspace iteration (Zhou & Saad) on C itself.  Every filter
step is one call of pods_cheb_step: out = alpha (C Y) + beta Y + gamma Z on fp64 MFMA (the
three-term recurrence fused into the GEMM's epilogue).  Between filter chunks the block is
re-orthonormalised by Cholesky QR (twice); a Rayleigh-Ritz step, whose m x m eigenproblem is
solved on the host, closes each round and measures the residuals.

    X0   = the m lowest-frequency Fourier vectors, orthonormalised
    round: repeat `chunks` times: Y = T_d((C - c I) / e) X (damps [lo, cut]); X = orth(Y)
           H = X^T C X; H V = V Theta; X = X V;  stop when max_j ||C x_j - theta_j x_j||
           <= tol * theta_0 over the k wanted pairs

At ns = 4096 (BASELINE config 3) the top of the POD spectrum is flat (lambda_19 / lambda_63
= 1.10) and one filter degree gains a factor ~1.85 on mode 19 with a 64-vector block; ~70
degrees take the residual to ~1e-14 lambda_0 (tools/subspace_probe.py, profiles/r3/).
"""
import ctypes

import numpy as np

from ._lib import check

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def fourier_start(n, m, device):
    t = torch.arange(n, dtype=torch.float64, device=device) * (2.0 * np.pi / n)
    cols = [torch.ones(n, dtype=torch.float64, device=device)]
    f = 1
    while len(cols) < m:
        cols.append(torch.cos(f * t))
        if len(cols) < m:
            cols.append(torch.sin(f * t))
        f += 1
    return torch.stack(cols, 1).contiguous()


def cholqr(Y):
    """Cholesky QR, twice (CholQR2): orthonormal columns to working precision."""
    for _ in range(2):
        G = Y.T @ Y
        G = 0.5 * (G + G.T)
        R = torch.linalg.cholesky(G, upper=True)
        Y = torch.linalg.solve_triangular(R, Y, upper=True, left=False)
    return Y.contiguous()


class Subspace:
    """Workspace + kernels of the iteration on one context (three n x m rotating buffers)."""

    def __init__(self, ctx, n, m):
        self.ctx, self.lib = ctx, ctx.lib
        self.n, self.m = n, m
        dev = torch.device("cuda", ctx.device)
        self.buf = [torch.empty((n, m), dtype=torch.float64, device=dev) for _ in range(3)]

    def step(self, C, Y, Z, alpha, beta, gamma, out):
        check(self.lib.pods_cheb_step(self.ctx.h, ctypes.c_void_p(C.data_ptr()), self.n,
                                      ctypes.c_void_p(Y.data_ptr()),
                                      None if Z is None else ctypes.c_void_p(Z.data_ptr()), self.m,
                                      float(alpha), float(beta), float(gamma), ctypes.c_void_p(out.data_ptr())),
              "pods_cheb_step")
        return out

    def product(self, C, X):
        out = self._free(X)
        return self.step(C, X, None, 1.0, 0.0, 0.0, out).clone()

    def _free(self, *used):
        for b in self.buf:
            if all(b.data_ptr() != u.data_ptr() for u in used):
                return b
        raise RuntimeError("no free buffer")

    def filter(self, C, X, degree, lo, cut, top):
        """T_degree((C - c I)/e) X, scaled (Zhou & Saad), damping [lo, cut]."""
        e = 0.5 * (cut - lo)
        c = 0.5 * (cut + lo)
        sigma = e / (top - c)
        tau = 2.0 / sigma
        b0 = self._free(X)
        X0 = b0.copy_(X)
        Y = self.step(C, X0, None, sigma / e, -c * sigma / e, 0.0, self._free(X0))
        Yp = X0
        for _ in range(2, degree + 1):
            sn = 1.0 / (tau - sigma)
            out = self._free(Y, Yp)
            Y, Yp = self.step(C, Y, Yp, 2.0 * sn / e, -c * 2.0 * sn / e, -sigma * sn, out), Y
            sigma = sn
        return Y

    def rayleigh_ritz(self, C, X):
        CX = self.product(C, X)
        H = (X.T @ CX).cpu().numpy()
        th, V = np.linalg.eigh(0.5 * (H + H.T))
        th, V = th[::-1].copy(), np.ascontiguousarray(V[:, ::-1])
        Vd = torch.from_numpy(V).to(X.device)
        return th, (X @ Vd).contiguous(), CX @ Vd


def leading_eigenpairs(ctx, C, k, m=64, degree=12, chunks=4, tol=3e-14, max_rounds=4, ws=None):
    """The k largest eigenpairs of the symmetric positive semi-definite device matrix C.

    Returns (theta (k,) numpy descending, X (n, k) device tensor, orthonormal columns, info)."""
    n = C.shape[0]
    if m % 64 or m > n or k > m:
        raise ValueError("leading_eigenpairs: m must be a multiple of 64 with k <= m <= n")
    ws = ws or Subspace(ctx, n, m)
    X = cholqr(fourier_start(n, m, C.device))
    th, X, CX = ws.rayleigh_ritz(C, X)
    res, gemms, r = np.inf, 1, 0
    for r in range(1, max_rounds + 1):
        cut, top = float(th[-1]), float(th[0])
        lo = -1e-3 * cut              # C is a PSD correlation: nothing meaningful below 0
        for _ in range(chunks):
            X = cholqr(ws.filter(C, X, degree, lo, cut, top))
            gemms += degree
        th, X, CX = ws.rayleigh_ritz(C, X)
        gemms += 1
        R = CX[:, :k] - X[:, :k] * torch.from_numpy(th[:k].copy()).to(C.device)
        res = float(torch.linalg.vector_norm(R, dim=0).max()) / float(th[0])
        if res <= tol:
            break
        chunks = 1                    # top-up rounds
    return th[:k].copy(), X[:, :k].contiguous(), dict(rounds=r, gemms=gemms, residual=res, block=m,
                                                        degree=degree)

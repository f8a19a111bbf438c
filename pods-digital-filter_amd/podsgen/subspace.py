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


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class Subspace:
    """Workspace of the iteration on one context: named n x m blocks (F*: the filter's three
    rotating terms, Q*: Cholesky QR, R*: Rayleigh-Ritz) and the m x m Gram / rotation."""

    def __init__(self, ctx, n, m=64):
        if m != 64:
            raise ValueError("Subspace: m = 64 (pods_cholqr's block)")
        self.ctx, self.lib, self.n, self.m = ctx, ctx.lib, n, m
        dev = torch.device("cuda", ctx.device)
        mk = lambda: torch.empty((n, m), dtype=torch.float64, device=dev)  # noqa: E731
        self.F = [mk(), mk(), mk()]
        self.Q0, self.Q1, self.R0, self.R1, self.R2 = mk(), mk(), mk(), mk(), mk()
        self.G = torch.empty((m, m), dtype=torch.float64, device=dev)
        self.V = torch.empty((m, m), dtype=torch.float64, device=dev)
        self._start = None

    # -- kernels (C-ABI) --------------------------------------------------------------------
    def prepare(self, C):
        """Tiled copy of C for the Chebyshev steps (once per matrix)."""
        check(self.lib.pods_cheb_prepare(self.ctx.h, _p(C), self.n), "pods_cheb_prepare")

    def step(self, C, Y, Z, alpha, beta, gamma, out):
        check(self.lib.pods_cheb_step(self.ctx.h, _p(C), self.n, _p(Y), None if Z is None else _p(Z), self.m,
                                      float(alpha), float(beta), float(gamma), _p(out)), "pods_cheb_step")
        return out

    def cholqr2(self, Y):
        """Orthonormal basis of span(Y) by two Cholesky-QR passes: Y -> Q0 -> Q1."""
        check(self.lib.pods_cholqr(self.ctx.h, _p(Y), self.n, self.m, _p(self.Q0)), "pods_cholqr")
        check(self.lib.pods_cholqr(self.ctx.h, _p(self.Q0), self.n, self.m, _p(self.Q1)), "pods_cholqr")
        return self.Q1

    def start(self):
        """The m lowest-frequency Fourier vectors, orthonormalised (cached per workspace)."""
        if self._start is None:
            X = fourier_start(self.n, self.m, self.G.device)
            self._start = self.cholqr2(X).clone()
        return self._start

    def filter(self, C, X, degree, lo, cut, top):
        """T_degree((C - c I)/e) X, scaled (Zhou & Saad), damping [lo, cut]; X not an F block."""
        e = 0.5 * (cut - lo)
        c = 0.5 * (cut + lo)
        sigma = e / (top - c)
        tau = 2.0 / sigma
        Y = self.step(C, X, None, sigma / e, -c * sigma / e, 0.0, self.F[0])
        Yp = X
        for _ in range(2, degree + 1):
            sn = 1.0 / (tau - sigma)
            out = next(b for b in self.F if b.data_ptr() not in (Y.data_ptr(), Yp.data_ptr()))
            Y, Yp = self.step(C, Y, Yp, 2.0 * sn / e, -c * 2.0 * sn / e, -sigma * sn, out), Y
            sigma = sn
        return Y

    def rayleigh_ritz(self, C, X):
        """Ritz values (host, descending), Ritz vectors R1 and C R1 = R2 of span(X)."""
        CX = self.step(C, X, None, 1.0, 0.0, 0.0, self.R0)
        check(self.lib.pods_gram(self.ctx.h, _p(X), _p(CX), self.n, self.m, _p(self.G)), "pods_gram")
        H = self.G.cpu().numpy()
        th, V = np.linalg.eigh(0.5 * (H + H.T))
        th, V = th[::-1].copy(), np.ascontiguousarray(V[:, ::-1])
        self.V.copy_(torch.from_numpy(V))
        check(self.lib.pods_right_mul(self.ctx.h, _p(X), _p(self.V), self.n, self.m, _p(self.R1)), "pods_right_mul")
        check(self.lib.pods_right_mul(self.ctx.h, _p(CX), _p(self.V), self.n, self.m, _p(self.R2)),
              "pods_right_mul")
        return th, self.R1, self.R2


def leading_eigenpairs(ctx, C, k, m=64, degree=12, chunks=3, warm=8, tol=3e-14, max_rounds=4, ws=None):
    """The k largest eigenpairs of the symmetric positive semi-definite device matrix C.

    A Rayleigh-Ritz step on the Fourier start, one `warm`-degree filter and a second
    Rayleigh-Ritz place the damping interval's upper edge (cut = the smallest Ritz value of
    the block, near lambda_m); then rounds of `chunks` filters of `degree` (CholQR2 between
    them, no host round trip) each closed by a Rayleigh-Ritz step and the residual check.
    Returns (theta (k,) numpy descending, X (n, k) device tensor, orthonormal columns, info)."""
    n = C.shape[0]
    if m != 64 or m > n or k > m:
        raise ValueError("leading_eigenpairs: m = 64 with k <= m <= n")
    ws = ws or Subspace(ctx, n, m)
    ws.prepare(C)
    th, X, CX = ws.rayleigh_ritz(C, ws.start())
    gemms = 1
    if warm:
        cut, top = float(th[-1]), float(th[0])
        X = ws.cholqr2(ws.filter(C, X, warm, -1e-3 * cut, cut, top))
        th, X, CX = ws.rayleigh_ritz(C, X)
        gemms += warm + 1
    res, r, hist = np.inf, 0, []
    for r in range(1, max_rounds + 1):
        cut, top = float(th[-1]), float(th[0])
        lo = -1e-3 * cut              # C is a PSD correlation: nothing meaningful below 0
        for _ in range(chunks):
            X = ws.cholqr2(ws.filter(C, X, degree, lo, cut, top))
            gemms += degree
        th, X, CX = ws.rayleigh_ritz(C, X)
        gemms += 1
        thd = torch.from_numpy(th[:k].copy()).to(C.device)
        res = float(torch.linalg.vector_norm(CX[:, :k] - X[:, :k] * thd, dim=0).max()) / float(th[0])
        hist.append(res)
        if res <= tol:
            break
        chunks = 1                    # top-up rounds
    return th[:k].copy(), X[:, :k].contiguous(), dict(rounds=r, gemms=gemms, residual=res, block=m,
                                                        degree=degree, hist=hist)

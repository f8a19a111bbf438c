"""The nm leading eigenpairs of the POD correlation matrix without a full tridiagonalisation.

PODFS.py:1309-1333 consumes only lambda_0..lambda_{nm-1} and the nm leading eigenvectors of C
(the temporal modes); the other eigenvalues reach POD.eigenvalues.dat and the printed valid-mode
count only (:1312-1320, :1339), and are computed apart (pods_eigvals_*).  This module finds the
leading block by Chebyshev-filtered subspace iteration (Zhou & Saad) on C itself.  Every filter
step is one call of pods_cheb_step: out = alpha (C Y) + beta Y + gamma Z on fp64 MFMA (the
three-term recurrence fused into the GEMM's epilogue).  The block is re-conditioned by one
Cholesky-QR pass between filter chunks and orthonormalised by two before a Rayleigh-Ritz step.

    X0   = cos / sin of the m/2 lowest non-zero frequencies, orthonormalised
    RR   : H = X^T C X, E = C X - X H, F = E^T E (device); eigh(H) = V Theta (host, 64 x 64);
           residual of pair j = sqrt(v_j^T F v_j) / theta_0 (no cancellation: E is the
           residual block itself) -- one host round trip per Rayleigh-Ritz step
    warm : a degree-20 filter on the interval the start's Rayleigh quotients give (no
           eigensolve), then RR (places the damped interval's edge near lambda_{m-5})
    round: d = the filter degree that takes the largest residual of the k wanted pairs to
           tol at the convergence rate per degree (first planned round: 0.8 x the Chebyshev
           rate of theta_{k-1} against the damped interval [lo, theta_{m-1}]; later: the rate
           the previous round achieved), in chunks whose condition growth stays below ~1e6;
           then RR and the residual check
    end  : X V[:, :k]

At ns = 4096 (BASELINE config 3) the top of the POD spectrum is flat (lambda_19 / lambda_63
= 1.10) and one filter degree gains ~0.5 nat on mode 19 with a 64-vector block; ~60 degrees
take the residual to ~1e-14 lambda_0 (tools/topk_probe.py, profiles/r3/).
"""
import ctypes

import numpy as np

from ._lib import check

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def fourier_start(n, m, device):
    """cos / sin of the m/2 lowest non-zero frequencies over the n snapshots.  No constant
    vector: the snapshots are centred (main :1492-1495), so C 1 = 0 and it would only place
    the damped interval's edge at 0."""
    t = torch.arange(n, dtype=torch.float64, device=device) * (2.0 * np.pi / n)
    cols = []
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
    rotating terms, Q*: Cholesky QR, R*: Rayleigh-Ritz) and the m x m Gram matrices."""

    def __init__(self, ctx, n, m=64):
        if m != 64:
            raise ValueError("Subspace: m = 64 (pods_cholqr's block)")
        self.ctx, self.lib, self.n, self.m = ctx, ctx.lib, n, m
        dev = torch.device("cuda", ctx.device)
        mk = lambda: torch.empty((n, m), dtype=torch.float64, device=dev)  # noqa: E731
        self.F = [mk(), mk(), mk()]
        self.Q0, self.Q1, self.R0, self.R1, self.R2 = mk(), mk(), mk(), mk(), mk()
        self.HF = torch.empty((2, m, m), dtype=torch.float64, device=dev)   # H and F of one RR
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

    def cholqr(self, Y, out):
        """One Cholesky-QR pass: out = Y R^{-1}, R^T R = Y^T Y."""
        check(self.lib.pods_cholqr(self.ctx.h, _p(Y), self.n, self.m, _p(out)), "pods_cholqr")
        return out

    def cholqr2(self, Y):
        """Orthonormal basis of span(Y) by two Cholesky-QR passes: Y -> Q0 -> Q1."""
        return self.cholqr(self.cholqr(Y, self.Q0), self.Q1)

    def start(self):
        """The m lowest-frequency Fourier vectors, orthonormalised (a constant basis, cached per
        workspace)."""
        if self._start is None:
            X = fourier_start(self.n, self.m, self.HF.device)
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

    def ritz(self, C, X, k):
        """Rayleigh-Ritz on span(X), X orthonormal and not R0/R1: Ritz values (descending), the
        rotation V (host, m x m) and the residual norms / theta_0 of the k leading pairs."""
        lib, h, n, m = self.lib, self.ctx.h, self.n, self.m
        CX = self.step(C, X, None, 1.0, 0.0, 0.0, self.R0)
        H, F = self.HF[0], self.HF[1]
        check(lib.pods_gram(h, _p(X), _p(CX), n, m, _p(H)), "pods_gram")
        check(lib.pods_ritz_residual(h, _p(X), _p(CX), _p(H), n, m, _p(self.R1)), "pods_ritz_residual")
        check(lib.pods_gram(h, _p(self.R1), _p(self.R1), n, m, _p(F)), "pods_gram")
        HF = self.HF.cpu().numpy()
        Hh, Fh = HF[0], HF[1]
        th, V = np.linalg.eigh(0.5 * (Hh + Hh.T))
        th, V = th[::-1].copy(), np.ascontiguousarray(V[:, ::-1])
        Vk = V[:, :k]
        r2 = np.einsum("ij,ij->j", Vk, (0.5 * (Fh + Fh.T)) @ Vk)
        res = np.sqrt(np.maximum(r2, 0.0)) / th[0]
        return th, V, res

    def quotients(self, C, X):
        """Rayleigh quotients x_j^T C x_j of the columns of an orthonormal X (host, descending):
        the damped interval of the first filter, without an eigensolve."""
        CX = self.step(C, X, None, 1.0, 0.0, 0.0, self.R0)
        H = self.HF[0]
        check(self.lib.pods_gram(self.ctx.h, _p(X), _p(CX), self.n, self.m, _p(H)), "pods_gram")
        return np.sort(torch.diagonal(H).cpu().numpy())[::-1].copy()

    def rotate(self, X, V):
        """X V (device), V a host m x m rotation; the result lives in R2."""
        self.V.copy_(torch.from_numpy(V))
        check(self.lib.pods_right_mul(self.ctx.h, _p(X), _p(self.V), self.n, self.m, _p(self.R2)),
              "pods_right_mul")
        return self.R2


def _chebyshev_rate(x):
    """Growth per degree of T_d at x >= 1 (0 inside the damped interval)."""
    return float(np.arccosh(x)) if x > 1.0 else 0.0


def leading_eigenpairs(ctx, C, k, m=64, tol=3e-14, max_degree=400, warm=20, rate_factor=0.85, margin=1.05,
                      cut_index=None, schedule=None, ws=None):
    """The k largest eigenpairs of the symmetric positive semi-definite device matrix C.

    The first round is a fixed `warm`-degree filter: the Fourier start's Ritz values sit far
    below the spectrum's (theta_59 ~ lambda_263 at C3), so the damped interval they give is too
    short to plan with.

    Returns (theta (k,) numpy descending, X (n, k) device tensor with orthonormal columns,
    info: rounds, gemms, filter degree, final max residual / theta_0, the residual history)."""
    n = C.shape[0]
    if m != 64 or m > n or k > m or k < 1:
        raise ValueError("leading_eigenpairs: m = 64 with 1 <= k <= m <= n")
    ws = ws or Subspace(ctx, n, m)
    ws.prepare(C)
    X = ws.start()
    if warm and schedule is None:
        th = ws.quotients(C, X)             # enough for the warm filter's interval
        worst = np.inf
    else:
        th, V, res = ws.ritz(C, X, k)
        worst = float(res.max())
    gemms, degrees, rounds, rate = 1, 0, 0, None
    hist = [worst]
    cuts = [] if schedule is not None else None
    while worst > tol and degrees < max_degree:
        rounds += 1
        # damped interval [lo, theta_{m-5}]: its edge converges (to ~lambda_{m-4}) within two
        # rounds, where theta_{m-1} is still far below lambda_{m-1} (profiles/r3/topk_*.json)
        top, cut = float(th[0]), float(th[m - 5 if cut_index is None else cut_index])
        lo = -1e-3 * cut                    # C is a PSD correlation: nothing meaningful below 0
        if schedule is not None:            # diagnostics: fixed degrees per round
            if rounds > len(schedule):
                break
            need = schedule[rounds - 1]
        elif rounds == 1 and warm:
            need = warm
        else:
            if rate is None:
                rate = rate_factor * _chebyshev_rate(2.0 * float(th[k - 1]) / cut - 1.0)
            rate = max(rate, 0.05)
            need = int(np.ceil(margin * np.log(worst / tol) / rate))
        need = max(2, min(need, max_degree - degrees))
        # condition growth of the block over one chunk ~ T_d(x_0): keep it below ~2e6
        grow = max(_chebyshev_rate(2.0 * top / cut - 1.0), 1e-3)
        chunk = int(min(20, max(2, np.floor(np.log(2e6) / grow))))
        nchunks = -(-need // chunk)
        per = -(-need // nchunks)
        for _ in range(nchunks):
            X = ws.cholqr(ws.filter(C, X, per, lo, cut, top), ws.Q0)
        X = ws.cholqr(X, ws.Q1)
        degrees += per * nchunks
        gemms += per * nchunks + 1
        th, V, res = ws.ritz(C, X, k)
        new = float(res.max())
        hist.append(new)
        if cuts is not None:
            cuts.append((per * nchunks, cut))
        if rounds > 1 or not warm:          # the warm round's rate says nothing about the next
            rate = np.log(worst / new) / (per * nchunks) if 0.0 < new < worst else 0.5 * rate
        worst = new
    Xk = ws.rotate(X, V)[:, :k].contiguous()
    info = dict(rounds=rounds, gemms=gemms, degrees=degrees, residual=worst, block=m, hist=hist)
    if cuts is not None:
        info["cuts"] = cuts
    return th[:k].copy(), Xk, info

#!/usr/bin/env python3
"""Numpy prototype of the two-stage symmetric eigensolver (index bookkeeping for the HIP
kernels in podsgen_sy2sb.hip): dense -> band (panel QR + two-sided blocked update), band ->
tridiagonal (bulge chasing, one Householder of length <= b per task), eigenvalues of the
tridiagonal, eigenvectors by inverse iteration on the band matrix + back-transformation
with the stage-1 reflectors.  Not product code; `python tools/twostage_proto.py` checks it
against numpy.linalg.eigh.
"""
import numpy as np


def house(x):
    """v (v[0] = 1), tau, beta with (I - tau v v^T) x = beta e1 (dlarfg)."""
    alpha = x[0]
    sigma = float(np.dot(x[1:], x[1:]))
    v = np.zeros_like(x)
    v[0] = 1.0
    if sigma == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.sqrt(alpha * alpha + sigma), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def panel_qr(P):
    """Householder QR of P (m x b) in place: returns V (unit lower), T (b x b upper), R."""
    m, b = P.shape
    P = P.copy()
    V = np.zeros((m, b))
    taus = np.zeros(b)
    for j in range(min(b, m)):
        v, tau, beta = house(P[j:, j])
        V[j:, j] = v
        taus[j] = tau
        if j + 1 < b:
            w = v @ P[j:, j + 1:]
            P[j:, j + 1:] -= tau * np.outer(v, w)
        P[j, j] = beta
        P[j + 1:, j] = 0.0
    # dlarft forward columnwise
    T = np.zeros((b, b))
    G = V.T @ V
    for i in range(b):
        T[i, i] = taus[i]
        if i:
            T[:i, i] = -taus[i] * (T[:i, :i] @ G[:i, i])
    return V, T, np.triu(P[:b, :])


def sy2sb(A, b):
    """Dense symmetric -> band (lower bandwidth b).  Returns the band matrix (dense array)
    and the list of (row offset, V, T) reflector blocks (Q = Q_0 Q_1 ...)."""
    A = A.copy()
    n = A.shape[0]
    blocks = []
    for c0 in range(0, n - b - 1, b):
        r0 = c0 + b
        P = A[r0:, c0:c0 + b]
        V, T, R = panel_qr(P)
        m = n - r0
        A[r0:, c0:c0 + b] = 0.0
        A[r0:r0 + min(b, m), c0:c0 + b] = R[:min(b, m)]
        A[c0:c0 + b, r0:] = A[r0:, c0:c0 + b].T
        A22 = A[r0:, r0:]
        X = A22 @ V @ T
        W = X - 0.5 * V @ (T.T @ (V.T @ X))
        A[r0:, r0:] = A22 - V @ W.T - W @ V.T
        blocks.append((r0, V, T))
    return A, blocks


def sb2st(B, b):
    """Band (lower bandwidth b, dense storage) -> tridiagonal by bulge chasing.  Sweep s
    annihilates column s below the subdiagonal; task (s, k) uses one Householder of
    length <= b on rows R_k = [s+1+k b, s+1+(k+1) b), applied to the blocks
    A[R_k, R_{k-1}] (left), A[R_k, R_k] (both sides), A[R_{k+1}, R_k] (right).
    Returns (d, e, reflectors) with reflectors[(s, k)] = (row0, v, tau)."""
    A = B.copy()
    n = A.shape[0]
    refl = []
    for s in range(n - 2):
        k = 0
        while True:
            r0 = s + 1 + k * b
            if r0 >= n - 1:
                break
            r1 = min(r0 + b, n)
            col = s if k == 0 else s + 1 + (k - 1) * b
            x = A[r0:r1, col].copy()
            if r1 - r0 < 2 or not np.any(x[1:]):
                if k > 0:
                    pass
                # nothing to annihilate; the chase ends when no bulge was created
                if k == 0:
                    break
            v, tau, beta = house(x)
            # left: rows R_k of every column < r0 that touches them (col .. r0-1)
            c_lo = col
            H = np.eye(r1 - r0) - tau * np.outer(v, v)
            A[r0:r1, c_lo:r0] = H @ A[r0:r1, c_lo:r0]
            A[c_lo:r0, r0:r1] = A[r0:r1, c_lo:r0].T
            # both sides on the diagonal block
            A[r0:r1, r0:r1] = H @ A[r0:r1, r0:r1] @ H
            # right: rows below R_k within reach (r1 .. min(r1 + b, n))
            r2 = min(r1 + b, n)
            if r2 > r1:
                A[r1:r2, r0:r1] = A[r1:r2, r0:r1] @ H
                A[r0:r1, r1:r2] = A[r1:r2, r0:r1].T
            refl.append((r0, v, tau))
            if r2 <= r1:
                break
            k += 1
    d = np.diag(A).copy()
    e = np.diag(A, -1).copy()
    return d, e, A, refl


def band_inverse_iteration(B, lam, iters=3, seed=0):
    """Eigenvector of the band matrix B for eigenvalue lam (dense solve stands in for the
    banded LU with partial pivoting)."""
    n = B.shape[0]
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n)
    M = B - lam * np.eye(n)
    for _ in range(iters):
        try:
            x = np.linalg.solve(M, x)
        except np.linalg.LinAlgError:
            x = np.linalg.lstsq(M, x, rcond=None)[0]
        x /= np.linalg.norm(x)
    return x


def apply_q1(blocks, y):
    """Q1 y with Q1 = Q_0 Q_1 ... (apply the last block first)."""
    y = y.copy()
    for r0, V, T in reversed(blocks):
        y[r0:] -= V @ (T @ (V.T @ y[r0:]))
    return y


def main():
    rng = np.random.default_rng(1)
    for n, b in [(64, 8), (97, 16), (256, 16), (200, 32)]:
        X = rng.standard_normal((3 * n, n)) * np.logspace(0, -6, n)[None, :]
        X -= X.mean(axis=1, keepdims=True)
        C = X.T @ X / n
        Bd, blocks = sy2sb(C, b)
        assert np.allclose(np.tril(Bd, -b - 1), 0.0, atol=0)
        lam_ref, Vref = np.linalg.eigh(C)
        lam_b = np.linalg.eigvalsh(Bd)
        d, e, Tm, refl = sb2st(Bd, b)
        lam_t = np.linalg.eigvalsh(np.diag(d) + np.diag(e, 1) + np.diag(e, -1))
        offband = np.max(np.abs(np.tril(Tm, -2)))
        err_b = np.max(np.abs(lam_b - lam_ref)) / lam_ref[-1]
        err_t = np.max(np.abs(lam_t - lam_ref)) / lam_ref[-1]
        # top eigenvectors
        verr = 0.0
        for j in range(1, 6):
            y = band_inverse_iteration(Bd, lam_t[-j])
            x = apply_q1(blocks, y)
            r = Vref[:, -j]
            verr = max(verr, np.max(np.abs(np.sign(x @ r) * x - r)))
        print("n=%d b=%d  band err %.2e  tri err %.2e  offband %.1e  vec err %.2e  tasks %d"
              % (n, b, err_b, err_t, offband, verr, len(refl)))


if __name__ == "__main__":
    main()

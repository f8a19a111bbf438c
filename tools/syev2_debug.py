#!/usr/bin/env python3
"""Stage-by-stage check of pods_syev2 on one POD-like matrix: band eigenvalues (stage 1),
tridiagonal eigenvalues (stage 2), final eigenvalues, against numpy."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pods-digital-filter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402
from test_gpu_eigen import pod_like  # noqa: E402


def dense_from_band(bd, n, LDB):
    A = np.zeros((n, n))
    for c in range(n):
        for d in range(LDB):
            if c + d < n:
                A[c + d, c] = bd[c * LDB + d]
                A[c, c + d] = bd[c * LDB + d]
    return A


def main():
    ctx = E.Context(0)
    for n in [int(x) for x in (sys.argv[1:] or ["34", "100"])]:
        C = pod_like(n, seed=n)
        lam = torch.empty(n, dtype=torch.float64, device="cuda")
        Y = torch.empty((n, 1), dtype=torch.float64, device="cuda")
        podsgen.check(ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, 0, E.ptr(lam), E.ptr(Y)), "syev2")
        podsgen.check(ctx.lib.pods_syev2_status(ctx.h), "status")
        Ch = C.cpu().numpy()
        lr = np.linalg.eigvalsh(Ch)[::-1]
        sc = abs(lr[0])
        LDB = 64
        b0 = np.empty(n * LDB)
        podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, 0, 0, E.ptr(b0), n * LDB), "inspect")
        Aw = np.empty(n * n)
        podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, 0, 3, E.ptr(Aw), n * n), "inspect")
        Aw = Aw.reshape(n, n)
        B0 = dense_from_band(b0, n, LDB)
        lb = np.linalg.eigvalsh(B0)[::-1]
        b1 = np.empty(n * LDB)
        podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, 0, 1, E.ptr(b1), n * LDB), "inspect")
        B1 = dense_from_band(b1, n, LDB)
        de = np.empty(2 * n)
        podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, 0, 2, E.ptr(de), 2 * n), "inspect")
        d, e = de[:n], de[n:2 * n - 1]
        lt = np.linalg.eigvalsh(np.diag(d) + np.diag(e, 1) + np.diag(e, -1))[::-1]
        print("n=%d  band(stage1) err %.2e  tri err %.2e  final err %.2e  offband(stage2) %.2e  "
              "band-nonzero-beyond-32 %.2e  Aw asym %.2e"
              % (n, np.max(np.abs(lb - lr)) / sc, np.max(np.abs(lt - lr)) / sc,
                 np.max(np.abs(lam.cpu().numpy() - lr)) / sc,
                 np.max(np.abs(np.tril(B1, -2))) / sc, np.max(np.abs(b0.reshape(n, LDB)[:, 33:])) / sc,
                 np.max(np.abs(Aw - Aw.T)) / sc))
        # also the stage-1 result through the prototype's sb2st for comparison
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import twostage_proto as TP
        dd, ee, _, _ = TP.sb2st(B0, 32)
        lp = np.linalg.eigvalsh(np.diag(dd) + np.diag(ee, 1) + np.diag(ee, -1))[::-1]
        print("      proto sb2st on the GPU band: err %.2e" % (np.max(np.abs(lp - lr)) / sc))


def vectors(n, nvec=20):
    """PODS_SY2SB_NOBT=1: the inverse-iteration vectors of the band matrix against eigh(B0)."""
    ctx = E.Context(0)
    C = pod_like(n, seed=n)
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    Y = torch.empty((n, nvec), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, nvec, E.ptr(lam), E.ptr(Y)), "syev2")
    b0 = np.empty(n * 64)
    podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, nvec, 0, E.ptr(b0), n * 64), "inspect")
    B0 = dense_from_band(b0, n, 64)
    lr, Vr = np.linalg.eigh(B0)
    lr, Vr = lr[::-1], Vr[:, ::-1]
    Yh = Y.cpu().numpy()
    lg = lam.cpu().numpy()
    res = np.linalg.norm(B0 @ Yh - Yh * lg[:nvec], axis=0) / abs(lr[0])
    gaps = np.abs(np.diff(lr[:nvec + 1])) / abs(lr[0])
    print("n=%d band-vector residuals" % n, np.array2string(res, precision=1))
    print("   rel gaps", np.array2string(gaps, precision=1))
    print("   |y_k . v_k|", np.array2string(np.abs(np.sum(Yh * Vr[:, :nvec], axis=0)), precision=3))


if os.environ.get("PODS_SY2SB_NOBT"):
    for n_ in [int(x) for x in sys.argv[1:]]:
        vectors(n_)
    sys.exit(0)


if __name__ == "__main__":
    main()

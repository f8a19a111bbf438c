#!/usr/bin/env python3
"""One stage-1 panel of pods_syev2 (PODS_SY2SB_PANELS=1) against numpy: V, tau, T, Y = A22 V,
X = Y T, W, and the updated trailing matrix."""
import os
import sys

import numpy as np

os.environ["PODS_SY2SB_PANELS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pods-digital-filter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402
from test_gpu_eigen import pod_like  # noqa: E402
import twostage_proto as TP  # noqa: E402


def get(ctx, n, what, count):
    out = np.empty(count)
    podsgen.check(ctx.lib.pods_syev2_inspect(ctx.h, n, 0, what, E.ptr(out), count), "inspect")
    return out


def main():
    ctx = E.Context(0)
    B = 32
    for n in [int(x) for x in (sys.argv[1:] or ["34", "100"])]:
        C = pod_like(n, seed=n)
        lam = torch.empty(n, dtype=torch.float64, device="cuda")
        Y = torch.empty((n, 1), dtype=torch.float64, device="cuda")
        podsgen.check(ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, 0, E.ptr(lam), E.ptr(Y)), "syev2")
        podsgen.check(ctx.lib.pods_syev2_status(ctx.h), "status")
        A = C.cpu().numpy()
        r0, m = B, n - B
        V, T, R = TP.panel_qr(A[r0:, 0:B])
        taus = np.diag(T)
        A22 = A[r0:, r0:]
        Yr = A22 @ V
        X = Yr @ T
        W = X - 0.5 * V @ (T.T @ (V.T @ X))
        A22n = A22 - V @ W.T - W @ V.T
        gV = get(ctx, n, 4, m * B).reshape(m, B)
        gT = get(ctx, n, 5, B * B).reshape(B, B)
        gtau = get(ctx, n, 6, B)
        gY = get(ctx, n, 7, 4 * m * B).reshape(4, m, B).sum(0)
        gX = get(ctx, n, 8, m * B).reshape(m, B)
        gW = get(ctx, n, 9, m * B).reshape(m, B)
        gA = get(ctx, n, 3, n * n).reshape(n, n)
        sc = np.max(np.abs(A))
        print("n=%d V %.2e tau %.2e T %.2e Y %.2e X %.2e W %.2e A22 %.2e R %.2e" % (
            n, np.max(np.abs(gV - V)), np.max(np.abs(gtau - taus)), np.max(np.abs(gT - T)),
            np.max(np.abs(gY - Yr)) / sc, np.max(np.abs(gX - X)) / sc, np.max(np.abs(gW - W)) / sc,
            np.max(np.abs(gA[r0:, r0:] - A22n)) / sc,
            np.max(np.abs(np.triu(gA[r0:r0 + min(B, m), 0:B]) - R[:min(B, m)])) / sc))


if __name__ == "__main__":
    main()

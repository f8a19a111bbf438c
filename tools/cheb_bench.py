"""Micro-benchmark of pods_cheb_step (the subspace iteration's GEMM step) and the block
kernels at n = 4096, m = 64, and of the whole leading-pair solve on a POD-like matrix, for A/B
runs of the step kernel (PODS_CHEB=lds|w, PODS_CHEB_PD) and rocprofv3 (PMC) runs:
    python tools/cheb_bench.py [reps]"""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))

from podsgen import engine as E  # noqa: E402
from podsgen.subspace import Subspace, _p, leading_eigenpairs  # noqa: E402


def pod_like(n, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    m = n + n // 2
    B = torch.randn(m, n, generator=g, dtype=torch.float64)
    k = torch.exp(-0.5 * (torch.arange(-12, 13, dtype=torch.float64) / 4.0) ** 2)
    Bs = torch.nn.functional.conv1d(B.unsqueeze(1), k.view(1, 1, -1), padding=12).squeeze(1) + 0.05 * B
    Bd = Bs.cuda()
    C = Bd.T @ Bd / m
    return (0.5 * (C + C.T)).contiguous()


def main(reps):
    ctx = E.Context(0)
    n = 4096
    tag = "PODS_CHEB=%s PD=%s" % (os.environ.get("PODS_CHEB", "w"), os.environ.get("PODS_CHEB_PD", "2"))
    C = torch.randn(n, n, dtype=torch.float64, device="cuda")
    C = (C + C.T).contiguous()
    ws = Subspace(ctx, n, 64)
    ws.prepare(C)
    Y = torch.randn(n, 64, dtype=torch.float64, device="cuda")
    Z = torch.randn(n, 64, dtype=torch.float64, device="cuda")
    out = torch.empty_like(Y)
    ws.step(C, Y, Z, 1.0, 0.5, 0.25, out)
    ref = C @ Y + 0.5 * Y + 0.25 * Z
    torch.cuda.synchronize()
    print("%s cheb rel err %.3e" % (tag, float((out - ref).abs().max() / ref.abs().max())), flush=True)
    for name, fn in (("cheb", lambda: ws.step(C, Y, Z, 1.0, 0.5, 0.25, out)),
                     ("cholqr", lambda: ctx.lib.pods_cholqr(ctx.h, _p(Y), n, 64, _p(out))),
                     ("gram", lambda: ctx.lib.pods_gram(ctx.h, _p(Y), _p(Z), n, 64, _p(ws.HF[0])))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        print("%s %s %.1f us" % (tag, name, (time.time() - t) / reps * 1e6), flush=True)
    Cp = pod_like(n, 1)
    lam_ref = torch.flip(torch.linalg.eigvalsh(Cp), (0,))[:20].cpu().numpy()
    ws2 = Subspace(ctx, n, 64)
    best = None
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.time()
        th, X, info = leading_eigenpairs(ctx, Cp, 20, ws=ws2)
        torch.cuda.synchronize()
        dt = (time.time() - t) * 1e3
        best = dt if best is None else min(best, dt)
    print("%s leading_eigenpairs n=%d: %.2f ms (best of 5), degrees %d, residual %.2e, max |dlam|/lam0 %.2e"
          % (tag, n, best, info["degrees"], info["residual"], float(np.max(np.abs(th - lam_ref)) / lam_ref[0])),
          flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)

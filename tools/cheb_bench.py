"""Micro-benchmark of pods_cheb_step (the subspace iteration's GEMM step) and the block
kernels at n = 4096, m = 64, for rocprofv3 (PMC) runs: python tools/cheb_bench.py [reps]"""
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))

from podsgen import engine as E  # noqa: E402
from podsgen.subspace import Subspace, _p  # noqa: E402


def main(reps):
    ctx = E.Context(0)
    n = 4096
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
    print("cheb rel err %.3e" % float((out - ref).abs().max() / ref.abs().max()), flush=True)
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
        print("%s %.1f us" % (name, (time.time() - t) / reps * 1e6), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)

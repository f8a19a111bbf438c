"""Rank 0 of an N-GPU run, on one GPU: does the leading-pair solve of step k-1 (subspace
iteration, engine.eigen_solve's split path) hide beside step k's generation + mean + partial
correlation of rank 0's row slab?  Three timings per world size, wall clock from enqueue to both
streams drained (median of reps):
  G   generate + mean + corr of the slab (main stream, the next step's jump-ahead prefetched)
  L   the solve alone (side stream) on a real correlation matrix of the full problem
  G|L the solve enqueued on the side stream right after G is enqueued on the main stream
    python tools/overlap_rank0.py [J K NS [WORLDS [reps]]]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
WORLDS = [int(w) for w in sys.argv[4].split(",")] if len(sys.argv) > 4 else [2, 4, 8]
REPS = int(sys.argv[5]) if len(sys.argv) > 5 else 7
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=12345)
ctx = E.Context(0)
# a real correlation matrix of the whole problem for the solve
g1 = E.Generator(s, rank=0, world=1, ctx=ctx)
g1.generate()
mean = torch.empty(g1.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")
C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1), "pods_corr")
torch.cuda.synchronize()
del g1, mean
torch.cuda.empty_cache()
side = ctx.side_stream()


def solve():
    with ctx.on_stream(side):
        E.eigen_solve(ctx, C, NS, s.nm, 1e-15, False, world=2, defer_full=True)


for world in WORLDS:
    gen = E.Generator(s, rank=0, world=world, ctx=ctx)
    Cw = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
    mw = torch.empty(gen.rowlen, dtype=torch.float64, device="cuda")

    def G():
        gen.generate()
        gen.prefetch_jump()
        podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mw), 1), "pods_mean")
        podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(Cw), 0), "pods_corr")
        gen.join_ahead()

    res = {"G": [], "L": [], "G|L": []}
    G()
    solve()
    torch.cuda.synchronize()
    for r in range(REPS):
        for name in ("G", "L", "G|L"):
            torch.cuda.synchronize()
            t = time.perf_counter()
            if name in ("G", "G|L"):
                G()
            if name in ("L", "G|L"):
                side.wait_stream(side)  # the solve waits for nothing on the main stream
                solve()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t) * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print("world %d rows [%d,%d): G %.2f ms  L %.2f ms  G|L %.2f ms  (serial %.2f; hidden %.2f of L)" % (
        world, gen.j0, gen.j1, med["G"], med["L"], med["G|L"], med["G"] + med["L"],
        med["G"] + med["L"] - med["G|L"]), flush=True)
    del gen, Cw, mw
    torch.cuda.empty_cache()

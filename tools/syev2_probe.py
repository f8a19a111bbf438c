#!/usr/bin/env python3
"""Time pods_syev2 (two-stage) against pods_syev (n <= 4096) and torch.linalg.eigh on
POD-like matrices; prints one JSON line per n."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pods-digital-filter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402
from test_gpu_eigen import pod_like  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts)


def main():
    ctx = E.Context(0)
    for n in [int(x) for x in (sys.argv[1:] or ["4096", "8192"])]:
        C = pod_like(n, seed=1)
        lam = torch.empty(n, dtype=torch.float64, device="cuda")
        Y = torch.empty((n, 20), dtype=torch.float64, device="cuda")
        out = {"n": n}
        out["syev2_ms"] = timed(lambda: podsgen.check(ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, 20, E.ptr(lam),
                                                                          E.ptr(Y)), "pods_syev2"))
        podsgen.check(ctx.lib.pods_syev2_status(ctx.h), "status")
        out["syev2_values_only_ms"] = timed(lambda: podsgen.check(
            ctx.lib.pods_syev2(ctx.h, E.ptr(C), n, 0, E.ptr(lam), E.ptr(Y)), "pods_syev2"))
        if n <= 4096:
            out["syev_ms"] = timed(lambda: podsgen.check(ctx.lib.pods_syev(ctx.h, E.ptr(C), n, 20, E.ptr(lam),
                                                                            E.ptr(Y)), "pods_syev"))
        out["torch_eigh_ms"] = timed(lambda: torch.linalg.eigh(C), reps=1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""A/B of the mean kernels on the C3 snapshot matrix in one process, alternating round by round
(PODS_MEAN=row: one thread per row, k_mean; default: k_mean_leaves); the means and devmax of every
configuration must equal the first's bit for bit.
    python tools/mean_ab.py rounds"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
s = podsgen.DFSetup(jma=256, kma=256, ns=4096, seed=3)
gen = E.Generator(s, device=0)
snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
configs = ["-", "row"]
res = {v: [] for v in configs}
ref = None
for r in range(rounds):
    for v in configs:
        os.environ.pop("PODS_MEAN", None)
        if v != "-":
            os.environ["PODS_MEAN"] = v
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
        e1.record()
        e1.synchronize()
        res[v].append(e0.elapsed_time(e1))
        cur = mean.clone()
        if ref is None:
            ref = cur
        elif not torch.equal(cur.view(torch.int64), ref.view(torch.int64)):
            print("config %s: mean differs from the first configuration" % v, flush=True)
    print("round %d: %s" % (r, "  ".join("%s %.3f" % (v, res[v][-1]) for v in configs)), flush=True)
for v in configs:
    x = sorted(res[v])
    print("%-6s median %.3f ms  min %.3f  (%.2f TB/s of A)" % (v, x[len(x) // 2], x[0],
                                                             snap.rowlen * 4096 * 8 / x[len(x) // 2] / 1e9), flush=True)

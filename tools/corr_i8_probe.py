"""pods_corr at J x K x NS: the exact int8 correlation (mode 1) against the fp64 MFMA SYRK
(mode 0) on a generated snapshot matrix -- times and the largest difference.
    python tools/corr_i8_probe.py J K NS reps"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=1)
gen = E.Generator(s, device=0)
snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
ops = 16.0 * 3 * J * K * NS * (NS + 1)
flops = 3.0 * J * K * NS * (NS + 1)


def run(mode, tag):
    ctx.set_corr_mode(mode)
    C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1))
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    med = ts[len(ts) // 2]
    print("%s corr median %.2f ms (min %.2f)  fp64-equivalent %.1f TFLOP/s%s" % (
        tag, med * 1e3, ts[0] * 1e3, flops / med / 1e12,
        ("  int8 %.0f TOP/s (16 residue SYRKs)" % (ops / med / 1e12)) if mode == 1 else ""), flush=True)
    return C


C1 = run(1, "int8-crt")
podsgen.check(ctx.lib.pods_center(ctx.h))
C0 = run(0, "fp64    ")
cm = float(C0.abs().max())
print("max |C_i8 - C_f64| / max|C| = %.3e   symmetric %s" % (float((C1 - C0).abs().max()) / cm,
                                                         bool(torch.equal(C1, C1.T))), flush=True)

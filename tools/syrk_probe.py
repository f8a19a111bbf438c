"""Time pods_corr alone at J x K x NS: python tools/syrk_probe.py J K NS reps [regen]
(regen: generate + mean + centre before every timed call, as in a pipeline step)"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import numpy as np, torch, podsgen
from podsgen import engine as E
J, K, NS = (int(a) for a in sys.argv[1:4]); reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=1)
gen = E.Generator(s, device=0); snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
podsgen.check(ctx.lib.pods_center(ctx.h))  # the production path: A centred in place
C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
flops = 3 * J * K * NS * (NS + 1)
regen = len(sys.argv) > 5 and sys.argv[5] == "regen"
for r in range(reps):
    if regen:
        gen.generate()
        podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
        podsgen.check(ctx.lib.pods_center(ctx.h))
    torch.cuda.synchronize(); t = time.time()
    podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1))
    torch.cuda.synchronize(); dt = time.time() - t
    print("corr %.2f ms  %.1f TFLOP/s (triangle flops)" % (dt * 1e3, flops / dt / 1e12), flush=True)
# correctness of the last C: sampled 256 x 256 tiles against torch's A_c^T A_c / ns
import ctypes
def _blk(i0, i1):
    out = torch.empty((i1 - i0, gen.rowlen), dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_copy_snapshots(ctx.h, i0, i1, ctypes.c_void_p(out.data_ptr())), "copy")
    return out
cm = float(C.abs().max())
worst = 0.0
for bi, bj in [(0, 0), (NS // 256 - 1, 0), (NS // 512, NS // 1024)]:
    X, Y = _blk(bi * 256, bi * 256 + 256), _blk(bj * 256, bj * 256 + 256)
    ref = X @ Y.T / NS
    worst = max(worst, float((C[bi * 256:bi * 256 + 256, bj * 256:bj * 256 + 256] - ref).abs().max()) / cm)
print("check max rel err %.3e symmetric %s" % (worst, bool(torch.equal(C, C.T))), flush=True)

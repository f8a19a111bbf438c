"""Time pods_spatial_modes_dev at a generated C3 field (J K NS, nm = 20), HIP events around each
call, median of reps; run once per library (PODSGEN_LIB=...) to A/B kernel variants:
    python tools/spatial_ab.py [reps] [J K NS]
Prints the median and a checksum of Phi (to compare variants bit for bit)."""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
J, K, NS = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (256, 256, 4096)
NM = 20
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=3)
gen = E.Generator(s, device=0)
snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
g = torch.Generator(device="cpu").manual_seed(5)
T = torch.randn(NS, NM, generator=g, dtype=torch.float64).cuda()
lam = (torch.rand(NM, generator=g, dtype=torch.float64) + 0.5).cuda()
phi = torch.empty(snap.rowlen, NM, dtype=torch.float64, device="cuda")
ts = []
for r in range(reps + 3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    podsgen.check(ctx.lib.pods_spatial_modes_dev(ctx.h, E.ptr(T), NM, E.ptr(lam), NM, E.ptr(phi)))
    e1.record()
    e1.synchronize()
    if r >= 3:
        ts.append(e0.elapsed_time(e1))
ts.sort()
print("pods_spatial_modes median %.3f ms (min %.3f)  phi sha1 %s  lib %s" % (
    ts[len(ts) // 2], ts[0], hashlib.sha1(phi.cpu().numpy().tobytes()).hexdigest()[:16],
    os.path.basename(os.environ.get("PODSGEN_LIB", "product"))), flush=True)

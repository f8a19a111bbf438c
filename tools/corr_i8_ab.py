"""A/B of int8 SYRK configurations inside one process at C3, alternating round by round; the
SYRK kernel timed by the library's HIP events (pods_corr_timing).  A configuration is a set of
environment assignments joined by ',' (e.g. PODS_SYRK_I8=5,PODS_CORR_ORDER=x; '-' = defaults).
    python tools/corr_i8_ab.py rounds config [config ...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

KEYS = ("PODS_SYRK_I8", "PODS_CORR_ORDER", "PODS_CORR_SPLITS", "PODS_RES_I8", "PODS_RES_LAYOUT", "PODS_SYRK_PACE", "PODS_SYRK_WIDE", "PODS_SYRK_LEAD", "PODS_SYRK_DMA")
rounds = int(sys.argv[1])
configs = sys.argv[2:]
J, K, NS = 256, 256, 4096
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=1)
gen = E.Generator(s, device=0)
snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
ops = 16.0 * 3 * J * K * NS * (NS + 1)
res = {v: [] for v in configs}
tot = {v: [] for v in configs}  # the whole pods_corr (residues + SYRK + CRT), CUDA events
ref = None
for r in range(rounds):
    for v in configs:
        for k in KEYS:
            os.environ.pop(k, None)
        if v != "-":
            for kv in v.split(","):
                k, val = kv.split("=")
                os.environ[k] = val
        podsgen.check(ctx.lib.pods_corr_timing(ctx.h, 1))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1))
        e1.record()
        e1.synchronize()
        tot[v].append(e0.elapsed_time(e1))
        ms, n = ctypes.c_double(), ctypes.c_int()
        podsgen.check(ctx.lib.pods_corr_kernel_ms(ctx.h, ctypes.byref(ms), ctypes.byref(n)))
        res[v].append(ms.value)
        if "9" not in v:
            if ref is None:
                ref = C.clone()
            elif not torch.equal(C, ref):
                print("config %s: C differs from the first configuration" % v, flush=True)
    print("round %d: %s" % (r, "  ".join("%s %.2f" % (v, res[v][-1]) for v in configs)), flush=True)
import hashlib  # noqa: E402
print("C sha1 %s (lib %s)" % (hashlib.sha1(C.cpu().numpy().tobytes()).hexdigest()[:16], os.environ.get("PODSGEN_LIB", "product")), flush=True)
for v in configs:
    x = sorted(res[v])
    med = x[len(x) // 2]
    tt = sorted(tot[v])
    print("%-40s median %.2f ms  min %.2f  (%.0f TOP/s, %.3f of 5033)  whole corr median %.2f ms" % (
        v, med, x[0], ops / med / 1e9, ops / med / 1e9 / 5033, tt[len(tt) // 2]), flush=True)

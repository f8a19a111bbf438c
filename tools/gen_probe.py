"""Generation-stage probe: the fused x+y+z pass (k_filter_xyz) against the two-pass path
(k_filter_x2 + k_filter_yz) and bit-for-bit equality of the snapshot matrices.
   python tools/gen_probe.py [J K NS [reps]]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=12345)
out = {}
for fused in ("1", "0"):
    os.environ["PODS_GEN_FUSED"] = fused
    ctx = E.Context(0)
    gen = E.Generator(s, ctx=ctx)
    rowpad = (gen.rowlen + 15) // 16 * 16
    for r in range(reps):
        tm = E.StageTimer()
        with tm("generate"):
            snap = gen.generate()
        st = tm.summary()
        print("fused=%s rep %d: generate %.3f ms" % (fused, r, st["generate"]), flush=True)
    A = torch.empty(NS * rowpad, dtype=torch.float64, device="cuda")
    podsgen.check(ctx.lib.pods_copy(ctx.h, E.ptr(A), E.ctypes.c_void_p(snap.data_ptr()), A.numel() * 8, 2))
    torch.cuda.synchronize()
    out[fused] = A
    del gen, ctx
    torch.cuda.empty_cache()
print("fused == two-pass generation:", torch.equal(out["1"], out["0"]), flush=True)

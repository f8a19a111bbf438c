"""A/B of generator configurations in one process, alternating round by round: per part of
pods_df_generate_parts (jump-ahead, random planes, x pass, y/z pass) the HIP-event time on the
main stream, for rank 0's row slab at the given world sizes; the snapshot matrix of every
configuration must equal the first one's bit for bit.  A configuration is a set of environment
assignments joined by ',' ('-' = defaults), e.g. PODS_MT_GEN=lds.
    python tools/gen_ab.py rounds J K NS worlds config [config ...]     (worlds: e.g. 1,8)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import _lib  # noqa: E402
from podsgen import engine as E  # noqa: E402

KEYS = ("PODS_MT_GEN", "PODS_MT_SUBSTREAMS")
rounds = int(sys.argv[1])
J, K, NS = (int(a) for a in sys.argv[2:5])
worlds = [int(w) for w in sys.argv[5].split(",")]
configs = sys.argv[6:]
# the x and y/z passes in one call
PARTS = [("jump", _lib.PODS_GEN_JUMP), ("planes", _lib.PODS_GEN_PLANES),
         ("xyz", _lib.PODS_GEN_XPASS | _lib.PODS_GEN_YZPASS)]
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=4242)
ctx = E.Context(0)
for world in worlds:
    gen = E.Generator(s, rank=0, world=world, ctx=ctx)
    ref = None
    res = {v: {p: [] for p, _ in PARTS} for v in configs}
    for r in range(rounds):
        for v in configs:
            for k in KEYS:
                os.environ.pop(k, None)
            if v != "-":
                for kv in v.split(","):
                    k, val = kv.split("=")
                    os.environ[k] = val
            torch.cuda.synchronize()
            for name, bit in PARTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                podsgen.check(ctx.lib.pods_df_generate_parts(ctx.h, bit), "pods_df_generate_parts")
                e1.record()
                e1.synchronize()
                res[v][name].append(e0.elapsed_time(e1))
            p = ctypes.c_void_p()
            n = ctypes.c_int64()
            podsgen.check(ctx.lib.pods_df_snapshots(ctx.h, ctypes.byref(p), ctypes.byref(n)), "snapshots")
            nbytes = n.value * 8 if n.value < (1 << 40) else 0
            rowpad = (gen.rowlen + 15) // 16 * 16
            cur = torch.empty(rowpad * NS, dtype=torch.float64, device="cuda")
            podsgen.check(ctx.lib.pods_copy(ctx.h, ctypes.c_void_p(cur.data_ptr()), p, cur.numel() * 8, 2), "copy")
            torch.cuda.synchronize()
            if ref is None:
                ref = cur
            elif not torch.equal(cur.view(torch.int64), ref.view(torch.int64)):
                print("world %d config %s: snapshots differ from the first configuration" % (world, v), flush=True)
        print("world %d round %d: %s" % (world, r, "  ".join(
            "%s [%s]" % (v, " ".join("%s %.3f" % (p, res[v][p][-1]) for p, _ in PARTS)) for v in configs)), flush=True)
    for v in configs:
        med = {p: sorted(x)[len(x) // 2] for p, x in res[v].items()}
        print("world %d %-30s median %s  sum %.3f ms" % (world, v, " ".join("%s %.3f" % kv for kv in med.items()),
                                                         sum(med.values())), flush=True)
    del gen, ref
    torch.cuda.empty_cache()

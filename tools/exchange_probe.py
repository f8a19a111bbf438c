"""Per-rank generation time of rank 0's row slab with and without the MT19937 state exchange
(pods_df_set_exchange), on one GPU: HIP-event time per part on the main stream.  Without the
exchange every rank twists the whole stream (jump + planes); with it, rank 0 jumps and twists its
1/world share (jump, record), then regenerates its own segments (planes).  The all_to_all itself
is not run here (one GPU): its bytes per rank are printed (received records x 2.5 KB); the
receive buffer is filled with rank 0's own records so the twist runs on valid states.
    python tools/exchange_probe.py [J K NS [WORLDS [reps]]]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import _lib  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
WORLDS = [int(w) for w in sys.argv[4].split(",")] if len(sys.argv) > 4 else [2, 4, 8]
REPS = int(sys.argv[5]) if len(sys.argv) > 5 else 5
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=4242)
ctx = E.Context(0)


def timed(parts_list, prep=None):
    out = {}
    for name, bit in parts_list:
        if prep is not None and name == "planes":
            prep()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        podsgen.check(ctx.lib.pods_df_generate_parts(ctx.h, bit), "pods_df_generate_parts")
        e1.record()
        e1.synchronize()
        out[name] = e0.elapsed_time(e1)
    return out


BASE = [("jump", _lib.PODS_GEN_JUMP), ("planes", _lib.PODS_GEN_PLANES), ("x", _lib.PODS_GEN_XPASS),
        ("yz", _lib.PODS_GEN_YZPASS)]
XCH = [("jump", _lib.PODS_GEN_JUMP), ("record", _lib.PODS_GEN_RECORD), ("planes", _lib.PODS_GEN_PLANES),
       ("x", _lib.PODS_GEN_XPASS), ("yz", _lib.PODS_GEN_YZPASS)]
for world in WORLDS:
    for mode in ("whole-stream", "exchange"):
        gen = E.Generator(s, rank=0, world=world, ctx=ctx, exchange=False)
        parts = BASE
        prep = None
        if mode == "exchange":
            gen.enable_exchange()
            parts = XCH
            n_r = sum(gen._xch[1])

            def prep(gen=gen, n_r=n_r):
                src = gen._send[:min(n_r, gen._send.numel())]
                gen._recv[:src.numel()].copy_(src)
        res = {}
        for r in range(REPS + 1):
            t = timed(parts, prep)
            if r:
                for k, v in t.items():
                    res.setdefault(k, []).append(v)
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        extra = ""
        if mode == "exchange":
            extra = "  all_to_all: sends %.1f MB, receives %.1f MB" % (sum(gen._xch[0]) / 1e6, sum(gen._xch[1]) / 1e6)
        print("world %d %-12s %s  sum %.3f ms (without jump %.3f)%s" % (
            world, mode, " ".join("%s %.3f" % kv for kv in med.items()), sum(med.values()),
            sum(med.values()) - med["jump"], extra), flush=True)
        del gen
        torch.cuda.empty_cache()

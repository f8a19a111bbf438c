"""Test helper: the multi-GPU MT19937 state exchange of `world` ranks emulated on ONE device and ONE
pods context (podsgen.h pods_df_set_exchange; engine.Generator.enable_exchange).

Phase 1, rank by rank: the rank's own substreams are jumped and twisted once, and the segment-start
states of every rank's row segments that fall in them are recorded (PODS_GEN_JUMP | PODS_GEN_RECORD)
into the rank's send buffer, which is kept (a copy).  Phase 2, rank by rank: the rank's receive
buffer is assembled exactly as one all_to_all_single would (rank r's chunk for q, concatenated over
r), and the rank regenerates its own segments from it (PODS_GEN_PLANES) and filters them (x, y/z
passes); visit(q, gen) then reads what it needs from the slab.  The context is reconfigured for
every rank, so only one rank's buffers are allocated at a time (C5 slabs: ~170 GB each).
"""
import torch

import podsgen
from podsgen import _lib
from podsgen import engine as E


def emulate_exchange(setup, ctx, world, visit):
    sends, sizes = [], []
    for r in range(world):
        g = E.Generator(setup, ctx=ctx, rank=r, world=world, exchange=False)
        assert g.enable_exchange()
        podsgen.check(ctx.lib.pods_df_generate_parts(ctx.h, _lib.PODS_GEN_JUMP | _lib.PODS_GEN_RECORD), "record")
        sb = g._xch[0]
        sends.append(g._send[:sum(sb)].clone())
        sizes.append(sb)
        del g
    torch.cuda.synchronize()
    for q in range(world):
        g = E.Generator(setup, ctx=ctx, rank=q, world=world, exchange=False)
        assert g.enable_exchange()
        chunks = [sends[r][sum(sizes[r][:q]):sum(sizes[r][:q + 1])] for r in range(world)]
        recv = torch.cat(chunks)
        assert recv.numel() == sum(g._xch[1])
        g._recv[:recv.numel()].copy_(recv)
        podsgen.check(ctx.lib.pods_df_generate_parts(
            ctx.h, _lib.PODS_GEN_PLANES | _lib.PODS_GEN_XPASS | _lib.PODS_GEN_YZPASS), "segments")
        visit(q, g)
        del g

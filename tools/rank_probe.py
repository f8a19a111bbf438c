"""Per-rank compute of the sharded path on ONE GPU (what each rank of an N-GPU run does before
the all-reduce): generate + mean (+ centre with the fp64 SYRK) + partial correlation for rank 0's row slab at world = 1, 2,
4, 8, in steady state, without and with the next step's MT19937 jump-ahead on the gen stream
(Generator.prefetch_jump, as bench.py runs it).
   python tools/rank_probe.py [J K NS [WORLDS]]   (WORLDS: comma-separated, default 1,2,4,8)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
WORLDS = [int(w) for w in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 4, 8]
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=12345)
ctx = E.Context(0)
MODES = [("plain", False, False, False), ("prefetched", True, False, False), ("exchange", True, True, False),
         ("exchange+early jump", True, True, True)]
for world in WORLDS:
  for mode, ahead, xch, early in MODES:
    if xch and world == 1:
        continue
    gen = E.Generator(s, rank=0, world=world, ctx=ctx, exchange=False)
    a2a = ""
    if xch:
        # the MT19937 state exchange (pods_df_set_exchange): this rank's own substreams, then the
        # all_to_all -- emulated on one GPU by a local copy of this rank's records (the twist is
        # data-independent); its bytes are printed for the xGMI estimate
        gen.enable_exchange()
        n_s, n_r = sum(gen._xch[0]), sum(gen._xch[1])

        def local_a2a(gen=gen, n=min(n_s, n_r)):
            gen._recv[:n].copy_(gen._send[:n])
        gen.exchange_states = local_a2a
        a2a = "  all_to_all %.1f MB out / %.1f MB in per rank (not timed here)" % (n_s / 1e6, n_r / 1e6)
    C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
    mean = torch.empty(gen.rowlen, dtype=torch.float64, device="cuda")
    if True:
        reps, walls = 5, []
        for rep in range(reps):
            tm = E.StageTimer()
            torch.cuda.synchronize()
            t = time.perf_counter()
            if early and ahead and rep < reps - 1:
                gen.prefetch_jump_early(tm)
            with tm("generate"):
                gen.generate()
            if ahead and rep < reps - 1:
                gen.prefetch_jump(tm)
            with tm("mean"):
                podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")
            if ctx.corr_mode() == 0:  # the fp64 SYRK reads A centred (run_pod does the same)
                with tm("center"):
                    podsgen.check(ctx.lib.pods_center(ctx.h), "pods_center")
            with tm("corr"):
                podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 0), "pods_corr")
            gen.join_ahead()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t) * 1e3)
            if rep == reps - 2:
                st = tm.summary()
        print("world %d rows [%d,%d) %s: %s  step wall %.2f ms%s" % (
            world, gen.j0, gen.j1, mode,
            {k: round(v, 2) for k, v in st.items()}, sum(walls[1:-1]) / (reps - 2), a2a), flush=True)
    del gen, C, mean
    torch.cuda.empty_cache()

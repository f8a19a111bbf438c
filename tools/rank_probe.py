"""Per-rank compute of the sharded path on ONE GPU (what each rank of an N-GPU run does before
the all-reduce): generate + mean + partial SYRK for rank 0's row slab at world = 1, 2, 4, 8.
   python tools/rank_probe.py [J K NS]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch  # noqa: E402

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=12345)
ctx = E.Context(0)
for world in (1, 2, 4, 8):
    gen = E.Generator(s, rank=0, world=world, ctx=ctx)
    C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
    mean = torch.empty(gen.rowlen, dtype=torch.float64, device="cuda")
    for rep in range(2):
        tm = E.StageTimer()
        with tm("generate"):
            gen.generate()
        with tm("mean"):
            podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1), "pods_mean")
        with tm("corr"):
            podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 0), "pods_corr")
        st = tm.summary()
    print("world %d rows [%d,%d): %s  total %.2f ms" % (world, gen.j0, gen.j1,
          {k: round(v, 2) for k, v in st.items()}, sum(st.values())), flush=True)
    del gen, C, mean
    torch.cuda.empty_cache()

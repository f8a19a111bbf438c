"""Does HBM-bound work overlap the MFMA-bound SYRK?  python tools/overlap_probe.py [J K NS]

Times, at C3 by default: pods_corr alone, the concurrent load alone (pods_mean x M, and the
whole pods_df_generate), then each load launched on a second stream beside pods_corr.  Data
races are deliberate (timing only: the numbers written are not used)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import torch, podsgen
from podsgen import engine as E

J, K, NS = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 4096)
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=1)
gen = E.Generator(s, device=0)
snap = gen.generate()
ctx = gen.ctx
mean = torch.empty(snap.rowlen, dtype=torch.float64, device="cuda")
podsgen.check(ctx.lib.pods_mean(ctx.h, E.ptr(mean), 1))
podsgen.check(ctx.lib.pods_center(ctx.h))
C = torch.empty((NS, NS), dtype=torch.float64, device="cuda")
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def on(st):
    podsgen.check(ctx.lib.pods_set_stream(ctx.h, ctypes_ptr(st)))


def ctypes_ptr(st):
    import ctypes
    return ctypes.c_void_p(st.cuda_stream)


def corr():
    podsgen.check(ctx.lib.pods_corr(ctx.h, E.ptr(C), 1))


def means(m):
    for _ in range(m):
        podsgen.check(ctx.lib.pods_mean(ctx.h, None, 1))


def generate():
    podsgen.check(ctx.lib.pods_df_generate(ctx.h))
    # generate clears the mean/centred state: restore it so the next pods_corr is accepted
    podsgen.check(ctx.lib.pods_mean(ctx.h, None, 1))
    podsgen.check(ctx.lib.pods_center(ctx.h))


def timed(fn_a, fn_b=None):
    torch.cuda.synchronize()
    ea0, ea1, eb0, eb1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    t = time.time()
    with torch.cuda.stream(sa):
        ea0.record(sa)
        on(sa)
        fn_a()
        ea1.record(sa)
    if fn_b is not None:
        with torch.cuda.stream(sb):
            eb0.record(sb)
            on(sb)
            fn_b()
            eb1.record(sb)
    torch.cuda.synchronize()
    wall = (time.time() - t) * 1e3
    a = ea0.elapsed_time(ea1)
    b = eb0.elapsed_time(eb1) if fn_b is not None else 0.0
    return wall, a, b


for rep in range(2):
    w, a, _ = timed(corr)
    print("corr alone           wall %7.2f  corr %7.2f" % (w, a), flush=True)
    w, a, _ = timed(lambda: means(20))
    print("mean x20 alone       wall %7.2f  load %7.2f" % (w, a), flush=True)
    w, a, b = timed(corr, lambda: means(20))
    print("corr || mean x20     wall %7.2f  corr %7.2f  load %7.2f" % (w, a, b), flush=True)
    w, a, _ = timed(generate)
    print("gen+mean+ctr alone       wall %7.2f  load %7.2f" % (w, a), flush=True)
    w, a, b = timed(corr, generate)
    print("corr || gen+mean+ctr wall %7.2f  corr %7.2f  load %7.2f" % (w, a, b), flush=True)

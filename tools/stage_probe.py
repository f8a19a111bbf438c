"""Stage timing probe: python tools/stage_probe.py J K NS [reps]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import numpy as np
import torch
import podsgen
from podsgen import engine as E

J, K, NS = (int(a) for a in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
s = podsgen.DFSetup(jma=J, kma=K, ns=NS, seed=12345)
t0 = time.time()
gen = E.Generator(s, device=0)
print("configure %.3f s" % (time.time() - t0), flush=True)
for r in range(reps):
    tm = E.StageTimer()
    torch.cuda.synchronize(); t0 = time.time()
    g, pod, fo = E.pipeline(s, gen=gen, timer=tm)
    torch.cuda.synchronize(); wall = time.time() - t0
    st = tm.summary()
    print("rep %d wall %.1f ms  %s  nm=%d valid=%d  Mpts/s=%.0f" % (
        r, wall * 1e3, {k: round(v, 2) for k, v in st.items()}, pod.nm, pod.num_valid,
        J * K * NS / wall / 1e6), flush=True)

"""Debug probe for pods_fourier_rank at large ns (GPU)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pods-digital-filter_amd"))
import numpy as np, torch
import podsgen
from podsgen import engine as E
ctx = E.Context(0)
rng = np.random.default_rng(11)
for ns, nm in [(8192, 2), (8193, 2), (12000, 1), (16384, 2)]:
    c = (rng.standard_normal((ns, nm)) + 1j * rng.standard_normal((ns, nm))).astype(np.complex64)
    cdev = torch.from_numpy(np.ascontiguousarray(c).view(np.float32).reshape(ns, nm, 2)).cuda()
    ind = torch.empty((nm, ns), dtype=torch.int32, device="cuda")
    cnt = torch.empty(nm, dtype=torch.int64, device="cuda")
    podsgen.check(ctx.lib.pods_fourier_rank(ctx.h, E.ptr(cdev), nm, ns, 0.9, E.ptr(ind), E.ptr(cnt)), "rank")
    ci = ind.cpu().numpy()
    ref, rc, _ = E.host_rank_and_count(c, 0.9)
    for i in range(nm):
        bad = np.nonzero(ci[i] != ref[i])[0]
        cm = np.abs(c[:, i])
        print(ns, i, "mismatches", len(bad), bad[:8], "sorted?", bool(np.all(np.diff(cm[ci[i]]) <= 0)),
              "perm?", len(set(ci[i].tolist())) == ns, cnt.cpu().numpy()[i], rc[i])

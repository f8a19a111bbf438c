"""GPU probe of the leading-eigenpair solver (podsgen.subspace) on the real C3 matrix:
accuracy against eigh and time per configuration; run under rocprofv3 for the kernel split.

usage: python tools/topk_probe.py [out_dir] [reps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))
sys.path.insert(0, HERE)

from subspace_probe import c3_matrix  # noqa: E402
from podsgen.subspace import Subspace, leading_eigenpairs  # noqa: E402


def main(out, reps):
    os.makedirs(out, exist_ok=True)
    gen, C = c3_matrix()
    n, k = C.shape[0], 20
    lr, Vr = torch.linalg.eigh(C)
    lam = torch.flip(lr, (0,)).cpu().numpy()
    Vh = torch.flip(Vr, (1,))[:, :k].cpu().numpy()
    ws = Subspace(gen.ctx, n, 64)
    rows = []
    configs = ((0.85, 1.05, 20), (0.9, 1.05, 16))
    if len(sys.argv) > 3:   # e.g. "0.8,1.1,8;0.7,1.2,8" (rate_factor, margin, warm)
        configs = [tuple(float(v) for v in c.split(",")) for c in sys.argv[3].split(";")]
        configs = [(a, b, int(c)) for a, b, c in configs]
    for rf, mg, wm in configs:
        for rep in range(reps):
            torch.cuda.synchronize()
            t = time.time()
            th, X, info = leading_eigenpairs(gen.ctx, C, k, m=64, rate_factor=rf, margin=mg, warm=wm, ws=ws)
            torch.cuda.synchronize()
            dt = time.time() - t
        Xh = X.cpu().numpy()
        err = max(float(np.max(np.abs(np.sign(np.dot(Xh[:, j], Vh[:, j])) * Xh[:, j] - Vh[:, j]))) for j in range(k))
        rows.append(dict(rate_factor=rf, margin=mg, warm=wm, ms=dt * 1e3, vec_err=err,
                         lam_err=float(np.max(np.abs(th - lam[:k])) / lam[0]), **info))
        print(json.dumps(rows[-1]), flush=True)
    # convergence per round for a fixed schedule and several damped-interval edges
    for ci, sched in ((63, [16] * 6), (59, [16] * 6), (55, [16] * 6), (59, [8] + [16] * 5), (59, [24] * 4),
                      (59, [12] * 8)):
        th, X, info = leading_eigenpairs(gen.ctx, C, k, m=64, cut_index=ci, schedule=sched, tol=1e-300, ws=ws)
        cuts = [(d, c / lam[0], int(np.searchsorted(-lam, -c))) for d, c in info["cuts"]]
        rows.append(dict(cut_index=ci, schedule=sched, hist=info["hist"], cuts=cuts))
        print(json.dumps(rows[-1]), flush=True)
    with open(os.path.join(out, "topk_probe.json"), "w") as f:
        json.dump(rows, f)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/topk", int(sys.argv[2]) if len(sys.argv) > 2 else 2)

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
    for warm, deg, ch in ((8, 12, 3), (8, 12, 4), (8, 16, 3), (10, 20, 2), (8, 10, 5), (6, 24, 2)):
        for rep in range(reps):
            torch.cuda.synchronize()
            t = time.time()
            th, X, info = leading_eigenpairs(gen.ctx, C, k, m=64, degree=deg, chunks=ch, warm=warm, ws=ws)
            torch.cuda.synchronize()
            dt = time.time() - t
        Xh = X.cpu().numpy()
        err = max(float(np.max(np.abs(np.sign(np.dot(Xh[:, j], Vh[:, j])) * Xh[:, j] - Vh[:, j]))) for j in range(k))
        rows.append(dict(warm=warm, deg=deg, chunks=ch, ms=dt * 1e3, vec_err=err,
                         lam_err=float(np.max(np.abs(th - lam[:k])) / lam[0]), **info))
        print(json.dumps(rows[-1]), flush=True)
    with open(os.path.join(out, "topk_probe.json"), "w") as f:
        json.dump(rows, f)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/topk", int(sys.argv[2]) if len(sys.argv) > 2 else 2)

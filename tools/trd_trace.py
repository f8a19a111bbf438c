"""Per-column stage timing of the tridiagonalisation (pods_sytrd_trace) on a POD-like matrix.

usage: python tools/trd_trace.py [n] [wg ...]
Prints, per 512-column range, the mean of each stage (us) for the traced workgroups.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))
sys.path.insert(0, HERE)

from podsgen._lib import check, ptr  # noqa: E402
from podsgen.engine import Context  # noqa: E402
from eig_probe import corr_like  # noqa: E402

STAGES = ["wait", "dot+B1", "col+B2", "hh", "symv", "B3", "pub+upd"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    wgs = [int(a) for a in sys.argv[2:]] or [0, 77, 255]
    ctx = Context(0)
    C = corr_like(n).contiguous()
    d = np.zeros(n)
    e = np.zeros(n)
    check(ctx.lib.pods_sytrd(ctx.h, ptr(C), n, ptr(d), ptr(e)), "warm")
    for wg in wgs:
        tr = np.zeros((n, 8), dtype=np.int64)
        check(ctx.lib.pods_sytrd_trace(ctx.h, ptr(C), n, wg, ptr(tr)), "pods_sytrd_trace")
        spins = tr[:, 1] >> 48
        tr[:, 1] &= (1 << 48) - 1
        ok = tr[:, 0] > 0
        dt = np.diff(tr, axis=1) * 0.01  # 100 MHz -> us
        per = (tr[1:, 0] - tr[:-1, 0]) * 0.01
        print(f"workgroup {wg}: {ok.sum()} traced columns, total {(tr[ok][-1, 7] - tr[ok][0, 0]) * 1e-5:.2f} ms")
        for k in range(0, n, 512):
            sel = np.zeros(n, bool)
            sel[k:k + 512] = True
            sel &= ok
            sel[-1] = False
            if sel.sum() < 2:
                continue
            st = dt[sel].mean(axis=0)
            cyc = per[sel[:-1]].mean()
            print(f"  cols {k:5d}+: spins {spins[sel].mean():5.2f} per column {cyc:6.2f} us | " +
                  " ".join(f"{nm} {v:5.2f}" for nm, v in zip(STAGES, st)), flush=True)


if __name__ == "__main__":
    main()

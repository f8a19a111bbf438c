"""Cross-workgroup view of the tridiagonalisation hand-off (pods_sytrd_trace, all workgroups).

For column j: publish = when the last workgroup passed its row-sum barrier in column j-1
(it stores p right after), arrive = when a workgroup's inputs for column j were complete.
usage: python tools/trd_hop.py [n]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))
sys.path.insert(0, HERE)

from podsgen._lib import check, ptr  # noqa: E402
from podsgen.engine import Context  # noqa: E402
from eig_probe import corr_like  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ctx = Context(0)
    C = corr_like(n).contiguous()
    d = np.zeros(n)
    e = np.zeros(n)
    check(ctx.lib.pods_sytrd(ctx.h, ptr(C), n, ptr(d), ptr(e)), "warm")
    tr = np.zeros((256, n, 8), dtype=np.int64)
    check(ctx.lib.pods_sytrd_trace(ctx.h, ptr(C), n, -1, ptr(tr)), "trace")
    tr[:, :, 1] &= (1 << 48) - 1
    G = min(256, n)
    tr = tr[:G].astype(np.float64) * 0.01  # us
    for k in range(0, n - 1, 512):
        js = np.arange(max(k, 1) + 8, min(k + 512, n - 1) - 8)
        js = js[(tr[:, js, 0] > 0).all(axis=0) & (tr[:, js - 1, 6] > 0).all(axis=0)]
        if len(js) < 4:
            continue
        pub_last = tr[:, js - 1, 6].max(axis=0)          # last producer passes B3 in column j-1
        pub_first = tr[:, js - 1, 6].min(axis=0)
        start = tr[:, js, 0]                               # consumers start column j
        arrive = tr[:, js, 1]
        print(f"cols {k:5d}+: B3 skew {np.mean(pub_last - pub_first):5.2f} | "
              f"start-after-last-pub {np.mean(start.mean(axis=0) - pub_last):6.2f} | "
              f"arrive-after-last-pub mean {np.mean(arrive.mean(axis=0) - pub_last):5.2f} "
              f"max {np.mean(arrive.max(axis=0) - pub_last):5.2f} | arrive skew "
              f"{np.mean(arrive.max(axis=0) - arrive.min(axis=0)):5.2f} | column "
              f"{np.mean(np.diff(tr[0, js, 0])):5.2f}", flush=True)


if __name__ == "__main__":
    main()

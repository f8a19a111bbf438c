"""Time pods_syev (n = 4096, nvec = 20) on a POD-like correlation matrix, CUDA events, median of
reps; run once per setting of an environment knob read at library load (e.g. PODS_BISECT_BL):
    PODS_BISECT_BL=32 python tools/syev_ab.py [reps]
Prints the median, the eigenvalues' max relative difference to torch.linalg.eigvalsh and a
checksum of the spectrum (to compare settings bit for bit)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))
sys.path.insert(0, HERE)

from podsgen import engine as E  # noqa: E402
from podsgen.engine import check, ptr  # noqa: E402
from cheb_bench import pod_like  # noqa: E402


def main(reps):
    ctx = E.Context(0)
    n, nvec = 4096, 20
    C = pod_like(n, 1)
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    Y = torch.empty(n, nvec, dtype=torch.float64, device="cuda")
    ts = []
    for r in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(ctx.lib.pods_syev(ctx.h, ptr(C), n, nvec, ptr(lam), ptr(Y)), "pods_syev")
        e1.record()
        e1.synchronize()
        check(ctx.lib.pods_syev_status(ctx.h), "pods_syev_status")
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    ref = torch.flip(torch.linalg.eigvalsh(C), (0,))
    err = float((lam - ref).abs().max() / ref.abs().max())
    ts.sort()
    print("%s pods_syev median %.3f ms (min %.3f)  max|dlam|/lam0 %.2e  sum %.17g" % (
        " ".join("%s=%s" % (k, v) for k, v in os.environ.items() if k.startswith("PODS_")) or "default",
        ts[len(ts) // 2], ts[0], err, float(lam.sum())), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10)

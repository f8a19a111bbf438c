"""Per-unit times of pods_eigvals_* (HIP events around every unit) at the given n, against the
SpectrumQueue's cost model: python tools/eigvals_units_probe.py 4096 8192 16384"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pods-digital-filter_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import podsgen  # noqa: E402
from podsgen import engine as E  # noqa: E402


def main(sizes):
    ctx = E.Context(0)
    lib = ctx.lib
    out = {}
    for n in sizes:
        g = torch.Generator(device="cuda").manual_seed(n)
        B = torch.randn(n + n // 2, n, device="cuda", dtype=torch.float64, generator=g)
        C = (B.T @ B / B.shape[0]).contiguous()
        del B
        for rep in range(2):   # the second pass is the steady state
            ev = [torch.cuda.Event(enable_timing=True)]
            ev[0].record()
            podsgen.check(lib.pods_eigvals_begin(ctx.h, 0, E.ptr(C), n), "begin")
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            ev.append(e)
            rem = ctypes.c_int(1)
            while rem.value:
                podsgen.check(lib.pods_eigvals_advance(ctx.h, 0, 1, ctypes.byref(rem)), "advance")
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                ev.append(e)
            torch.cuda.synchronize()
            podsgen.check(lib.pods_eigvals_status(ctx.h, 0), "status")
        ms = [round(a.elapsed_time(b), 3) for a, b in zip(ev[:-1], ev[1:])]
        model = E.SpectrumQueue.UNIT_MS if n == 4096 else E.SpectrumQueue.two_stage_costs(n)
        out[n] = dict(units_ms=ms, total_ms=round(sum(ms), 2), model_ms=[round(x, 2) for x in model])
        print(json.dumps({"n": n, **out[n]}), flush=True)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [8192])

"""A/B of libpodsgen variants (tools/trd_variants.sh) on the fused eigensolve at n = 4096:
median pods_syev time over reps and the bits of its eigenvalues / vectors, one process per
variant (the library is loaded once per process):
    python tools/trd_ab.py [reps] default base k1 ..."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")


def child(reps):
    sys.path.insert(0, os.path.join(ROOT, "pods-digital-filter_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch
    import podsgen
    from podsgen import engine as E
    ctx = E.Context(0)
    n, nvec = 4096, 20
    g = torch.Generator(device="cpu").manual_seed(5)
    m = n + n // 2
    B = torch.randn(m, n, generator=g, dtype=torch.float64)
    k = torch.exp(-0.5 * (torch.arange(-12, 13, dtype=torch.float64) / 4.0) ** 2)
    Bs = torch.nn.functional.conv1d(B.unsqueeze(1), k.view(1, 1, -1), padding=12).squeeze(1) + 0.05 * B
    Bd = Bs.cuda()
    C = (Bd.T @ Bd / m)
    C = (0.5 * (C + C.T)).contiguous()
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    Y = torch.empty((n, nvec), dtype=torch.float64, device="cuda")
    ts = []
    for r in range(reps + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        podsgen.check(ctx.lib.pods_syev(ctx.h, E.ptr(C), n, nvec, E.ptr(lam), E.ptr(Y)), "pods_syev")
        b.record()
        torch.cuda.synchronize()
        podsgen.check(ctx.lib.pods_syev_status(ctx.h), "status")
        if r >= 2:
            ts.append(a.elapsed_time(b))
    out = os.environ["TRD_AB_OUT"]
    np.save(out + "_lam.npy", lam.cpu().numpy())
    np.save(out + "_Y.npy", Y.cpu().numpy())
    print(json.dumps({"lib": os.environ.get("PODSGEN_LIB", "default"), "syev_ms_median": float(np.median(ts)),
                      "syev_ms_min": float(np.min(ts))}), flush=True)


def main(reps, names):
    import numpy as np
    res = {}
    for nm in names:
        env = dict(os.environ)
        if nm != "default":
            env["PODSGEN_LIB"] = os.path.join(ROOT, "pods-digital-filter_amd", "podsgen", "variants",
                                              "libpodsgen_%s.so" % nm)
        env["TRD_AB_OUT"] = os.path.join("/tmp", "trd_ab_" + nm)
        r = subprocess.run([sys.executable, __file__, "--child", str(reps)], env=env, capture_output=True, text=True,
                           timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not line:
            print(nm, "FAILED", r.stderr[-2000:], flush=True)
            sys.exit(1)
        res[nm] = json.loads(line[-1])
        print(nm, line[-1], flush=True)
    ref = names[0]
    la = np.load("/tmp/trd_ab_%s_lam.npy" % ref)
    Ya = np.load("/tmp/trd_ab_%s_Y.npy" % ref)
    for nm in names[1:]:
        lb = np.load("/tmp/trd_ab_%s_lam.npy" % nm)
        Yb = np.load("/tmp/trd_ab_%s_Y.npy" % nm)
        print(nm, "eigenvalues bit-equal to", ref, bool(np.array_equal(la, lb)), "vectors bit-equal",
              bool(np.array_equal(Ya, Yb)), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]))
    else:
        main(int(sys.argv[1]), sys.argv[2:])

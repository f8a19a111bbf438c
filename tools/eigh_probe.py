import time, torch, sys
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
torch.manual_seed(0)
A = torch.randn(n, 3 * n // 2, dtype=torch.float64, device="cuda")
C = A @ A.T / n
torch.cuda.synchronize()
def bench(name, fn, reps=3):
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.time(); fn(); torch.cuda.synchronize(); ts.append(time.time() - t)
    print("%-28s n=%d  %.1f ms (min of %d)" % (name, n, 1e3 * min(ts), reps), flush=True)
print("default lib:", torch.backends.cuda.preferred_linalg_library(), flush=True)
bench("eigh default", lambda: torch.linalg.eigh(C))
bench("eigvalsh default", lambda: torch.linalg.eigvalsh(C))
for lib in ("magma", "cusolver"):
    try:
        torch.backends.cuda.preferred_linalg_library(lib)
        bench("eigh " + lib, lambda: torch.linalg.eigh(C))
        bench("eigvalsh " + lib, lambda: torch.linalg.eigvalsh(C))
    except Exception as e:
        print(lib, "failed", e)
t = time.time(); import numpy as np; Cn = C.cpu().numpy(); w = np.linalg.eigvalsh(Cn); print("numpy eigvalsh %.1f ms" % (1e3*(time.time()-t)))

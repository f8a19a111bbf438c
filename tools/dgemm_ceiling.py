"""fp64 GEMM ceiling on this GPU (rocBLAS/hipBLASLt via torch.mm): the SYRK's shape as a full
GEMM (4096 x 196608 x 4096) and a square 8192^3.  python tools/dgemm_ceiling.py"""
import time

import torch

for (m, k, n) in [(4096, 196608, 4096), (8192, 8192, 8192)]:
    a = torch.randn(m, k, dtype=torch.float64, device="cuda")
    b = torch.randn(k, n, dtype=torch.float64, device="cuda")
    torch.mm(a, b)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.time()
        torch.mm(a, b)
        torch.cuda.synchronize()
        best = min(best, time.time() - t)
    print("dgemm %dx%dx%d: %.2f ms  %.1f TFLOP/s" % (m, k, n, best * 1e3, 2.0 * m * k * n / best / 1e12), flush=True)
    del a, b
    torch.cuda.empty_cache()

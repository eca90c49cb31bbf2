"""Standalone share-GEMM microbenchmark through the C-ABI (one stream, no
co-located parties): per-kernel times from the library's HIP-event probe."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
sizes = [tuple(map(int, s.split("x"))) for s in (sys.argv[1:] or ["1024x1024x1024", "2048x2048x2048", "4096x4096x4096"])]
for (M, K, N) in sizes:
    A = torch.randint(-2**62, 2**62, (2 * M * K,), dtype=torch.int64, device="cuda")
    B = torch.randint(-2**62, 2**62, (2 * K * N,), dtype=torch.int64, device="cuda")
    wsb = L.dll.aby3g_mul_workspace_bytes(1, M, K, N)
    ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device="cuda")
    C0 = torch.empty(M * N, dtype=torch.int64, device="cuda")
    for _ in range(5):
        L.mul_local(1, P(A), P(B), P(C0), M, K, N, None, P(ws), wsb, None)
    torch.cuda.synchronize()
    # exact check of 64 sampled outputs: C0 = A0 (B0 + B1) + A1 B0 mod 2^64
    import numpy as np
    a = A.cpu().numpy().view(np.uint64).reshape(2, M, K)
    b = B.cpu().numpy().view(np.uint64).reshape(2, K, N)
    c = C0.cpu().numpy().view(np.uint64).reshape(M, N)
    rs = np.random.default_rng(1)
    bad = 0
    with np.errstate(over="ignore"):
        for _ in range(64):
            m, n = int(rs.integers(M)), int(rs.integers(N))
            exp = (a[0, m] * (b[0, :, n] + b[1, :, n]) + a[1, m] * b[0, :, n]).sum(dtype=np.uint64)
            bad += int(exp != c[m, n])
    print(f"{M}x{K}x{N}: sampled check {'ok' if bad == 0 else f'FAILED ({bad}/64)'}", flush=True)
    L.probe_enable(1)
    L.probe_reset()
    it = 20
    t = time.time()
    for _ in range(it):
        L.mul_local(1, P(A), P(B), P(C0), M, K, N, None, P(ws), wsb, None)
    torch.cuda.synchronize()
    dt = (time.time() - t) / it
    res = {}
    for f, name in [(0, "gemm"), (1, "epi"), (5, "digits")]:
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        L.dll.aby3g_probe_read(f, ctypes.byref(ms), ctypes.byref(cnt))
        res[name] = round(ms.value / it * 1e3, 1)
    L.probe_enable(0)
    tops = 144 * M * K * N / (res["gemm"] * 1e-6) / 1e12
    print(f"{M}x{K}x{N}: wall {dt * 1e6:.1f} us/call, kernel us {res}, gemm {tops:.0f} int8 TOP/s "
          f"({100 * tops / 5033:.1f} % of 5033)", flush=True)

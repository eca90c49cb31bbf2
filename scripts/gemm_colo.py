"""The share GEMM alone at C2's shape with the co-located plan (128
workgroups, aby3g_set_gemm_sharing(3)): average launch time from HIP events
over 50 launches (kernel-variant experiments; no result check)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
L.dll.aby3g_set_gemm_sharing(3)
P = lambda t: ctypes.c_void_p(t.data_ptr())
M = K = N = 1024
A = torch.randint(-2**62, 2**62, (2 * M * K,), dtype=torch.int64, device="cuda")
B = torch.randint(-2**62, 2**62, (2 * K * N,), dtype=torch.int64, device="cuda")
wsb = L.dll.aby3g_mul_workspace_bytes(1, M, K, N)
ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device="cuda")
C0 = torch.empty(M * N, dtype=torch.int64, device="cuda")
for _ in range(10):
    L.mul_local(1, P(A), P(B), P(C0), M, K, N, None, P(ws), wsb, None)
torch.cuda.synchronize()
L.probe_enable(1)
L.probe_reset()
for _ in range(50):
    L.mul_local(1, P(A), P(B), P(C0), M, K, N, None, P(ws), wsb, None)
torch.cuda.synchronize()
ms, cnt = ctypes.c_double(), ctypes.c_uint64()
L.dll.aby3g_probe_read(0, ctypes.byref(ms), ctypes.byref(cnt))
print(f"[{os.path.basename(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}] share GEMM 1024^3, 128 "
      f"workgroups: {ms.value / max(cnt.value, 1) * 1e3:.1f} us per launch ({cnt.value} launches)", flush=True)

"""Standalone timings of the non-GEMM kernels of one party's asyncMul +
truncation at 1024x1024 (one stream, nothing beside them): the truncation
pair (AES-CTR of both streams), the round-2 finalize, the digit split and the
split-K slab pass, with their algorithmic byte / block rates."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
M = K = N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = M * N
it = 50


def timed(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3  # us


ts = nt.TruncStreams()
ctypes.memmove(ts.next_seed, bytes(range(16)), 16)
ctypes.memmove(ts.prev_seed, bytes(range(16, 32)), 16)
ts.next_off, ts.prev_off = 8 * 12345, 8 * 777
R = torch.empty(n, dtype=torch.int64, device="cuda")
C = torch.empty(2 * n, dtype=torch.int64, device="cuda")
us = timed(lambda: L.trunc_tuple(ctypes.byref(ts), n, 16, P(R), P(C), None))
print(f"trunc_tuple n={n}: {us:.1f} us, {n / us * 1e-3:.1f} G AES blocks/s, {24 * n / us * 1e-3:.0f} GB/s written",
      flush=True)

z = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda") for _ in range(3)]
us = timed(lambda: L.trunc_finalize(0, P(z[0]), P(z[1]), P(z[2]), 16, P(C), n, None))
print(f"trunc_finalize n={n}: {us:.1f} us, {32 * n / us * 1e-3:.0f} GB/s", flush=True)

A = torch.randint(-2**62, 2**62, (2 * M * K,), dtype=torch.int64, device="cuda")
B = torch.randint(-2**62, 2**62, (2 * K * N,), dtype=torch.int64, device="cuda")
wsb = L.dll.aby3g_mul_workspace_bytes(1, M, K, N)
ws = torch.empty(wsb // 8 + 1, dtype=torch.int64, device="cuda")
out = torch.empty(n, dtype=torch.int64, device="cuda")
fn = lambda: L.mul_sub_local(1, P(A), P(B), P(R), None, P(out), M, K, N, P(ws), wsb, None)
wall = timed(fn)
L.probe_enable(1)
L.probe_reset()
for _ in range(it):
    fn()
torch.cuda.synchronize()
res = {}
for f, name in [(0, "gemm"), (1, "epi"), (5, "digits")]:
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    L.dll.aby3g_probe_read(f, ctypes.byref(ms), ctypes.byref(cnt))
    res[name] = ms.value / it * 1e3
L.probe_enable(0)
dig_bytes = 8 * (2 * M * K + 2 * K * N) + 16 * (M * K + K * N)
print(f"mul_sub_local {M}^3: {wall:.1f} us/call; digits {res['digits']:.1f} us ({dig_bytes / res['digits'] * 1e-3:.0f} "
      f"GB/s), gemm {res['gemm']:.1f} us, slab pass {res['epi']:.1f} us", flush=True)

key = (ctypes.c_uint8 * 16)(*range(16))
for nb in (4096, 65536, n // 4, n, 8 * n):
    o = torch.empty(2 * nb, dtype=torch.int64, device="cuda")
    us = timed(lambda: L.aes_ctr(key, 0, nb, P(o), None))
    print(f"aes_ctr {nb} blocks: {us:.1f} us, {nb / us * 1e-3:.1f} G blocks/s", flush=True)

kp = (ctypes.c_uint8 * 16)(*range(16))
kn = (ctypes.c_uint8 * 16)(*range(1, 17))
for nd in (2 * 491520 * 2, 8 * n):
    o = torch.empty(nd, dtype=torch.int64, device="cuda")
    us = timed(lambda: L.share_draws(nt.DRAW_BIN, kp, kn, 3, nd, None, P(o), None, None))
    print(f"share_draws BIN {nd} draws: {us:.1f} us, {nd / us * 1e-3:.1f} G AES blocks/s (2 keys)", flush=True)

"""AES-CTR kernel throughput through the C-ABI (one stream): raw counter
blocks, zero-share draws and the truncation pair, in G blocks/s."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
key = nt.key16(bytes(range(16)))
key2 = nt.key16(bytes(range(16, 32)))
n = 1 << 24
out = torch.empty(2 * n, dtype=torch.int64, device="cuda")
o2 = torch.empty(n, dtype=torch.int64, device="cuda")


def timed(f, blocks, name, it=10):
    f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / it * 1e3
    print(f"{name}: {us:.1f} us, {blocks / us / 1e3:.1f} G AES blocks/s", flush=True)


timed(lambda: L.aes_ctr(key, 0, n, P(out), None), n, "aes_ctr 16M blocks")
timed(lambda: L.share_draws(0, key, key2, 0, n, None, P(o2), None, None), n, "share_draws ARITH 16M draws (2 keys)")
ts = nt.TruncStreams()
ts.next_seed[:] = bytes(16)
ts.prev_seed[:] = bytes(range(16))
ts.next_off = ts.prev_off = 0
m = 1 << 20
R = torch.empty(m, dtype=torch.int64, device="cuda")
RT = torch.empty(2 * m, dtype=torch.int64, device="cuda")
timed(lambda: L.trunc_tuple(ctypes.byref(ts), m, 16, P(R), P(RT), None), m, "trunc_tuple 1M elements (1M blocks)")

"""Standalone timings of the binary engine's bit-slicing passes at C3's size
(2^20 rows, one stream, nothing beside them): the two-input resharing
transpose (party 0's four sources), the plain two-share transposes and the
output transposes, with their algorithmic byte rates and output checksums."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
words = 32 * ((rows + 2047) // 2048)
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


def csum(t):
    return int(t.view(torch.int64).sum().item()) & 0xFFFFFFFF


g = torch.Generator(device="cuda").manual_seed(5)
x0 = torch.randint(-2**62, 2**62, (rows,), dtype=torch.int64, device="cuda", generator=g)
x2 = torch.randint(-2**62, 2**62, (rows,), dtype=torch.int64, device="cuda", generator=g)
mem = torch.zeros(2 * 128 * words, dtype=torch.int64, device="cuda")
v = torch.zeros(rows, dtype=torch.int64, device="cuda")
Src = nt.WireSrc * 4
s = Src()
for k in range(4):
    s[k].cols64, s[k].nbits = 1, 64
for k, (share, wire0) in enumerate([(0, 0), (1, 0), (0, 64), (1, 64)]):
    s[k].wire_rows = ctypes.cast(mem.data_ptr() + 8 * (share * 128 + wire0) * words, ctypes.POINTER(ctypes.c_uint64))
s[0].term[0] = ctypes.cast(x0.data_ptr(), ctypes.POINTER(ctypes.c_int64))
s[0].term[1] = ctypes.cast(x2.data_ptr(), ctypes.POINTER(ctypes.c_int64))
s[0].coef[0] = s[0].coef[1] = 1
s[0].constant = -12345
s[0].copy_out = ctypes.cast(v.data_ptr(), ctypes.POINTER(ctypes.c_int64))
us = timed(lambda: L.bits_to_wires_lin(s, 4, rows, words, None))
byts = 8 * rows * (2 + 1) + 4 * 64 * 8 * words
print(f"bits_to_wires_lin P0 (4 sources) {rows} rows: {us:.1f} us, {byts / us * 1e-3:.0f} GB/s, "
      f"csum {csum(mem)} {csum(v)}", flush=True)
us = timed(lambda: L.bits_to_wires_lin(s, 1, rows, words, None))
byts = 8 * rows * 3 + 64 * 8 * words
print(f"bits_to_wires_lin 1 source: {us:.1f} us, {byts / us * 1e-3:.0f} GB/s", flush=True)

xs = torch.cat([x0, x2])
mem.zero_()
us = timed(lambda: L.bits_to_wires2(P(xs), rows, 1, 64, P(mem), 128 * words, words, None))
byts = 2 * (8 * rows + 64 * 8 * words)
print(f"bits_to_wires2 64 bits x 2 shares: {us:.1f} us, {byts / us * 1e-3:.0f} GB/s, csum {csum(mem)}", flush=True)

wires = torch.arange(128, dtype=torch.int32, device="cuda")
for nb in (1, 64):
    out = torch.zeros(2 * rows * ((nb + 63) // 64), dtype=torch.int64, device="cuda")
    us = timed(lambda: L.wires_to_bits2(P(mem), 128 * words, P(wires), nb, words, P(out), rows, None))
    byts = 2 * (8 * rows * ((nb + 63) // 64) + nb * 8 * (rows // 64))
    print(f"wires_to_bits2 {nb} bits x 2 shares: {us:.1f} us, {byts / us * 1e-3:.0f} GB/s, csum {csum(out)}",
          flush=True)

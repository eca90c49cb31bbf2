"""Standalone timing of aby3g_bits_to_wires_lin in C3's shape (fetch_msb's
two-input resharing over 2^20 rows: per party four sources of 64 wire rows,
two of them linear combinations of two share columns, two zero) beside
aby3g_bits_to_wires_map_n over the same bytes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
N = 1 << 20
words = N // 64
it = 50


class WireSrc(ctypes.Structure):
    _fields_ = [("term", ctypes.c_void_p * 4), ("coef", ctypes.c_int64 * 4), ("constant", ctypes.c_int64),
                ("cols64", ctypes.c_uint64), ("nbits", ctypes.c_uint32), ("wire_rows", ctypes.c_void_p),
                ("copy_out", ctypes.c_void_p)]


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
    return e0.elapsed_time(e1) / it * 1e3


x = torch.randint(-2**62, 2**62, (4, N), dtype=torch.int64, device="cuda")
mem = torch.zeros(4 * 64 * words, dtype=torch.int64, device="cuda")
srcs = (WireSrc * 4)()
for k in range(4):
    s = srcs[k]
    if k < 2:
        s.term[0], s.term[1] = x[2 * k].data_ptr(), x[2 * k + 1].data_ptr()
        s.coef[0], s.coef[1] = 1, 1
    s.cols64, s.nbits = 1, 64
    s.wire_rows = mem.data_ptr() + k * 64 * words * 8
f = L.dll.aby3g_bits_to_wires_lin
f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
us = timed(lambda: f(ctypes.addressof(srcs), 4, N, words, None))
gb = (2 * 2 * N * 8 + 4 * N * 8) / 1e9  # two sources read two columns; four write 64 wire rows
print(f"bits_to_wires_lin, 4 sources (2 with 2 terms) over 2^20 rows: {us:.1f} us, {gb / us * 1e6:.0f} GB/s", flush=True)

"""Standalone timings of the mapped transposes of a merge round (C5 shapes:
2^20 keys, 2^19 compare-exchange pairs): both gathers of a round in one
launch (aby3g_bits_to_wires_map_n) and both scatters (aby3g_wires_to_bits_map_n),
for round 0 (contiguous halves) and a later round (stride-2 rows), beside the
unmapped register transposes of the same bytes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aby3_amd import native as nt  # noqa: E402

L = nt.lib()
L.set_device(0)
P = lambda t: ctypes.c_void_p(t.data_ptr())
N = 1 << 20
pairs = N // 2
words = pairs // 64
W = 128 + 64
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
    return e0.elapsed_time(e1) / it * 1e3


keys = torch.randint(-2**62, 2**62, (2 * N,), dtype=torch.int64, device="cuda")
mem = torch.zeros(2 * W * words, dtype=torch.int64, device="cuda")
out = torch.zeros(2 * N, dtype=torch.int64, device="cuda")
wires = torch.arange(128, 192, dtype=torch.int32, device="cuda")
wires2 = torch.arange(0, 64, dtype=torch.int32, device="cuda")


def rm(first, start, step, per, stride):
    m = nt.RowMap()
    m.first, m.start, m.step, m.per_rep, m.rep_stride, m.idx = first, start, step, per, stride, None
    return m


cases = {
    "round 0 (halves)": (rm(0, 0, 1, pairs, N), rm(0, pairs, 1, pairs, N)),
    "round j (stride 2, d=1)": (rm(0, 1, 2, pairs - 1, N), rm(0, 2, 2, pairs - 1, N)),
}
gb = 2 * 2 * pairs * 8 * 2 / 1e9  # two maps, two shares, 8 B in + 8 B out
for name, (mx, my) in cases.items():
    maps = (nt.RowMap * 2)(mx, my)
    wrows = (ctypes.POINTER(ctypes.c_uint64) * 2)(
        ctypes.cast(mem.data_ptr(), ctypes.POINTER(ctypes.c_uint64)),
        ctypes.cast(mem.data_ptr() + 64 * words * 8, ctypes.POINTER(ctypes.c_uint64)))
    rows = pairs if "halves" in name else pairs - 1
    us = timed(lambda: L.dll.aby3g_bits_to_wires_map_n(P(keys), N, 1, 64, ctypes.cast(maps, ctypes.c_void_p), ctypes.cast(wrows, ctypes.c_void_p), 2, rows, W * words, words, None))
    print(f"gather {name}: {us:.1f} us, {gb / us * 1e6:.0f} GB/s", flush=True)
    wl = (ctypes.POINTER(ctypes.c_uint32) * 2)(ctypes.cast(wires.data_ptr(), ctypes.POINTER(ctypes.c_uint32)),
                                               ctypes.cast(wires2.data_ptr(), ctypes.POINTER(ctypes.c_uint32)))
    us = timed(lambda: L.dll.aby3g_wires_to_bits_map_n(P(mem), W * words, ctypes.cast(wl, ctypes.c_void_p), 64, words, P(out), N, ctypes.cast(maps, ctypes.c_void_p), 2, rows,
                                                       None))
    print(f"scatter {name}: {us:.1f} us, {gb / us * 1e6:.0f} GB/s", flush=True)

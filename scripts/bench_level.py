"""Standalone timing of one binary-engine level launch (aby3g_bin_level, no
hand-offs) at C3's size: 2^20 rows, one batch of 64 AND + 64 XOR gates over
128 input wires, alone on the GPU. Prints the launch time, the algorithmic
byte rate and an output checksum (equal across kernel variants)."""
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
nand = int(sys.argv[2]) if len(sys.argv) > 2 else 64
words = 32 * ((rows + 2047) // 2048)
wires = 128 + 2 * nand
g = torch.Generator(device="cuda").manual_seed(7)
mem = torch.randint(-2**62, 2**62, (2 * wires * words,), dtype=torch.int64, device="cuda", generator=g)
z = torch.randint(-2**62, 2**62, (nand * words,), dtype=torch.int64, device="cuda", generator=g)
send = torch.zeros(nand * words, dtype=torch.int64, device="cuda")
gates = (nt.Gate * (2 * nand))()
for k in range(nand):
    a, b = (2 * k) % 128, (2 * k + 1) % 128
    gates[k].in0, gates[k].in1, gates[k].out, gates[k].type = a, b, 128 + k, 2  # AND
    gates[k].z_row, gates[k].send_row = k, k
    x = nand + k
    gates[x].in0, gates[x].in1, gates[x].out, gates[x].type = a, b, 128 + nand + k, 0  # XOR
dg = torch.frombuffer(bytearray(bytes(gates)), dtype=torch.uint8).cuda()
ends = torch.tensor([2 * nand], dtype=torch.int32, device="cuda")


def run():
    L.bin_level(P(dg), P(ends), 1, None, None, 0, P(mem), wires, words, P(z), P(send), None)


for _ in range(5):
    run()
torch.cuda.synchronize()
it = 50
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(it):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / it * 1e3
byts = 8 * words * (nand * 7 + nand * 6)
cs = int(mem.sum().item() + send.sum().item()) & 0xFFFFFFFF
print(f"level {rows} rows, {nand} AND + {nand} XOR: {us:.1f} us, {byts / us * 1e-3:.0f} GB/s, csum {cs} "
      f"[{os.environ.get('ABY3_LVL_WIDE', '0')}]", flush=True)

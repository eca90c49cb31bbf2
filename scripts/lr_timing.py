"""LR iteration timing under different process conditions (host-overhead study)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
if mode != "plain":
    import torch

    if mode == "cuda":
        torch.zeros(1, device="cuda")
from aby3_amd import native as nt  # noqa: E402

for rep in range(2):
    with nt.Session(nt.JOB_LR, [1000000, 128, 256, 16, 11], devices=(0, 0, 0), probe=False) as s:
        s.run(5)
        for steps in (20, 50):
            t = time.perf_counter()
            s.run(steps)
            dt = (time.perf_counter() - t) / steps
            print(f"{mode} rep{rep} {steps} steps: {dt * 1e3:.3f} ms/iter", flush=True)

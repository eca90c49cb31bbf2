"""Profiling driver: runs exactly `--steps` steps of one bench job (no
warmup, no check, no probes), so per-kernel counter totals divide cleanly by
the number of steps. Used under rocprofv3 (scripts/gpu_profile.sh)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--job", choices=["mul", "msb", "lr", "a2b", "bitinj", "sort"], required=True)
ap.add_argument("--steps", type=int, default=4)
a = ap.parse_args()
if a.job == "mul":
    s = nt.Session(nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], probe=False)
elif a.job == "msb":
    s = nt.Session(nt.JOB_MSB, [1 << 20], probe=False)
elif a.job == "a2b":
    s = nt.Session(nt.JOB_A2B, [1 << 20], probe=False)
elif a.job == "sort":
    s = nt.Session(nt.JOB_SORT, [1 << 20], probe=False)
elif a.job == "bitinj":
    s = nt.Session(nt.JOB_BITINJ, [1 << 16, 64], probe=False)
else:
    s = nt.Session(nt.JOB_LR, [100000, 128, 256, 16, 11], probe=False)
s.run(a.steps)
s.close()
print("done", a.job, a.steps)

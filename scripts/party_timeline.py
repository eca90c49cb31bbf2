"""Merges the three party processes' rocprofv3 kernel traces
(scripts/prof_parties.sh) into one timeline: per party its kernels in a
window of the steady state, and per kernel family the time per step."""
import collections
import csv
import glob
import json
import os
import re
import sys

O = sys.argv[1]
# the kernel launched once per step by every party (steps are counted by it)
STEP_KERNEL = sys.argv[2] if len(sys.argv) > 2 else "k_bin_level_in"
rows = []
for p in range(3):
    f = glob.glob(os.path.join(O, f"p{p}", "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no kernel trace for party {p}")
    for r in csv.DictReader(open(f[0])):
        m = re.search(r"\b(k_[A-Za-z0-9_]+|__amd_rocclr_[A-Za-z]+)", r["Kernel_Name"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), p, m.group(1) if m else r["Kernel_Name"][:30]))
rows.sort()
steps = [json.loads(open(os.path.join(O, f"p{p}.json")).read().strip().splitlines()[-1]) for p in range(3)]
ms = max(s["ms_per_step"] for s in steps)
print(f"ms per step (slowest party): {ms:.4f}")
# steady state: the last 40 % of the trace
t_lo = rows[int(len(rows) * 0.6)][0]
t_hi = rows[-1][1]
win = [r for r in rows if r[0] >= t_lo]
span = (t_hi - t_lo) / 1e3
fam = collections.defaultdict(float)
for s, e, p, k in win:
    fam[(p, k)] += (e - s) / 1e3
steps_p = collections.Counter(p for s, e, p, k in win if k == STEP_KERNEL)
print(f"window {span:.0f} us; kernel us per step by party (steps counted by {STEP_KERNEL}):")
for (p, k), us in sorted(fam.items(), key=lambda x: (x[0][0], -x[1])):
    print(f"  party {p} {k:32s} {us / max(1, steps_p[p]):8.1f}")
print("\ntimeline (first 2 steps of the window):")
t0 = win[0][0]
for s, e, p, k in win:
    if s - t0 > 2 * ms * 1e6:
        break  # ms per step * 1e6 = ns per step
    print(f"{(s - t0) / 1e3:9.1f} us {(e - s) / 1e3:8.1f} us  P{p}  {k}")

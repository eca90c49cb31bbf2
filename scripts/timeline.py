"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV: for a window
in the middle of the run, lists every dispatch (start offset, duration, queue)
and sums busy time, so the critical path and the gaps can be read off."""
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"\b(k_[A-Za-z0-9_]+|__amd_rocclr_[A-Za-z]+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30],
                 r.get("Queue_Id", r.get("Stream_Id", "?"))))
rows.sort()
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
n = int(sys.argv[3]) if len(sys.argv) > 3 else 60
i0 = int(len(rows) * lo)
win = rows[i0:i0 + n]
t0 = win[0][0]
busy_end = t0
busy = 0
for s, e, k, q in win:
    if e > busy_end:
        busy += e - max(s, busy_end)
        busy_end = e
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  q{q:>3s}  {k}")
span = win[-1][1] - t0
print(f"window span {span / 1e3:.1f} us, GPU busy (union) {busy / 1e3:.1f} us ({100 * busy / span:.0f} %)")

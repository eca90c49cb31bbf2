"""Launch-to-start delays from a rocprofv3 --hip-trace --kernel-trace run
(scripts/gpu_hostdev.sh): for each kernel of the middle of the run, the time
between the end of its launch call on the host and its start on the device.
Kernels that start right after their launch were waiting for the host."""
import csv
import glob
import os
import re
import statistics
import sys

d = sys.argv[1]
kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
at = glob.glob(os.path.join(d, "*hip_api_trace.csv"))[0]
api = {}
for r in csv.DictReader(open(at)):
    api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r["Thread_Id"])
ks = []
for r in csv.DictReader(open(kt)):
    m = re.search(r"(k_\w+|__amd\w+)", r["Kernel_Name"])
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(0) if m else r["Kernel_Name"][:30],
               r["Correlation_Id"]))
ks.sort()
lo, hi = ks[len(ks) // 4][0], ks[-len(ks) // 10][0]
by = {}
for s, e, n, c in ks:
    if not (lo <= s <= hi) or c not in api:
        continue
    a = api[c]
    by.setdefault(n, []).append((s - a[1]) / 1e3)
print(f"window {(hi - lo) / 1e3:.0f} us")
for n, v in sorted(by.items(), key=lambda x: -len(x[1])):
    v.sort()
    near = sum(1 for x in v if x < 5) / len(v)
    print(f"{n:30s} n={len(v):5d} launch->start median {statistics.median(v):8.1f} us, p10 {v[len(v) // 10]:8.1f}, "
          f"started within 5 us of the launch call: {near:.2f}")
# host API time per thread in the window
th = {}
for c, (s, e, f, t) in api.items():
    if lo <= s <= hi:
        th.setdefault(t, [0, 0])
        th[t][0] += e - s
        th[t][1] += 1
for t, (tot, n) in sorted(th.items(), key=lambda x: -x[1][0])[:6]:
    print(f"thread {t}: {n} HIP calls, {tot / 1e3:.0f} us inside them ({tot / (hi - lo):.2f} of the window)")

"""Steady-state HIP API calls per party per step from two rocprofv3
--hip-trace --stats runs of one job at different step counts
(scripts/gpu_apidiff.sh): (stats(n1) - stats(n0)) / (n1 - n0) / parties."""
import csv
import glob
import sys


def load(d):
    f = glob.glob(f"{d}/**/*hip_api_stats.csv", recursive=True)
    if not f:
        raise SystemExit(f"no hip_api_stats.csv under {d}")
    out = {}
    for r in csv.DictReader(open(f[0])):
        out[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    return out


d0, d1, n0, n1 = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
title = sys.argv[5] if len(sys.argv) > 5 else ""
parties = 3
a, b = load(d0), load(d1)
rows = []
for k in set(a) | set(b):
    c = (b.get(k, (0, 0))[0] - a.get(k, (0, 0))[0]) / (n1 - n0) / parties
    t = (b.get(k, (0, 0))[1] - a.get(k, (0, 0))[1]) / (n1 - n0) / parties / 1e3
    if abs(c) >= 0.01:
        rows.append((k, c, t))
rows.sort(key=lambda r: -r[1])
print(title)
print(f"= (rocprofv3 --hip-trace stats of a {n1}-step run - those of a {n0}-step run) / {n1 - n0} / {parties} parties")
print("(scripts/gpu_apidiff.sh; times are under the tracer)")
tc = tt = 0.0
for k, c, t in rows:
    print(f"{k:38s} {c:7.2f} calls {t:8.1f} us")
    tc += c
    tt += t
print(f"{'total':38s} {tc:7.2f} calls {tt:8.1f} us")

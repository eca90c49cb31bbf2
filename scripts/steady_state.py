"""Where do the driver's short C2 runs lose time? Runs the C2 session the way
bench.py does (2 steps, check, W warmup, K timed) for several (W, K) pairs and
a time-based warm-up, and prints ms per step of each timed region plus the
per-step times of a run of single steps after an idle gap."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

P = [1024, 1024, 1024, 16, 1]
out = {}
with nt.Session(nt.JOB_MUL_TRUNC, P, probe=False) as s:
    s.run(2)
    assert s.check()
    for w, k in ((5, 20), (20, 100), (5, 20), (50, 20), (5, 100), (0, 20)):
        time.sleep(0.2)  # idle gap like the reveal / setup before the driver's timing
        s.run(w)
        t = time.perf_counter()
        s.run(k)
        out[f"w{w}_k{k}"] = (time.perf_counter() - t) / k * 1e3
    # per-step after an idle gap: 30 single-step runs (each includes a host sync)
    time.sleep(0.2)
    single = []
    for _ in range(30):
        t = time.perf_counter()
        s.run(1)
        single.append(round((time.perf_counter() - t) * 1e3, 4))
    out["single_after_idle"] = single
    # time-based warm-up then 20 steps
    for secs in (0.05, 0.2, 0.5):
        time.sleep(0.2)
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < secs:
            s.run(5)
            n += 5
        t = time.perf_counter()
        s.run(20)
        out[f"warm{secs}s_k20"] = (time.perf_counter() - t) / 20 * 1e3
    # a run of k steps: total time = fill + k * steady; fit from k in 10..200
    time.sleep(0.2)
    s.run(200)
    fit = {}
    for k in (10, 20, 40, 80, 160):
        t = time.perf_counter()
        s.run(k)
        fit[k] = (time.perf_counter() - t) * 1e3
    out["run_ms_by_k_hot"] = fit
print(json.dumps(out))

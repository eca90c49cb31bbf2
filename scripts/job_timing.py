"""Times one session job (3 co-located parties on GPU 0): prints ms per step
after warmup and the job's own check. Used by the A/B scripts."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

job = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
jobs = {"mul": (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 10),
        "mul2": (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1, 2], 10), "msb": (nt.JOB_MSB, [1 << 20], 5),
        "msb17": (nt.JOB_MSB, [1 << 17], 5),
        "sort": (nt.JOB_SORT, [1 << 20], 1), "lr": (nt.JOB_LR, [1000000, 128, 256, 16, 11], 20),
        "a2b": (nt.JOB_A2B, [1 << 20], 5)}
j, params, warm = jobs[job]
with nt.Session(j, params, probe=False) as s:
    s.run(warm)
    t = time.perf_counter()
    s.run(steps)
    dt = (time.perf_counter() - t) / steps
    ok = s.check()
print(json.dumps(dict(job=job, ms=round(dt * 1e3, 4), ok=bool(ok), env=os.environ.get("AB_TAG", ""))))

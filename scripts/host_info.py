"""Host-side timing of a session job: ms per step next to the host's enqueue
time per step, the drain after the loop and the HIP API time, to tell a
host-bound step from a device-bound one."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

jobs = {"mul": (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1]), "msb": (nt.JOB_MSB, [1 << 20]),
        "lr": (nt.JOB_LR, [1000000, 128, 256, 16, 11])}
for name in sys.argv[1:] or ["msb", "mul"]:
    j, p = jobs[name]
    with nt.Session(j, p, probe=False) as s:
        s.run(20)
        t = time.perf_counter()
        s.run(200)
        dt = (time.perf_counter() - t) / 200
        info = s.info()
    print(json.dumps(dict(job=name, ms=round(dt * 1e3, 4), **{k: info[k] for k in info if k.startswith("host")})))

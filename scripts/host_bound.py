"""Is the host on a job's critical path? Runs a session job (3 co-located
parties on GPU 0) and prints ms per step beside the session's own host
figures: the host time per step spent issuing work (max over the parties),
the drain after the last step, the time in HIP calls and the waits for
peer messages. Issue time close to the step time with a short drain means
the device waits for the host."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

jobs = {"mul": (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 10, 100), "msb": (nt.JOB_MSB, [1 << 20], 5, 300),
        "sort": (nt.JOB_SORT, [1 << 20], 1, 3), "lr": (nt.JOB_LR, [1000000, 128, 256, 16, 11], 20, 1000)}
for name in (sys.argv[1:] or list(jobs)):
    j, params, warm, steps = jobs[name]
    with nt.Session(j, params, probe=False) as s:
        s.run(warm)
        t = time.perf_counter()
        s.run(steps)
        ms = (time.perf_counter() - t) / steps * 1e3
        i = s.info()
        print(json.dumps(dict(job=name, ms_per_step=round(ms, 4), host_enqueue_us=round(i["host_enqueue_us"], 1),
                              host_drain_us=round(i["host_drain_us"], 1), host_api_us=round(i["host_api_us"], 1),
                              host_api_calls=round(i["host_api_calls"], 1),
                              host_recv_wait_us=round(i["host_recv_wait_us"], 1))), flush=True)

"""Times the C5 job (odd_even_merge_sort of 2^20 keys, 3 co-located parties)
and prints per-sort time and host-side counters."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native as nt  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
with nt.Session(nt.JOB_SORT, [n], probe=False) as s:
    t = time.perf_counter()
    s.run(1)
    first = time.perf_counter() - t
    t = time.perf_counter()
    s.run(reps)
    dt = (time.perf_counter() - t) / reps
    ok = s.check()
    print(json.dumps(dict(keys=n, first_s=first, s_per_sort=dt, ok=ok, info=s.info())))

import sys, time, json
sys.path.insert(0, '.')
from aby3_amd import native as nt
for rows in (1 << 20, 1 << 19, 1 << 18, 1 << 16):
    with nt.Session(nt.JOB_MSB, [rows], probe=False) as s:
        s.run(20); t = time.perf_counter(); s.run(200); dt = (time.perf_counter() - t) / 200
        print(json.dumps(dict(job="msb", rows=rows, ms=round(dt * 1e3, 4))), flush=True)

import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from aby3_amd import native as nt
for job, params, name in [(nt.JOB_MSB, [1 << 20], "msb"), (nt.JOB_LR, [1000000, 128, 256, 16, 11], "lr"), (nt.JOB_MUL_TRUNC, [1024,1024,1024,16,1], "mul")]:
    with nt.Session(job, params, probe=False) as s:
        s.run(3)
        t = time.perf_counter(); s.run(20); dt = (time.perf_counter() - t) / 20
        info = s.info()
        print(name, f"{dt*1e3:.3f} ms/step", {k: (round(v, 1) if isinstance(v, float) else v) for k, v in info.items()}, flush=True)

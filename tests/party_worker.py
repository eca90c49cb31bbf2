"""One party of a three-process session (aby3h_party_create), started by
tests/test_gpu_parties.py and bench.py's party deployment checks: runs
`steps` steps of a job, checks the revealed result, prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aby3_amd import native  # noqa: E402


def main():
    job, party, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    link, device = sys.argv[4], int(sys.argv[5])
    params = [int(x) for x in sys.argv[6].split(",")] if len(sys.argv) > 6 and sys.argv[6] else []
    # layout (aby3h_party_create's colocated): 1 the three on one GPU with
    # in-kernel hand-offs, 2 on one GPU taking the cross-GPU branches
    layout = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    s = native.Session.party(job, params, party, link, device=device, colocated=layout)
    # a lagging party (tests): its host sleeps between steps, so the others run ahead
    lag = float(os.environ.get("ABY3_TEST_LAG_MS", "0")) / 1e3
    try:
        s.run(1)  # warm-up
        # bench: more untimed steps first (clock ramp after setup)
        warm = int(os.environ.get("ABY3_WARMUP_STEPS", "0"))
        if warm:
            s.run(warm)
        t0 = time.perf_counter()
        if lag:
            for _ in range(steps):
                s.run(1)
                time.sleep(lag)
        else:
            s.run(steps)
        dt = time.perf_counter() - t0
        digest = s.digest(party)  # this party's shares of the result, before check() reveals
        ok = s.check()
        info = s.info()
    finally:
        s.close()
    print(json.dumps({"party": party, "ok": ok, "ms_per_step": 1e3 * dt / steps,
                      "recv_wait_us": info["host_recv_wait_us"], "digest": digest,
                      "lr_fused": info["lr_fused"], "lr_sys_scope": info["lr_sys_scope"]}), flush=True)


if __name__ == "__main__":
    main()

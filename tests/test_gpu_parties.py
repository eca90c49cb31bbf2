"""The north_star deployment's transport: three processes, one ABY3 party
each (aby3h_party_create), joined by shared-memory links and IPC-exported
device staging slots (aby3_amd/host/Link.h, Channel.cpp). On the one-GPU box
the three processes share cuda:0, so the payload copies run over IPC
mappings of one device; between GPUs the same code path reads the peer's
slot over xGMI. Each job's revealed result is checked by party 0 against
plaintext exactly as the in-process sessions of test_gpu_protocols.py."""
import json
import os
import subprocess
import sys

import pytest

from aby3_amd import native as nt

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def run_parties(job, params, steps, tag, timeout=150, lag_ms=0, layout=1):
    link = f"gt{os.getpid()}.{tag}"
    env = dict(os.environ, ABY3_LINK_TIMEOUT_S="100")
    args = [str(job), None, str(steps), link, "0", ",".join(str(p) for p in params), str(layout)]
    procs = []
    for party in range(3):
        a = list(args)
        a[1] = str(party)
        penv = dict(env, ABY3_TEST_LAG_MS=str(lag_ms)) if party == 0 and lag_ms else env
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "party_worker.py"), *a],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=penv))
    res = []
    try:
        for p in procs:
            try:
                o, e = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                p.kill()
                o, e = p.communicate()
            res.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    # every party's exit and stderr tail on a failure: a party that waits out
    # its link timeout is usually the symptom, the cause is in a peer's log
    if any(rc != 0 for rc, _, _ in res):
        report = "\n".join(f"--- party {i} exited {rc}:\n{e[-2000:]}" for i, (rc, _, e) in enumerate(res))
        raise AssertionError("a party failed\n" + report)
    return [json.loads(o.strip().splitlines()[-1]) for _, o, _ in res]


def colocated_digests(job, params, steps):
    """The same job run by three parties in one process (the same seeds):
    each party's digest of its result shares."""
    with nt.Session(job, params, probe=False) as s:
        s.run(steps)
        return [s.digest(p) for p in range(3)]


@pytest.mark.parametrize("job,params,steps", [
    (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 3),   # C2 shapes
    (nt.JOB_MUL_TRUNC, [257, 200, 250, 8, 1], 2),       # ragged GEMM, D8
    (nt.JOB_MUL, [128, 128, 128, 0], 3),                # C1 Hadamard
    (nt.JOB_MSB, [1 << 16], 2),                         # C3 circuit levels
    (nt.JOB_LR, [20000, 128, 256, 16, 11], 5),          # C4 (dataset trimmed), fused across processes
    (nt.JOB_LR, [20000, 128, 256, 16, 11, 1], 90),      # C4 with getSubset in every step, across a reshuffle
    (nt.JOB_SORT, [4096], 1),                           # C5 network, every key checked
    (nt.JOB_A2B, [5000], 2),                            # toBinaryMatrix
    (nt.JOB_BITINJ, [777, 13], 2),                      # bitInjection (OT messages)
    (nt.JOB_MSB, [6244, 1, 2], 2),                      # a row slice: its masks in two strided pieces
    (nt.JOB_MUL_TRUNC, [257, 200, 250, 8, 1, 1, 1, 3], 2),  # a row slice of the GEMM
])
def test_three_party_processes(gpu, job, params, steps):
    """Every job by three processes: the revealed result checked against
    plaintext, and every party's result shares identical to the same job's
    in one process (share-exact across the two layouts)."""
    outs = run_parties(job, params, steps, f"{job}_{params[0]}_{len(params)}")
    assert sorted(o["party"] for o in outs) == [0, 1, 2]
    assert all(o["ok"] for o in outs), outs
    if job == nt.JOB_LR:
        # the fused iteration runs across the processes (IPC-mapped mailboxes)
        assert all(o["lr_fused"] == 1 for o in outs), outs
    ref = colocated_digests(job, params, steps + 1)  # the worker's warm-up step + steps
    got = [o["digest"] for o in sorted(outs, key=lambda o: o["party"])]
    assert got == ref


@pytest.mark.parametrize("job,params,steps", [
    (nt.JOB_LR, [20000, 128, 256, 16, 11], 5),          # C4: the fused iteration's system-scope mailboxes
    (nt.JOB_LR, [20000, 128, 256, 16, 11, 1], 40),      # C4 with getSubset in every step
    (nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 3),   # C2: every z message as a staged IPC copy
    (nt.JOB_MSB, [1 << 16], 2),                         # C3: every level's AND shares staged
    (nt.JOB_SORT, [4096], 1),                           # C5
])
def test_three_party_processes_remote_branches(gpu, job, params, steps):
    """The north-star layout's cross-GPU branches, run on the one GPU
    (aby3h_party_create colocated = 2): no IPC arenas, every device message a
    staged copy read out of the sender's exported slot, and the fused LR
    iteration with uncached mailboxes and system-scope stores and loads
    (aby3ML.cpp FusedLr::make, lr.hip sys_scope). Share-exact against the
    same job in one process."""
    outs = run_parties(job, params, steps, f"remote{job}_{params[0]}_{len(params)}", layout=2)
    assert sorted(o["party"] for o in outs) == [0, 1, 2]
    assert all(o["ok"] for o in outs), outs
    if job == nt.JOB_LR:
        assert all(o["lr_fused"] == 1 and o["lr_sys_scope"] == 1 for o in outs), outs
    ref = colocated_digests(job, params, steps + 1)
    got = [o["digest"] for o in sorted(outs, key=lambda o: o["party"])]
    assert got == ref


def test_lagging_party_many_steps(gpu):
    """Party 0's host sleeps 5 ms between 60 steps of the C2 multiplication:
    party 2 only sends (Sh3Evaluator.cpp:152-153) and runs ahead until its
    staging slots are all in flight, then waits for them (Channel.cpp, the
    sender's throttle) instead of failing or growing without bound."""
    outs = run_parties(nt.JOB_MUL_TRUNC, [1024, 1024, 1024, 16, 1], 60, "lag", timeout=200, lag_ms=5)
    assert sorted(o["party"] for o in outs) == [0, 1, 2]
    assert all(o["ok"] for o in outs), outs


@pytest.mark.parametrize("params", [[1024, 1024, 1024, 16, 1], [257, 200, 250, 8, 1]])
def test_products_in_flight_share_exact(gpu, params):
    """MulJob with two products in flight per party (the next product issued
    before the previous one's reshare round completes, each into its own
    output): every party's shares of the last product are those of the
    one-at-a-time run, and the revealed result matches plaintext."""
    ref = colocated_digests(nt.JOB_MUL_TRUNC, params, 5)
    with nt.Session(nt.JOB_MUL_TRUNC, params + [2], probe=False) as s:
        s.run(5)
        got = [s.digest(p) for p in range(3)]
        assert s.check()
    assert got == ref
    outs = run_parties(nt.JOB_MUL_TRUNC, params + [2], 4, f"inflight_{params[0]}")
    assert all(o["ok"] for o in outs), outs
    assert [o["digest"] for o in sorted(outs, key=lambda o: o["party"])] == ref

"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks, each an
independent replica (weak scaling). Checks the control plane the bench
relies on -- rendezvous on 127.0.0.1, barrier, max over ranks of the timed
region -- and that no data-path collective is needed (each rank's result is
computed from its own inputs only)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import bench

    w, r, local, pg = bench.dist_setup()
    assert (w, r, local) == (world, rank, rank)
    bench.barrier(pg)
    # the timed region's max over ranks: rank r "took" 1 + r seconds
    dt = bench.allmax(pg, 1.0 + rank)
    q.put((rank, dt))
    pg.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_control_plane():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=5) for _ in range(world))
    assert got == [(0, 2.0), (1, 2.0)]


def test_single_rank_has_no_process_group(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    import bench

    world, rank, local, pg = bench.dist_setup()
    assert (world, rank, local, pg) == (1, 0, 0, None)
    assert bench.allmax(pg, 3.5) == 3.5


def _party_rank(rank, world, port, exe, q):
    """One gloo rank = one ABY3 party: ranks agree on the session name over
    the process group, then each runs its party of every job in its own
    process (the null-device driver of tests/cpp/nulldev/party_procs.cpp)."""
    import subprocess

    import torch
    import torch.distributed as dist

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo")
    tag = torch.tensor([os.getpid() if rank == 0 else 0], dtype=torch.int64)
    dist.broadcast(tag, 0)
    name = f"g{int(tag.item())}"
    # (1 MiB hand-off arenas: the null device's shared memory is a 1 GiB bump allocator)
    env = dict(os.environ, ND_ARENA=f"/aby3nd.{name}", ABY3_LINK_TIMEOUT_S="60", ABY3_ARENA_MB="1")
    dist.barrier()
    r = subprocess.run([exe, str(rank), name], capture_output=True, text=True, timeout=300, env=env)
    dist.barrier()
    if rank == 0:
        try:
            os.unlink(f"/dev/shm/aby3nd.{name}")
        except OSError:
            pass
    q.put((rank, r.returncode, r.stdout[-2000:] + r.stderr[-2000:]))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_three_ranks_are_three_parties(tmp_path):
    """The north_star split on CPU: world size 3, rank i runs party i of each
    session job (not a replica), over the shared-memory links."""
    import glob
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    nd = os.path.join(root, "tests", "cpp", "nulldev")
    src = str(tmp_path / "nulldev.cpp")
    subprocess.run([sys.executable, os.path.join(nd, "gen_nulldev.py"), src], check=True)
    exe = str(tmp_path / "party_rank")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I" + os.path.join(root, "include"),
                    "-I" + os.path.join(root, "aby3_amd", "host"),
                    *sorted(glob.glob(os.path.join(root, "aby3_amd", "host", "*.cpp"))), src,
                    os.path.join(nd, "party_procs.cpp"), "-o", exe, "-pthread", "-lrt"], check=True, timeout=600)
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_party_rank, args=(r, world, port, exe, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=500) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, rc, log in res:
        assert rc == 0, f"party {rank}: {log}"

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

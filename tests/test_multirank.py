"""Multi-rank path of bench.py on CPU (gloo, world_size 2): the barrier-bracketed timing
takes the MAX over ranks, so the whole-job value = units of all ranks / slowest rank's time
(weak scaling, no data-path collective: every rank processes its own cells / codeblocks)."""
import os
import sys
import time
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    args = types.SimpleNamespace(warmup=1, steps=3)
    delay = 0.02 * (rank + 1)  # rank 1 is the slow one

    def step():
        time.sleep(delay)

    elapsed, step_ms = bench.timed(args, dist, world, torch.device("cpu"), None, step)
    q.put((rank, elapsed, step_ms))
    dist.destroy_process_group()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(120)
def test_timed_takes_max_over_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    (_, e0, s0), (_, e1, s1) = out
    # every rank reports the slowest rank's time: 3 steps x 40 ms on rank 1
    assert e0 == e1
    assert e0 >= 3 * 0.04
    # the barrier after the timed steps makes the fast rank wait for the slow one
    assert s0 >= 40.0 and s1 >= 40.0

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


def _fanout_worker(rank, world, port, q, nof_cells):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from srsran_project_amd.cell_fanout import SlotFanout, cell_range

    fan = SlotFanout(dist, world, rank, nof_cells)
    first, count = cell_range(nof_cells, world, rank)
    # rank 0 holds every cell's slot input (cell c: values c * 1000 + k)
    full_in = (torch.arange(nof_cells).view(-1, 1) * 1000 + torch.arange(6).view(1, -1)).to(torch.int32) \
        if rank == 0 else None
    mine = torch.empty((count, 6), dtype=torch.int32)
    fan.scatter(full_in, mine)
    # the rank's "processing": results tagged with the rank that produced them
    results = mine * 2 + rank
    full_out = torch.zeros((nof_cells, 6), dtype=torch.int32) if rank == 0 else None
    fan.gather(results, full_out)
    q.put((rank, first, count, mine.numpy().copy(), None if full_out is None else full_out.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("nof_cells", [8, 7, 3])
def test_cell_fanout_scatter_gather(nof_cells):
    """The multi-GPU slot ingest on CPU tensors (gloo, world 2): every cell goes to exactly one rank, each rank
    gets its contiguous share, and rank 0 gathers every cell's result from the rank that owns it."""
    import numpy as np

    from srsran_project_amd.cell_fanout import cell_range

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanout_worker, args=(r, world, port, q, nof_cells)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=90) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    owned = []
    for rank, first, count, mine, _ in out:
        assert (first, count) == cell_range(nof_cells, world, rank)
        cells = np.arange(first, first + count)
        owned.extend(cells.tolist())
        assert np.array_equal(mine, cells[:, None] * 1000 + np.arange(6)[None, :])
    assert sorted(owned) == list(range(nof_cells))  # every cell on exactly one rank
    full = out[0][4]
    for c in range(nof_cells):
        r = next(rk for rk in range(world) if c in range(*((lambda a, n: (a, a + n))(*cell_range(nof_cells, world,
                                                                                               rk)))))
        assert np.array_equal(full[c], (c * 1000 + np.arange(6)) * 2 + r)


def test_cell_range_balanced():
    from srsran_project_amd.cell_fanout import cell_range

    for n in range(0, 20):
        for w in (1, 2, 3, 8):
            shares = [cell_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in shares) == n
            assert max(c for _, c in shares) - min(c for _, c in shares) <= 1
            pos = 0
            for a, c in shares:
                assert a == pos
                pos += c


@pytest.mark.timeout(180)
def test_bench_spawns_ranks(tmp_path):
    """`bench.py --gpus 2` starts two ranks itself (before any GPU call) and reports n_gpus = 2: exercised on CPU
    through a tiny entry that reuses bench.spawn_ranks with gloo ranks."""
    import json
    import subprocess

    script = tmp_path / "entry.py"
    script.write_text(
        "import os, sys, json\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "if 'WORLD_SIZE' not in os.environ:\n"
        "    sys.argv = [sys.argv[0], '--gpus', '2']\n"
        "    bench.__file__ = __file__\n"
        "    sys.exit(bench.spawn_ranks(2))\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "r, w = dist.get_rank(), dist.get_world_size()\n"
        "if r == 0: print(json.dumps({'n_gpus': w, 'local_rank': os.environ['LOCAL_RANK']}))\n"
        "dist.destroy_process_group()\n" % ROOT)
    out = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=150)
    assert out.returncode == 0, out.stderr
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2

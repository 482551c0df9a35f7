"""Do the PDSCH and PUSCH chains of a step overlap?  Wall time per step (10 steps after warm-up) of the PDSCH chain
alone, the PUSCH chain alone, and both (fork / join on two streams) with the PUSCH stream taken from the torch pool
(several pool slots), as a high-priority stream, and as a fresh stream created after the library objects.
  PYTHONPATH=. python tools/overlap_probe.py [pipeline|slot]"""
import sys
import time

import torch

import bench_pipeline as bp
from bench_slot import SlotPipeline

dev = torch.device("cuda", 0)
kind = sys.argv[1] if len(sys.argv) > 1 else "slot"
pl = SlotPipeline(64, 8, dev, seed=0, iters=6, snr_db=30.0) if kind == "slot" else bp.Pipeline(64, dev)
main = torch.cuda.current_stream(dev)


def wall(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) * 1e3 / n


def both(us):
    fork, join = torch.cuda.Event(), torch.cuda.Event()

    def step():
        fork.record(main)
        us.wait_event(fork)
        with torch.cuda.stream(main):
            pl.pdsch(main)
        with torch.cuda.stream(us):
            pl.pusch(us)
        join.record(us)
        main.wait_event(join)
    return step


def alone(chain, s):
    def step():
        with torch.cuda.stream(s):
            chain(s)
    return step


print("%s: pdsch alone %.3f ms, pusch alone %.3f ms" % (kind, wall(alone(pl.pdsch, main)), wall(alone(pl.pusch, main))))
for i in range(5):
    s = torch.cuda.Stream(dev)
    print("  both, pool stream %d: %.3f ms" % (i, wall(both(s))))
print("  both, high-priority stream: %.3f ms" % wall(both(torch.cuda.Stream(dev, priority=-1))))
print("  both, pusch on the main stream too: %.3f ms" % wall(both(main)))

"""Host and device time of the PUSCH slot call of a mixed slot_pipeline step (bench.py --workload slot_pipeline
--mixed), and of the same slot restricted to each PDU kind, to see where a mixed slot's time goes.
  PYTHONPATH=. python tools/mixed_slot_probe.py [cells]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import srsran_project_amd as amd
from bench_slot import SlotPipeline

dev = torch.device("cuda", 0)
cells = int(sys.argv[1]) if len(sys.argv) > 1 else 64
only = sys.argv[2] if len(sys.argv) > 2 else None  # time only this kind (for a profiler run)
pl = SlotPipeline(cells, 8, dev, seed=0, iters=6, snr_db=35.0, mixed=True)
stream = torch.cuda.current_stream(dev)
pl.pusch(stream)
torch.cuda.synchronize(dev)


def timed(label, slot, reps=5):
    tbs = torch.zeros(max(slot.tb_total, 1), dtype=torch.uint8, device=dev)
    res = torch.zeros((slot.n, amd.pusch_processor.RESULT_BYTES), dtype=torch.uint8, device=dev)
    uci = torch.zeros(max(slot.uci_total, 1), dtype=torch.uint8, device=dev)
    pl.proc.process_slot(pl.grid_ul, slot, tbs=tbs, results=res, stream=stream, uci=uci)
    torch.cuda.synchronize(dev)
    host, wall = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        pl.proc.process_slot(pl.grid_ul, slot, tbs=tbs, results=res, stream=stream, uci=uci)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    print("%-8s %4d PDUs  host %.3f ms  wall %.3f ms" % (label, slot.n, min(host), min(wall)), flush=True)


soft = {i: pl.ul_slot.soft[i] for i in range(len(pl.ul))}
full = [(pp, c, soft[i]) if soft[i] is not None else (pp, c) for i, (pp, c) in enumerate(pl.ul)]
if only in (None, "all"):
    timed("all", amd.PuschSlot(full))
for kind in ("data", "uci", "harq", "tp") if only is None else (() if only == "all" else (only,)):
    sub = [x for x, k in zip(full, pl.kinds) if k == kind]
    if sub:
        timed(kind, amd.PuschSlot(sub))

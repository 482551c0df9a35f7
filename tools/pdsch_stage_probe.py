"""The 64-cell PDSCH encode stage alone: HIP-event time of encode_batch on one warm stream (20 calls), with and without
the TB-CRC overlap (SRSRAN_AMD_PDSCH_OVERLAP read per call).  Run under rocprofv3 --kernel-trace --stats for the
kernels' own durations.  PYTHONPATH=. python tools/pdsch_stage_probe.py"""
import os

import torch

import bench_pipeline as bp

dev = torch.device("cuda", 0)
pl = bp.Pipeline(64, dev)
s = torch.cuda.Stream(dev)
for ov in ("0", "1"):
    os.environ["SRSRAN_AMD_PDSCH_OVERLAP"] = ov
    for _ in range(3):
        pl.enc.encode_batch(pl.tb_dl, pl.plan_dl, out=pl.cw_dl, stream=s)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        pl.enc.encode_batch(pl.tb_dl, pl.plan_dl, out=pl.cw_dl, stream=s)
    e1.record(s)
    torch.cuda.synchronize(dev)
    print("overlap %s: %.4f ms per encode_batch (64 TBs, 8256 codeblocks)" % (ov, e0.elapsed_time(e1) / 20))

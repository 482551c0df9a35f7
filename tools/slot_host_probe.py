"""Host time of each C-ABI call of one slot_pipeline step (perf_counter around the call: descriptor building,
uploads and any host wait inside it) next to the step's wall time, with the packed decoder and the fused PDSCH
encoder switched on and off in-process (both read their environment switch per call).
  PYTHONPATH=. python tools/slot_host_probe.py [cells]"""
import os
import sys
import time

import torch

import bench_pipeline as bp
from bench_slot import SlotPipeline

dev = torch.device("cuda", 0)
cells = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pl = SlotPipeline(cells, 8, dev, seed=0, iters=6, snr_db=30.0)
stream = torch.cuda.current_stream(dev)
T = {}


def timed(name, fn):
    t0 = time.perf_counter()
    fn()
    T.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)


def step():
    t = torch
    if pl.ul_stream is None:
        pl.ul_stream = t.cuda.Stream(dev)
        pl.ev_fork, pl.ev_join = t.cuda.Event(), t.cuda.Event()
    pl.ev_fork.record(stream)
    pl.ul_stream.wait_event(pl.ev_fork)
    with t.cuda.stream(stream):
        timed("encode_slot", lambda: pl.enc.encode_slot(pl.tb_dl, pl.tx_desc, out=pl.cw_dl, stream=stream))
        timed("modulate_slot", lambda: pl.mod.modulate_slot(pl.grid_dl, pl.dl_slot, codewords=pl.cw_dl, stream=stream))
        timed("ofdm_modulate", lambda: pl.ofdm_mod.modulate_batch(
            pl.grid_dl.view(t.int16).view(pl.S, 4, 14, 2 * 12 * 273), bp.SLOT, out=pl.samp_dl, stream=stream))
    us = pl.ul_stream
    with t.cuda.stream(us):
        timed("ofdm_demodulate", lambda: pl.ofdm_dem.demodulate_batch(
            pl.samp_ul, bp.SLOT, grid=pl.grid_ul.view(t.int16).view(pl.S, 4, 14, 2 * 12 * 273), stream=us))
        timed("process_slot", lambda: pl.proc.process_slot(pl.grid_ul, pl.ul_slot, tbs=pl.tb_rx, results=pl.res_ul,
                                                           stream=us))
    pl.ev_join.record(us)
    stream.wait_event(pl.ev_join)


for cfg in [{}, {"SRSRAN_AMD_LDPC_PK": "0"}, {"SRSRAN_AMD_PDSCH_FUSED": "0"},
            {"SRSRAN_AMD_LDPC_PK": "0", "SRSRAN_AMD_PDSCH_FUSED": "0"}]:
    for k in ("SRSRAN_AMD_LDPC_PK", "SRSRAN_AMD_PDSCH_FUSED"):
        os.environ.pop(k, None)
    os.environ.update(cfg)
    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    T.clear()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        timed("step_host", step)
    host_done = (time.perf_counter() - t0) * 1e3 / n
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t0) * 1e3 / n
    print("%-60s wall %.3f ms/step, host submit %.3f ms/step" % (cfg or "default", wall, host_done))
    for k, v in T.items():
        v = sorted(v)
        print("   %-16s median %.3f ms  min %.3f  max %.3f" % (k, v[len(v) // 2], v[0], v[-1]))

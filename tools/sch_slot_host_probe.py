"""Host time of the sch_slot step's two C-ABI calls (encode_slot, decode_slot: descriptor building, uploads, waits)
beside the step's wall time, and the CPUs this process may run on.  PYTHONPATH=. python tools/sch_slot_host_probe.py"""
import os
import time

import torch

import srsran_project_amd as amd
from bench_slot import make_slot

dev = torch.device("cuda", 0)
plans = make_slot(amd, 64, 8, 4321)
tx, rx, tpos, cpos = [], [], 0, 0
for p in plans:
    tx.append((p, tpos, cpos))
    rx.append((p, 8 * cpos, tpos))
    tpos += p.tbs // 8
    cpos += (p.cw_length + 7) // 8
tbs = torch.randint(0, 256, (tpos,), device=dev, dtype=torch.uint8)
cws = torch.zeros(cpos, dtype=torch.uint8, device=dev)
enc, dec = amd.PdschEncoder(device=0), amd.PuschDecoder("simd", device=0)
cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6)
llrs = torch.randint(-20, 20, (cpos * 8,), device=dev, dtype=torch.int8)
rx_tbs = torch.zeros(tpos, dtype=torch.uint8, device=dev)
txd, rxd = amd.SlotUes(amd.PdschUe, tx), amd.SlotUes(amd.PuschUe, rx)
s = torch.cuda.current_stream(dev)
T = {"encode_slot": [], "decode_slot": []}
for k in range(30):
    t0 = time.perf_counter()
    enc.encode_slot(tbs, txd, out=cws, stream=s)
    t1 = time.perf_counter()
    dec.decode_slot(llrs, rxd, cfg, tbs=rx_tbs, stream=s)
    t2 = time.perf_counter()
    if k >= 5:
        T["encode_slot"].append((t1 - t0) * 1e3)
        T["decode_slot"].append((t2 - t1) * 1e3)
torch.cuda.synchronize(dev)
t0 = time.perf_counter()
for k in range(20):
    enc.encode_slot(tbs, txd, out=cws, stream=s)
    dec.decode_slot(llrs, rxd, cfg, tbs=rx_tbs, stream=s)
torch.cuda.synchronize(dev)
wall = (time.perf_counter() - t0) * 1e3 / 20
aff = sorted(os.sched_getaffinity(0))
print("cpus allowed: %d (%s...), running on cpu %d" % (len(aff), aff[:8], os.sched_getcpu() if hasattr(os, "sched_getcpu") else -1))
for k, v in T.items():
    v = sorted(v)
    print("%-12s host median %.3f ms min %.3f max %.3f" % (k, v[len(v) // 2], v[0], v[-1]))
print("wall %.3f ms per step" % wall)

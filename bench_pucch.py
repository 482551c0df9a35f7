"""bench.py --workload pucch: every PUCCH of a slot of many cells on the MI355X (include/srsran_amd/pucch.h).

One step runs the slot forms of the five formats over --slots-pipeline cells (273 PRBs, 4 receive ports,
numerology 1): per cell 8 Format 0 PDUs (2 symbols, 2 HARQ-ACK bits + SR), 2 Format 1 batches of 12 multiplexed PUCCHs
(14 symbols, hopping), 4 Format 2 PDUs (4 PRBs, 2 symbols, 20-bit CSI), 2 Format 3 PDUs (2 PRBs, 14 symbols,
hopping, 40 bits) and 1 Format 4 PDU (OCC 2, 20 bits): 39 UCI messages per cell.  Grids are synthetic (random
cbf16); the work per PDU does not depend on the received values.  The metric is UCI messages per second; the CPU
baseline is the reference's pucch_processor_impl (oracle/_ref, built once, one thread) over one cell's PDUs.
"""
import ctypes
import threading
import time

import numpy as np

NPRB, PORTS, MU, SLOT = 273, 4, 1, 3


def cell_pdus(amd, grid):
    pu = amd.pucch
    f0 = [pu.make_f0_pdu(numerology=MU, slot_index=SLOT, starting_prb=i, start_symbol_index=12, nof_symbols=2,
                         initial_cyclic_shift=i % 12, n_id=100 + i, nof_harq_ack=2, sr_opportunity=True,
                         ports=(0, 1, 2, 3), grid=grid) for i in range(8)]
    f1 = [pu.make_f1_batch([(ics, occ, 1 + (ics + occ) % 2) for occ in range(2) for ics in range(0, 12, 2)],
                           numerology=MU, slot_index=SLOT, starting_prb=10 + b, second_hop_prb=262 + b,
                           start_symbol_index=0, nof_symbols=14, n_id=300 + b, ports=(0, 1, 2, 3), grid=grid)
          for b in range(2)]
    f2 = [pu.make_f2_pdu(numerology=MU, slot_index=SLOT, bwp_size_rb=NPRB, starting_prb=20 + 4 * i, nof_prb=4,
                         start_symbol_index=12, nof_symbols=2, rnti=0x4601 + i, n_id=7, n_id_0=9, nof_harq_ack=2,
                         nof_csi_part1=18, ports=(0, 1, 2, 3), grid=grid) for i in range(4)]
    f34 = [pu.make_f34_pdu(format=3, numerology=MU, slot_index=SLOT, bwp_size_rb=NPRB, starting_prb=40 + 2 * i,
                           second_hop_prb=230 + 2 * i, nof_prb=2, start_symbol_index=0, nof_symbols=14,
                           rnti=0x5000 + i, n_id_hopping=11, n_id_scrambling=12, nof_harq_ack=4, nof_csi_part1=36,
                           ports=(0, 1, 2, 3), grid=grid) for i in range(2)]
    f34.append(pu.make_f34_pdu(format=4, numerology=MU, slot_index=SLOT, bwp_size_rb=NPRB, starting_prb=50,
                               start_symbol_index=0, nof_symbols=14, rnti=0x6000, n_id_hopping=13,
                               n_id_scrambling=14, nof_harq_ack=2, nof_csi_part1=18, occ_index=1, occ_length=2,
                               ports=(0, 1, 2, 3), grid=grid))
    return f0, f1, f2, f34


def cpu_baseline(args, amd, grid_np):
    """The reference pucch_processor_impl over one cell's PDUs, repeated for about --cpu-seconds."""
    import oracle
    from srsran_project_amd.pucch import PucchF0Pdu, PucchF1Batch, PucchF2Pdu, PucchF34Pdu

    ref = oracle.REF
    f = ref.srs_ref_pucch_time
    f.restype = ctypes.c_double
    P = ctypes.c_void_p
    f.argtypes = [P, ctypes.c_uint, ctypes.c_uint, P, ctypes.c_uint, P, ctypes.c_uint, P, ctypes.c_uint, P,
                  ctypes.c_uint, ctypes.c_uint]
    f0, f1, f2, f34 = cell_pdus(amd, 0)
    a0, a1 = (PucchF0Pdu * len(f0))(*f0), (PucchF1Batch * len(f1))(*f1)
    a2, a34 = (PucchF2Pdu * len(f2))(*f2), (PucchF34Pdu * len(f34))(*f34)
    g = np.ascontiguousarray(grid_np, np.uint32)
    call = lambda reps: f(g.ctypes.data, g.shape[0], g.shape[2], a0, len(f0), a1, len(f1), a2, len(f2), a34,  # noqa
                          len(f34), reps)
    t1 = max(call(1), 1e-6)
    reps = max(1, int(args.cpu_seconds / t1))
    msgs = len(f0) + sum(b.nof_entries for b in f1) + len(f2) + len(f34)
    # the same host-core share as the headline's CPU leg (--cpu-threads, 16 = one GPU's share of the node): one
    # pucch_processor_impl per thread over the cell (ctypes releases the GIL for the call; inputs are read only)
    nth = max(1, args.cpu_threads)
    threads = [threading.Thread(target=call, args=(reps,)) for _ in range(nth)]
    t0 = time.perf_counter()
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    t = time.perf_counter() - t0
    return dict(value=nth * msgs * reps / t, unit="UCI messages/s", cores=nth, kind="reference",
                sample="%d threads x %d passes over one cell's %d PUCCH messages (pucch_processor_impl, one instance "
                       "per thread, %.1f s wall)" % (nth, reps, msgs, t))


def run_pucch(args, dist, world, rank, dev, timed):
    import torch

    import srsran_project_amd as amd

    ncell = args.slots_pipeline
    proc = amd.PucchProcessor(device=dev.index or 0)
    gen = torch.Generator(device=dev).manual_seed(1 + rank)
    grids = torch.randint(-(1 << 31), (1 << 31) - 1, (ncell, PORTS, 14, 12 * NPRB), dtype=torch.int32, device=dev,
                          generator=gen)
    f0, f1, f2, f34 = [], [], [], []
    for c in range(ncell):
        a, b, x, y = cell_pdus(amd, c)
        f0 += a
        f1 += b
        f2 += x
        f34 += y
    msgs = len(f0) + sum(b.nof_entries for b in f1) + len(f2) + len(f34)
    stream = torch.cuda.current_stream(dev)
    # the C-ABI slot calls with their PDU arrays and output buffers built once, as a C++ caller would hold them
    pu = amd.pucch
    L, h = proc._lib, proc._h
    a0, a1 = (pu.PucchF0Pdu * len(f0))(*f0), (pu.PucchF1Batch * len(f1))(*f1)
    a2, a34 = (pu.PucchF2Pdu * len(f2))(*f2), (pu.PucchF34Pdu * len(f34))(*f34)
    n1 = sum(b.nof_entries for b in f1)
    r0 = torch.zeros((len(f0), pu.RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    r1 = torch.zeros((n1, pu.RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    r2 = torch.zeros((len(f2), pu.UCI_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    r34 = torch.zeros((len(f34), pu.UCI_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    p2 = torch.zeros((len(f2), 64), dtype=torch.uint8, device=dev)
    p34 = torch.zeros((len(f34), 64), dtype=torch.uint8, device=dev)
    gp, gs, nsubc = grids.data_ptr(), grids.stride(0), grids.shape[-1]
    sp = ctypes.c_void_p(stream.cuda_stream)
    chk = amd._lib.check

    def c0():
        chk(L.srs_amd_pucch_f0_detect_slot(h, a0, len(f0), gp, gs, ncell, PORTS, nsubc, r0.data_ptr(), sp), "f0")

    def c1():
        chk(L.srs_amd_pucch_f1_detect_slot(h, a1, len(f1), gp, gs, ncell, PORTS, nsubc, r1.data_ptr(), sp), "f1")

    def c2():
        chk(L.srs_amd_pucch_f2_process_slot(h, a2, len(f2), gp, gs, ncell, PORTS, nsubc, r2.data_ptr(), p2.data_ptr(),
                                            64, sp), "f2")

    def c34():
        chk(L.srs_amd_pucch_f34_process_slot(h, a34, len(f34), gp, gs, ncell, PORTS, nsubc, r34.data_ptr(),
                                             p34.data_ptr(), 64, sp), "f34")

    def step():
        c0()
        c1()
        c2()
        c34()

    elapsed, event_ms = timed(args, dist, world, dev, stream, step)
    # per-format device time of one step (events around each slot call, after a synchronise)
    fmt_ms = {}
    for name, fn in (("f0", c0), ("f1", c1), ("f2", c2), ("f34", c34)):
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(5):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        fmt_ms[name] = dict(device_ms=round(e0.elapsed_time(e1) / 5, 4),
                            wall_ms=round((time.perf_counter() - t0) * 1e3 / 5, 4))
    ms = elapsed * 1e3 / args.steps
    line = {
        "metric": "PUCCH UCI messages/s (Formats 0-4, slot forms)",
        "value": round(msgs * world / (elapsed / args.steps), 1),
        "unit": "UCI messages/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
        "event_ms_per_step": round(event_ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 (cbf16 grids)",
        "data": "synthetic (random cbf16 grids)",
        "config": {"workload": "pucch: %d cells x (8 F0 + 2 F1 batches of 12 + 4 F2 + 2 F3 + 1 F4), 273 PRB, 4 rx, "
                               "numerology 1" % ncell, "messages_per_step": msgs, "pdus_per_cell": 39},
        "per_format": fmt_ms,
        "roofline": None,
    }
    if rank == 0 and not args.no_cpu_baseline:
        g0 = grids[0].cpu().numpy().view(np.uint32)
        line["cpu_baseline"] = cpu_baseline(args, amd, g0)
    return line

"""`bench.py --workload sch_slot`: the channel coding of heterogeneous slots.

Every cell carries `--ues-per-cell` UEs whose PRB share, MCS (QPSK .. 256QAM) and layer count
differ, so their transport blocks segment differently (BG1/BG2, many lifting sizes, CRC16/24A/24B).
One step PDSCH-encodes every UE's TB of the batch (srs_amd_pdsch_encode_slot) and PUSCH-decodes every
UE's received codeword (srs_amd_pusch_decode_slot, new transmissions) -- the transport-block chains of
pdsch_encoder_impl / pusch_decoder_impl for all PDUs of the cells' slots, each as one launch sequence.
The same slot is also timed with one per-plan `_batch` launch sequence per UE (what a uniform-batch API
costs on a mixed slot).  Synthetic data: random TBs, LLRs = the encoded bits at +-10 plus Gaussian noise.
"""
import numpy as np

# (Qm, R x 1024): a spread of the MCS table (TS 38.214 table 5.1.3.1-2)
MCS = [(2, 308), (2, 602), (4, 434), (4, 616), (6, 567), (6, 719), (6, 873), (8, 682.5), (8, 797), (8, 948)]
NOF_PRB = 273
DATA_SYMBOLS = 12   # 14 OFDM symbols, 2 DM-RS
DMRS_RE_PER_PRB = 24


def base_graph(tbs, rate):
    """TS 38.212 7.2.2 base-graph selection (the reference's get_ldpc_base_graph)."""
    if tbs <= 292 or (tbs <= 3824 and rate <= 0.67) or rate <= 0.25:
        return 2
    return 1


def make_slot(amd, cells, ues_per_cell, seed):
    """Plans of every UE of `cells` cells: PRBs split at random, MCS and layers drawn per UE."""
    rng = np.random.default_rng(seed)
    plans = []
    for _ in range(cells):
        cuts = np.sort(rng.choice(np.arange(1, NOF_PRB), ues_per_cell - 1, replace=False))
        prbs = np.diff(np.concatenate([[0], cuts, [NOF_PRB]]))
        for n_prb in prbs:
            qm, r = MCS[rng.integers(len(MCS))]
            layers = int(rng.integers(1, 5))
            tbs = amd.tbs_calculator_calculate(14, DMRS_RE_PER_PRB, 0, qm, r, layers, 0, int(n_prb))
            nre = int(n_prb) * 12 * DATA_SYMBOLS * layers
            plans.append(amd.sch_plan(tbs, base_graph(tbs, r / 1024), 0, qm, 0, layers, nre))
    return plans


def run_sch_slot(args, dist, world, rank, dev, timed):
    import torch

    import srsran_project_amd as amd

    cells = args.slots_pipeline
    plans = make_slot(amd, cells, args.ues_per_cell, 4321 + rank)
    tx_ues, rx_ues, tpos, cpos = [], [], 0, 0
    for p in plans:
        tx_ues.append((p, tpos, cpos))
        rx_ues.append((p, 8 * cpos, tpos))  # LLR u at bit u of the packed codewords
        tpos += p.tbs // 8
        cpos += (p.cw_length + 7) // 8
    g = torch.Generator(device=dev)
    g.manual_seed(99 + rank)
    tbs = torch.randint(0, 256, (tpos,), device=dev, generator=g, dtype=torch.uint8)
    cws = torch.zeros(cpos, dtype=torch.uint8, device=dev)
    enc = amd.PdschEncoder(device=dev.index)
    dec = amd.PuschDecoder(args.arith, device=dev.index)
    cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6)
    stream = torch.cuda.current_stream(dev)
    # received codewords: the encoded bits at +-10 LLRs plus noise (sigma 3: decodable at every MCS)
    enc.encode_slot(tbs, tx_ues, out=cws, stream=stream)
    shifts = torch.arange(7, -1, -1, device=dev, dtype=torch.uint8)
    bits = ((cws[:, None] >> shifts) & 1).reshape(-1).float()
    llrs = ((1 - 2 * bits) * 10 + 3 * torch.randn(bits.shape, device=dev, generator=g)).round().clamp(-120, 120)
    llrs = llrs.to(torch.int8)
    rx_tbs = torch.zeros(tpos, dtype=torch.uint8, device=dev)
    # the slot's C descriptor arrays, built once (a PHY builds them natively per slot)
    tx_desc, rx_desc = amd.SlotUes(amd.PdschUe, tx_ues), amd.SlotUes(amd.PuschUe, rx_ues)

    def step():
        enc.encode_slot(tbs, tx_desc, out=cws, stream=stream)
        dec.decode_slot(llrs, rx_desc, cfg, tbs=rx_tbs, stream=stream)

    elapsed, step_ms = timed(args, dist, world, dev, stream, step)
    _, res = dec.decode_slot(llrs, rx_ues, cfg, tbs=rx_tbs, stream=stream)
    torch.cuda.synchronize(dev)
    res = res.cpu().numpy()
    ok = float(res[:, 0].mean())
    tb_equal = bool(torch.equal(rx_tbs, tbs))

    # the same slot as one per-plan launch sequence per UE
    per_ue = {}
    if not args.no_latency:
        def step_per_ue():
            for (p, to, co), (_, lo, _) in zip(tx_ues, rx_ues):
                enc.encode_batch(tbs[to:to + p.tbs // 8].view(1, -1), p, out=cws[co:co + (p.cw_length + 7) // 8]
                                 .view(1, -1), stream=stream)
                dec.decode_batch(llrs[lo:lo + p.cw_length].view(1, -1), p, cfg,
                                 tbs=rx_tbs[to:to + p.tbs // 8].view(1, -1), stream=stream)
        for _ in range(2):
            step_per_ue()
        torch.cuda.synchronize(dev)
        import time
        t0 = time.perf_counter()
        n = max(2, args.steps // 4)
        for _ in range(n):
            step_per_ue()
        torch.cuda.synchronize(dev)
        per_ue = {"ms_per_step": (time.perf_counter() - t0) / n * 1e3, "launch_sequences": 2 * len(plans)}

    cbs_tx = sum(p.nof_segments for p in plans)
    total_cbs = 2 * cbs_tx * args.steps * world
    if rank != 0:
        return None
    bgs = sorted({(p.base_graph, p.lifting_size) for p in plans})
    return {
        "metric": "PDSCH encode + PUSCH decode codeblocks/s, heterogeneous slots (per-UE PRB / MCS / layers)",
        "value": total_cbs / elapsed,
        "unit": "codeblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (random TBs; LLRs = encoded bits at +-10 + N(0, 3^2))",
        "config": {
            "workload": "sch_slot: %d cells x %d UEs (273 PRB split at random, MCS QPSK..256QAM, 1-4 layers)"
                        % (cells, args.ues_per_cell),
            "ues_per_step_per_gpu": len(plans),
            "codeblocks_per_step_per_gpu": 2 * cbs_tx,
            "distinct_lifting_sizes": len(bgs),
            "parallelism": "cells sharded over ranks" if world > 1 else "single GPU",
        },
        "step_event_ms": step_ms,
        "pusch_tb_ok_fraction": ok,
        "pusch_tbs_equal_sent": tb_equal,
        "per_ue_launches": per_ue,
    }

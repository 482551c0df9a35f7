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


class SlotPipeline:
    """`bench.py --workload slot_pipeline`: the full PDSCH + PUSCH chains of cells whose 273 PRBs are shared by
    `ues_per_cell` UEs (own PRBs, MCS, layers, rnti).  Per step and rank:
      PDSCH  every UE's TB -> srs_amd_pdsch_encode_slot (one launch sequence) -> srs_amd_pdsch_modulate_slot
             (data + DM-RS of every PDU of every cell: two launches) -> OFDM modulator (4 ports per cell);
      PUSCH  OFDM demodulator (4 rx ports per cell) -> srs_amd_pusch_process_slot (estimator, fused equalizer,
             slot decoder, results of every PDU of every cell: one launch sequence).
    DL: 1-4 layers on 4 ports (DFT precoding), symbols 1-13.  UL: 1-2 layers (the reference-pinned ZF) through a
    fixed channel + AWGN, symbols 0-13; the UE transmissions are synthesised before the timed region (the PDSCH
    modulator as the UE transmitter, per-UE channel as its precoder) and every run checks the decoded TBs."""

    def __init__(self, cells, ues_per_cell, dev, seed=0, iters=6, snr_db=35.0, ul_max_layers=2, mixed=False):
        import torch

        import bench_pipeline as bp
        import srsran_project_amd as amd

        self.torch, self.dev, self.S = torch, dev, cells
        d = dev.index
        rng = np.random.default_rng(777 + seed)
        self.enc = amd.PdschEncoder(device=d)
        self.mod = amd.PdschModulator(device=d)
        self.proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters), device=d)
        self.ofdm_mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(bp.MU, NOF_PRB, bp.NFFT, 0, 1.0, 3.5e9),
                                              device=d)
        self.ofdm_dem = amd.OfdmSlotDemodulator(
            amd.OfdmDemodulatorConfiguration(bp.MU, NOF_PRB, bp.NFFT, 0, 1.0, 3.5e9, 0), device=d)
        nsubc = 12 * NOF_PRB
        dl, ul, ue_tx = [], [], []   # (sch plan, mod plan, dmrs, cell) / (processor plan, cell) / UE TX
        self.kinds = []              # UL PDU kinds (mixed: "uci", "harq", "tp" or "data")
        self.tp_ues = []             # DFT-s-OFDM UEs: (cell, first PRB, end PRB, channel [port], n_rs_id)
        self.ul_pdus = []            # the UL PDUs (UCI UEs multiplex their UCI REs at the transmitter)
        self.uci_sent = {}           # CSI part 1 / CSI part 2 payloads of the "csi2" / "ucionly" UEs, by UL PDU index
        for c in range(cells):
            n_id = int(rng.integers(0, 1008))
            for side in ("dl", "ul"):
                cuts = np.sort(rng.choice(np.arange(1, NOF_PRB), ues_per_cell - 1, replace=False))
                edges = np.concatenate([[0], cuts, [NOF_PRB]])
                for u in range(ues_per_cell):
                    lo, hi = int(edges[u]), int(edges[u + 1])
                    crbs = list(range(lo, hi))
                    qm, r = MCS[rng.integers(len(MCS))]
                    rnti = int(rng.integers(1, 65520))
                    if side == "dl":
                        layers = int(rng.integers(1, 5))
                        w = bp.dl_weights(layers, 4)
                        mp = self.mod.plan(amd.PdschModulatorConfig(
                            rnti=rnti, bwp_start=0, bwp_size=NOF_PRB, modulation=qm, crbs=crbs, start_symbol=1,
                            nof_symbols=13, dmrs_symb_pos=bp.DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=2,
                            n_id=n_id, precoding=w), nsubc)
                        tbs = amd.tbs_calculator_calculate(13, 24, 0, qm, r, layers, 0, hi - lo)
                        sp = amd.sch_plan(tbs, base_graph(tbs, r / 1024), 0, qm, 0, layers, mp.nof_re * layers)
                        assert sp.cw_length == mp.nof_bits
                        dm = amd.DmrsPdschConfig(slot_index=bp.SLOT, reference_point_k_rb=0, type=1,
                                                 scrambling_id=n_id, n_scid=False, amplitude=bp.DMRS_AMP,
                                                 symbols_mask=bp.DMRS_MASK, crbs=crbs, precoding=w)
                        dl.append((sp, mp, dm, c))
                    else:
                        j = len(ul)
                        kind = "data"
                        if mixed:
                            # ~20 % HARQ-ACK + CSI part 1 on the UL-SCH, ~6 % CSI part 1 + CSI part 2 (its size from
                            # the CSI part 1 payload) on the UL-SCH, ~3 % UCI-only PUSCH (CSI part 1 + CSI part 2, no
                            # codeword), ~10 % retransmissions (new_data = 0, combined into a soft buffer; rv 0,
                            # decodable alone from the cleared buffer), ~3 % DFT-s-OFDM
                            kind = ("tp" if j % 32 == 17 else "ucionly" if j % 32 == 9 else "csi2" if j % 16 == 7
                                    else "uci" if j % 5 == 1 else "harq" if j % 10 == 3 else "data")
                        layers = 1 if kind in ("tp", "uci", "csi2", "ucionly") else int(rng.integers(1, ul_max_layers + 1))
                        if kind == "ucionly":
                            # one polar codeword per UCI field: a narrow allocation (E <= 8192)
                            hi = lo + min(hi - lo, 6)
                            crbs = list(range(lo, hi))
                        if kind == "tp":
                            n = hi - lo
                            while not amd.transform_precoding_nof_prbs_valid(n):
                                n -= 1
                            hi = lo + n
                            crbs = list(range(lo, hi))
                        extra = {}
                        if kind == "uci":
                            extra = dict(nof_harq_ack=4, nof_csi_part1=20, beta_offset_harq_ack=8.0,
                                         beta_offset_csi_part1=6.25, alpha_scaling=1.0)
                        if kind == "tp":
                            extra = dict(transform_precoding=1, n_rs_id=n_id)
                        if kind in ("csi2", "ucionly"):
                            # (UCI-only PUSCH carries no CSI part 2: the reference sizes CSI part 1 of a UCI-only PDU
                            # for "no CSI part 2" before CSI part 2 is known, ulsch_info.cpp:96-123)
                            extra = dict(nof_csi_part1=CSI1_BITS, beta_offset_csi_part1=6.25, alpha_scaling=1.0)
                            if kind == "csi2":
                                extra.update(beta_offset_csi_part2=5.0, csi_part2_size=PART2)
                        rv, new_data = (0, 0) if kind == "harq" else (0, 1)
                        tbs = 0 if kind == "ucionly" else amd.tbs_calculator_calculate(14, 24, 0, qm, r, layers, 0, hi - lo)
                        pdu = amd.make_pdu(numerology=bp.MU, slot_index=bp.SLOT, rnti=rnti, bwp_start_rb=0,
                                           bwp_size_rb=NOF_PRB, modulation=qm, target_code_rate=r, rv=rv,
                                           base_graph=base_graph(tbs, r / 1024), new_data=new_data, n_id=n_id,
                                           nof_tx_layers=layers, nof_rx_ports=4, dmrs_symbol_mask=bp.DMRS_MASK,
                                           scrambling_id=n_id, n_scid=0, nof_cdm_groups_without_data=2, rb_start=lo,
                                           rb_count=hi - lo, start_symbol_index=0, nof_symbols=14, tbs=tbs, **extra)
                        self.kinds.append(kind)
                        self.ul_pdus.append(pdu)
                        pp = self.proc.plan(pdu, nsubc)
                        h = bp.ul_channel(layers, 4)
                        mp = self.mod.plan(amd.PdschModulatorConfig(
                            rnti=rnti, bwp_start=0, bwp_size=NOF_PRB, modulation=qm, crbs=crbs, start_symbol=0,
                            nof_symbols=14, dmrs_symb_pos=bp.DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=2,
                            n_id=n_id, precoding=h), nsubc)
                        assert kind in ("uci", "csi2", "ucionly") or mp.nof_bits == pp.sch.cw_length
                        dm = amd.DmrsPdschConfig(slot_index=bp.SLOT, reference_point_k_rb=0, type=1,
                                                 scrambling_id=n_id, n_scid=False, amplitude=bp.DMRS_AMP,
                                                 symbols_mask=bp.DMRS_MASK, crbs=crbs, precoding=h)
                        ul.append((pp, c))
                        if kind == "tp":
                            self.tp_ues.append((c, lo, hi, h[0], n_id))
                        # the UE transmits the codeword of the PDU's own rv (UCI UEs multiplexed and DFT-s-OFDM
                        # UEs DFT-spread below); a CSI part 2 UE rate-matches its UL-SCH to the REs its CSI part 2
                        # leaves (the size its CSI part 1 payload selects)
                        sp_tx = pp.sch
                        if kind in ("csi2", "ucionly"):
                            csi1 = rng.integers(0, 2, CSI1_BITS).astype(np.uint8)
                            n2 = amd.uci_part2_get_size(csi1, pdu.csi_part2_size) if kind == "csi2" else 0
                            self.uci_sent[j] = (csi1, rng.integers(0, 2, n2).astype(np.uint8))
                            if kind == "csi2" and n2:
                                g = self._ulsch_info(amd, pdu, n2)["nof_ul_sch_bits"]
                                sp_tx = amd.sch_plan(tbs, pdu.base_graph, 0, qm, pp.sch.Nref, layers, g // qm)
                        ue_tx.append((sp_tx, mp, dm, c))
        self.dl, self.ul = dl, ul
        g = torch.Generator(device=dev)
        g.manual_seed(4242 + d + 7919 * seed)
        # ---- PDSCH: TBs, codewords, grids, samples ------------------------------------------------------------
        self.tx_ues, tpos, cpos = [], 0, 0
        for sp, _, _, _ in dl:
            self.tx_ues.append((sp, tpos, cpos))
            tpos += sp.tbs // 8
            cpos += (sp.cw_length + 7) // 8 + 64
        self.tb_dl = torch.randint(0, 256, (tpos,), device=dev, dtype=torch.uint8, generator=g)
        self.cw_dl = torch.zeros(cpos, dtype=torch.uint8, device=dev)
        self.tx_desc = amd.SlotUes(amd.PdschUe, self.tx_ues)
        self.dl_slot = amd.PdschSlot([(mp, dm, c, co) for (sp, mp, dm, c), (_, _, co) in zip(dl, self.tx_ues)])
        self.grid_dl = torch.zeros((cells, 4, 14, nsubc), dtype=torch.int32, device=dev)
        self.samp_dl = torch.empty((cells, 4, self.ofdm_mod.max_slot_size()), dtype=torch.complex64, device=dev)
        # ---- PUSCH: the UE transmissions (untimed), received grids, results -------------------------------------
        ul_ues, tpos, cpos = [], 0, 0
        for sp, _, _, _ in ue_tx:
            ul_ues.append((sp, tpos, cpos))
            tpos += sp.tbs // 8
            cpos += (sp.cw_length + 7) // 8 + 64
        self.tb_ul = torch.randint(0, 256, (max(tpos, 1),), device=dev, dtype=torch.uint8, generator=g)
        cw_ul = torch.zeros(cpos, dtype=torch.uint8, device=dev)
        self.enc.encode_slot(self.tb_ul, [u for u, k in zip(ul_ues, self.kinds) if k != "ucionly"], out=cw_ul)
        # the UEs' transmitted codewords: the UL-SCH codeword, or for a UCI UE the whole multiplexed codeword (its
        # UL-SCH bits at the REs the receiver's demultiplexer takes them from; random bits on the HARQ-ACK / CSI part 1
        # REs of "uci" UEs, the encoded CSI part 1 / CSI part 2 of "csi2" / "ucionly" UEs)
        cw_host = cw_ul.cpu().numpy()
        tx_parts, tx_off, pos = [], [], 0
        for j, ((sp, mp, dm, c), (_, _, co)) in enumerate(zip(ue_tx, ul_ues)):
            if self.kinds[j] in ("uci", "csi2", "ucionly"):
                sch = (np.unpackbits(cw_host[co:co + (sp.cw_length + 7) // 8])[:sp.cw_length]
                       if self.kinds[j] != "ucionly" else np.zeros(0, np.uint8))
                part = np.packbits(self._multiplex(amd, self.ul_pdus[j], sch, mp.nof_bits, rng, j))
            else:
                part = cw_host[co:co + (sp.cw_length + 7) // 8]
            tx_off.append(pos)
            tx_parts.append(part)
            pos += (part.size + 63) // 64 * 64
        cw_tx = np.zeros(max(pos, 1), np.uint8)
        for off, part in zip(tx_off, tx_parts):
            cw_tx[off:off + part.size] = part
        grid = torch.zeros((cells, 4, 14, nsubc), dtype=torch.int32, device=dev)
        self.mod.modulate_slot(grid, amd.PdschSlot([(mp, dm, c, off) for (sp, mp, dm, c), off in zip(ue_tx, tx_off)]),
                               codewords=torch.from_numpy(cw_tx).to(dev))
        for c, lo, hi, h, n_rs_id in self.tp_ues:
            self._transform_precode(amd, bp, grid, c, lo, hi, h, n_rs_id)
        samp = self.ofdm_mod.modulate_batch(grid.view(torch.int16).view(cells, 4, 14, 2 * nsubc), bp.SLOT)
        p = float(torch.mean(torch.abs(samp) ** 2).item())
        sigma = np.sqrt(p / 10 ** (snr_db / 10) / 2)
        noise = torch.complex(torch.randn(samp.shape, device=dev, generator=g),
                              torch.randn(samp.shape, device=dev, generator=g)) * sigma
        self.samp_ul = (samp + noise.to(torch.complex64)).contiguous()
        self.ul_tb_off = [to for _, to, _ in ul_ues]
        # retransmissions: one soft buffer each, cleared at the start of every step (the state a failed first
        # transmission leaves is modelled as empty; clearing keeps every step's decoding work the same)
        soft_sizes = [amd.soft_buffer_size(pp.sch) if k == "harq" else 0 for (pp, _), k in zip(ul, self.kinds)]
        self.soft_all = torch.zeros(max(sum((n + 255) // 256 * 256 for n in soft_sizes), 1), dtype=torch.int8,
                                    device=dev)
        items, off = [], 0
        for (pp, c), n in zip(ul, soft_sizes):
            if n:
                items.append((pp, c, self.soft_all[off:off + n]))
                off += (n + 255) // 256 * 256
            else:
                items.append((pp, c))
        self.ul_slot = amd.PuschSlot(items)
        self.uci = torch.zeros(max(self.ul_slot.uci_total, 1), dtype=torch.uint8, device=dev)
        self.grid_ul = torch.zeros((cells, 4, 14, nsubc), dtype=torch.int32, device=dev)
        self.tb_rx = torch.zeros(max(self.ul_slot.tb_total, 1), dtype=torch.uint8, device=dev)
        self.res_ul = torch.zeros((len(ul), amd.pusch_processor.RESULT_BYTES), dtype=torch.uint8, device=dev)
        self.ul_stream = None
        torch.cuda.synchronize(dev)

    @staticmethod
    def _ulsch_info(amd, pdu, n2):
        """get_ulsch_information of a UL PDU with n2 CSI part 2 bits."""
        return amd.ulsch_information(amd.UlschConfig(
            tbs=pdu.tbs, modulation=pdu.modulation, target_code_rate=pdu.target_code_rate,
            nof_harq_ack_bits=pdu.nof_harq_ack, nof_csi_part1_bits=pdu.nof_csi_part1, nof_csi_part2_bits=n2,
            alpha_scaling=pdu.alpha_scaling, beta_offset_harq_ack=pdu.beta_offset_harq_ack,
            beta_offset_csi_part1=pdu.beta_offset_csi_part1, beta_offset_csi_part2=pdu.beta_offset_csi_part2,
            nof_rb=pdu.rb_count, start_symbol_index=pdu.start_symbol_index, nof_symbols=pdu.nof_symbols,
            dmrs_type=pdu.dmrs_type, dmrs_symbol_mask=pdu.dmrs_symbol_mask,
            nof_cdm_groups_without_data=pdu.nof_cdm_groups_without_data, nof_layers=pdu.nof_tx_layers))

    def _multiplex(self, amd, pdu, sch_bits, nof_bits, rng, j):
        """UE-side UL-SCH / UCI multiplexing for the timing bench (untimed setup): every stream placed where the
        MI355X demultiplexer (srs_amd_ulsch_demultiplex, this library's own) reads it -- found by passing
        RE-index-coded LLRs through it, seven bits per pass.  HARQ-ACK / CSI part 1 of "uci" UEs are random bits (the
        bench checks their transport blocks); "csi2" / "ucionly" UEs send an encoded CSI part 1 (polar, CRC11) whose
        first bits select the CSI part 2 size, and that CSI part 2 encoded the same way (TS 38.212 6.3.2.4), checked
        by check() -- so the receiver's device-side CSI part 2 sizing is exercised with real sizes."""
        qm, L = pdu.modulation, pdu.nof_tx_layers
        bpre = qm * L
        nre = nof_bits // bpre
        csi1, csi2 = self.uci_sent.get(j, (None, None))
        n2 = csi2.size if csi2 is not None else 0
        info = self._ulsch_info(amd, pdu, n2)
        if not hasattr(self, "_demux"):
            self._demux = amd.UlschDemux(device=self.dev.index)
        plan = self._demux.plan(amd.UlschDemuxConfig(
            qm, L, pdu.rb_count, pdu.start_symbol_index, pdu.nof_symbols, info["nof_harq_ack_rvd"], pdu.dmrs_type,
            pdu.dmrs_symbol_mask, pdu.nof_cdm_groups_without_data, pdu.nof_harq_ack, info["nof_harq_ack_bits"],
            pdu.nof_csi_part1, info["nof_csi_part1_bits"], (pdu.rnti << 15) + pdu.n_id, n2,
            info["nof_csi_part2_bits"] if n2 else 0))
        if pdu.tbs == 0:  # UCI only: the REs the UCI leaves carry nothing the receiver decodes
            sch_bits = rng.integers(0, 2, plan.nof_sch_bits).astype(np.uint8)
        assert plan.nof_codeword_bits == nof_bits and plan.nof_sch_bits == sch_bits.size, (
            j, self.kinds[j], n2, plan.nof_codeword_bits, nof_bits, plan.nof_sch_bits, sch_bits.size)
        streams = None
        for k in range(3):
            code = (((np.arange(nre) >> (7 * k)) & 0x7F) + 1).astype(np.int8)
            out = self._demux.demultiplex(np.repeat(code, bpre), plan)
            if streams is None:
                streams = [np.zeros(o.size // bpre, np.int64) for o in out]
            for s, o in zip(streams, out):
                s += (np.abs(o[::bpre].astype(np.int64)) - 1) << (7 * k)  # 128 wraps to -128 in int8
        cw = rng.integers(0, 2, nof_bits).astype(np.uint8)

        def place(re_of, bits):
            cw[(re_of[:, None] * bpre + np.arange(bpre)).ravel()] = bits

        place(streams[0], sch_bits)
        if csi1 is not None:
            place(streams[2], _uci_encode(amd, csi1, info["nof_csi_part1_bits"], self.dev.index))
            if n2:
                place(streams[3], _uci_encode(amd, csi2, info["nof_csi_part2_bits"], self.dev.index))
        return cw

    def _transform_precode(self, amd, bp, grid, c, lo, hi, h, n_rs_id):
        """A DFT-s-OFDM UE's transmission (untimed setup): the data symbols the PDSCH modulator mapped (scrambled,
        modulated, times the channel h[port]) DFT-spread over the allocation per OFDM symbol (TS 38.211 6.3.1.4,
        unit-energy DFT; one layer, so the per-port channel factor commutes with the DFT), and the DM-RS replaced by
        the low-PAPR sequence of n_rs_id on the even subcarriers (TS 38.211 6.4.1.1.1.2, no hopping, one layer)."""
        torch = self.torch
        k0, k1 = 12 * lo, 12 * hi
        g = grid[c].view(torch.int16).view(4, 14, 2 * grid.shape[-1])
        x = g[:, :, 2 * k0:2 * k1].contiguous().view(torch.bfloat16).float().view(4, 14, k1 - k0, 2)
        z = torch.view_as_complex(x.contiguous())
        seq = torch.from_numpy(amd.low_papr_sequence((k1 - k0) // 2, n_rs_id % 30)).to(z.device)
        for l in range(14):
            if (bp.DMRS_MASK >> l) & 1:
                z[:, l, :] = 0
                for p in range(4):
                    z[p, l, 0::2] = seq * np.complex64(bp.DMRS_AMP * h[p])
            else:
                z[:, l, :] = torch.fft.fft(z[:, l, :], norm="ortho")
        y = torch.view_as_real(z).to(torch.bfloat16).contiguous().view(torch.int16).view(4, 14, 2 * (k1 - k0))
        g[:, :, 2 * k0:2 * k1] = y

    def pdsch(self, stream):
        import bench_pipeline as bp

        t = self.torch
        self.enc.encode_slot(self.tb_dl, self.tx_desc, out=self.cw_dl, stream=stream)
        self.mod.modulate_slot(self.grid_dl, self.dl_slot, codewords=self.cw_dl, stream=stream)
        self.ofdm_mod.modulate_batch(self.grid_dl.view(t.int16).view(self.S, 4, 14, 2 * 12 * NOF_PRB), bp.SLOT,
                                     out=self.samp_dl, stream=stream)

    def pusch(self, stream):
        import bench_pipeline as bp

        t = self.torch
        self.ofdm_dem.demodulate_batch(self.samp_ul, bp.SLOT,
                                       grid=self.grid_ul.view(t.int16).view(self.S, 4, 14, 2 * 12 * NOF_PRB),
                                       stream=stream)
        if any(k == "harq" for k in self.kinds):
            self.soft_all.zero_()
        self.proc.process_slot(self.grid_ul, self.ul_slot, tbs=self.tb_rx, results=self.res_ul, stream=stream,
                               uci=self.uci if self.ul_slot.uci_total else None)

    def step(self, stream):
        """Both chains of every cell, concurrently on two HIP streams (fork / join on `stream`)."""
        import bench_pipeline as bp

        t = self.torch
        if self.ul_stream is None:
            self.dl_stream, self.ul_stream = bp.chain_streams(t, self.dev)
            self.ev_fork, self.ev_join = t.cuda.Event(), [t.cuda.Event(), t.cuda.Event()]
        self.ev_fork.record(stream)
        self.dl_stream.wait_event(self.ev_fork)
        self.ul_stream.wait_event(self.ev_fork)
        with t.cuda.stream(self.dl_stream):
            self.pdsch(self.dl_stream)
        with t.cuda.stream(self.ul_stream):
            self.pusch(self.ul_stream)
        self.ev_join[0].record(self.dl_stream)
        self.ev_join[1].record(self.ul_stream)
        stream.wait_event(self.ev_join[0])
        stream.wait_event(self.ev_join[1])

    def check(self):
        """Fraction of PUSCH TBs with CRC ok and equal to what the UE sent, mean LDPC iterations per codeblock."""
        import srsran_project_amd as amd

        res = amd.pusch_processor.parse_results(self.res_ul.cpu().numpy())
        rx, tx = self.tb_rx.cpu().numpy(), self.tb_ul.cpu().numpy()
        ok = []
        self.ok_by_kind = {}
        uci = self.uci.cpu().numpy()
        for j, ((pp, _), r, off, toff, k) in enumerate(zip(self.ul, res, self.ul_slot.offsets, self.ul_tb_off,
                                                           self.kinds)):
            n = pp.tb_bytes
            good = k == "ucionly" or (bool(r.data.tb_crc_ok) and np.array_equal(rx[off:off + n], tx[toff:toff + n]))
            if j in self.uci_sent:
                # CSI part 1 and the CSI part 2 of the size it selected, as the UE sent them
                csi1, csi2 = self.uci_sent[j]
                row = uci[self.ul_slot.uci_offsets[j]:]
                n1 = csi1.size
                good = (good and r.csi_part1_status == 1 and np.array_equal(row[:n1], csi1)
                        and r.nof_csi_part2 == csi2.size and (csi2.size == 0 or (
                            r.csi_part2_status == 1 and np.array_equal(row[n1:n1 + csi2.size], csi2))))
            ok.append(good)
            self.ok_by_kind.setdefault(k, []).append(ok[-1])
        self.ok_by_kind = {k: float(np.mean(v)) for k, v in self.ok_by_kind.items()}
        its = sum(r.data.ldpc_iterations_sum for r in res) / max(1, sum(r.data.nof_codeblocks_total for r in res))
        return float(np.mean(ok)), float(its)

    def codeblocks(self):
        return (sum(sp.nof_segments for sp, _, _, _ in self.dl), sum(pp.sch.nof_segments for pp, _ in self.ul))


# CSI part 1 / CSI part 2 of the mixed slot's "csi2" and "ucionly" UEs: 20 CSI part 1 bits (polar, CRC11) whose
# first two bits select a CSI part 2 of 0, 20, 24 or 40 bits (uci_part2_size_description, one entry)
CSI1_BITS = 20
PART2 = [([(0, 2)], [0, 20, 24, 40])]


def _uci_crc(bits, L):
    """TS 38.212 5.1 CRC6 (D^6 + D^5 + 1) / CRC11 (D^11 + D^10 + D^9 + D^5 + 1) parity bits of a UCI payload."""
    poly = {6: 0x21, 11: 0x621}[L]
    reg = 0
    for b in bits:
        fb = ((reg >> (L - 1)) & 1) ^ int(b)
        reg = (reg << 1) & ((1 << L) - 1)
        reg ^= poly if fb else 0
    return np.array([(reg >> (L - 1 - i)) & 1 for i in range(L)], np.uint8)


_POLAR = {}


def _uci_encode(amd, payload, E, device):
    """UCI on PUSCH for 12 <= A < 360 payload bits: CRC, polar code (nMax 10, channel interleaver), rate matching to
    E bits (TS 38.212 6.3.2.4 / 5.3.1; the decoder side is uci_decoder_impl)."""
    A = payload.size
    L = 6 if A < 20 else 11
    assert 12 <= A < 360
    key = (A + L, E, device)
    if key not in _POLAR:
        _POLAR[key] = amd.PolarCode(A + L, E, 10, amd.PolarCodeIbil.present, device=device)
    return _POLAR[key].encode(np.concatenate([payload, _uci_crc(payload, L)]))


def run_slot_pipeline(args, dist, world, rank, dev, timed):
    import torch

    cells = args.slots_pipeline
    pl = SlotPipeline(cells, args.ues_per_cell, dev, seed=rank, iters=args.iters, snr_db=args.snr_db,
                      mixed=args.mixed)
    stream = torch.cuda.current_stream(dev)
    elapsed, step_ms = timed(args, dist, world, dev, stream, lambda: pl.step(stream))
    torch.cuda.synchronize(dev)
    ok, its = pl.check()
    cb_dl, cb_ul = pl.codeblocks()
    if rank != 0:
        return None
    return {
        "metric": "PDSCH+PUSCH codeblocks/s, multi-UE slots (per-UE PRBs / MCS / layers / rnti on shared grids)",
        "value": (cb_dl + cb_ul) * args.steps * world / elapsed,
        "unit": "codeblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8 LLR / bf16 grid / f32 DSP",
        "data": "synthetic (random TBs; UE transmissions through fixed channels + AWGN at %.1f dB)" % args.snr_db,
        "config": {
            "workload": "slot_pipeline: %d cells x %d DL + %d UL UEs (273 PRB split at random, MCS QPSK..256QAM, "
                        "DL 1-4 layers x 4 ports, UL 1-2 layers x 4 rx ports, ZF)"
                        % (cells, args.ues_per_cell, args.ues_per_cell),
            "pdus_per_step_per_gpu": len(pl.dl) + len(pl.ul),
            "codeblocks_per_step_per_gpu": {"pdsch": cb_dl, "pusch": cb_ul},
            "parallelism": "cells sharded over ranks" if world > 1 else "single GPU",
        },
        "step_event_ms": step_ms,
        "pusch_pdu_kinds": {k: pl.kinds.count(k) for k in sorted(set(pl.kinds))},
        "pusch_tb_ok_fraction_by_kind": pl.ok_by_kind,
        "pusch_tb_ok_fraction": ok,
        "pusch_mean_ldpc_iterations": its,
    }

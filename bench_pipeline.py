"""bench_pipeline.py -- the `--workload pipeline` leg of bench.py: the full
PDSCH + PUSCH slot chain of one 100 MHz cell per slot (BASELINE.json metric
"PDSCH+PUSCH codeblocks/s (and Gb/s) @ 100 MHz 273-PRB 4x4 MIMO").

Per slot (= one cell; `--slots` cells per step and rank, all resident in HBM):
  PDSCH  (gNB TX, 4 layers x 4 ports, 256QAM R = 948/1024, 273 PRB, symbols 1-13)
         transport block -> pdsch_encoder (CRC, segmentation, LDPC, rate matching)
         -> pdsch_modulator (scrambling, modulation, layer mapping, precoding, RE mapping)
         -> dmrs_pdsch_processor -> OFDM modulator (4096-point IDFT, CP) -> baseband.
  PUSCH  (gNB RX, 2 layers x 4 rx ports -- the widest spatial setting the open reference
         equalizer supports -- 256QAM R = 948/1024, 273 PRB, symbols 0-13)
         baseband -> OFDM demodulator -> DM-RS channel estimator (filter / average / CFO)
         -> pusch_demodulator (equalizer, soft demapper, descrambler)
         -> pusch_decoder (rate dematching, LDPC decoding with CRC early stop, CB/TB CRC).
The PUSCH input is a UE transmission synthesised before the timed region with
the same TX chain through a fixed 4x2 MIMO channel plus AWGN (35 dB SNR); the
bench reports the fraction of decoded transport blocks whose TB CRC passes and
which equal the transmitted bits (the chain is checked end to end on every run).
A step processes every slot of the batch through both chains; `value` counts
the codeblocks encoded (PDSCH) plus decoded (PUSCH) per second.
"""
import time

import numpy as np

NPRB, NSUBC, MU, NFFT = 273, 273 * 12, 1, 4096
QM, RATE = 8, 948.0  # 256QAM, target code rate x 1024 (MCS 27 of the 256QAM table)
DL_LAYERS, DL_PORTS = 4, 4
UL_LAYERS, UL_PORTS = 2, 4
DMRS_MASK = (1 << 2) | (1 << 11)
DL_START, DL_NSYM = 1, 13
UL_START, UL_NSYM = 0, 14
RNTI, N_ID, SLOT = 0x4601, 500, 0
SNR_DB = 35.0
UL_LANES = 1  # PUSCH streams (cell shares) next to the PDSCH stream; 2 measured 10% slower (smaller kernels contend)


def base_graph(tbs, r):
    """TS 38.212 7.2.2 base-graph selection."""
    if tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25:
        return 2
    return 1


def _dl_weights():
    k = np.arange(DL_PORTS)
    return (np.exp(-2j * np.pi * np.outer(np.arange(DL_LAYERS), k) / DL_PORTS) / 2.0).astype(np.complex64)


def _ul_channel():
    # [layer][rx port]: the 4x2 channel the UE transmission goes through
    h = np.array([[1.0, 0.2j, 0.7 + 0.1j, 0.3], [0.1, 0.9, -0.2j, 0.8 - 0.2j]], np.complex64)
    return h * np.float32(0.8)


class Pipeline:
    def __init__(self, slots, dev, iters=6):
        import torch

        import srsran_project_amd as amd

        self.torch, self.dev, self.S = torch, dev, slots
        self.ul_stream = None
        d = dev.index
        all_crbs = list(range(NPRB))
        # ---- plans -------------------------------------------------------------------------
        self.tbs_dl = amd.tbs_calculator_calculate(DL_NSYM, 24, 0, QM, RATE, DL_LAYERS, 0, NPRB)
        self.tbs_ul = amd.tbs_calculator_calculate(UL_NSYM, 24, 0, QM, RATE, UL_LAYERS, 0, NPRB)
        nre_dl = NPRB * 12 * (DL_NSYM - 2)
        nre_ul = NPRB * 12 * (UL_NSYM - 2)
        self.plan_dl = amd.sch_plan(self.tbs_dl, base_graph(self.tbs_dl, RATE / 1024), 0, QM, 0, DL_LAYERS,
                                    nre_dl * DL_LAYERS)
        self.plan_ul = amd.sch_plan(self.tbs_ul, base_graph(self.tbs_ul, RATE / 1024), 0, QM, 0, UL_LAYERS,
                                    nre_ul * UL_LAYERS)
        self.enc = amd.PdschEncoder(device=d)
        self.mod = amd.PdschModulator(device=d)
        wdl = _dl_weights()
        self.mod_plan_dl = self.mod.plan(amd.PdschModulatorConfig(
            rnti=RNTI, bwp_start=0, bwp_size=NPRB, modulation=QM, crbs=all_crbs, start_symbol=DL_START,
            nof_symbols=DL_NSYM, dmrs_symb_pos=DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=2, n_id=N_ID,
            precoding=wdl), NSUBC)
        assert self.mod_plan_dl.nof_bits == self.plan_dl.cw_length, (self.mod_plan_dl.nof_bits,
                                                                      self.plan_dl.cw_length)
        self.dmrs_dl = amd.DmrsPdschConfig(slot_index=SLOT, reference_point_k_rb=0, type=1, scrambling_id=N_ID,
                                           n_scid=False, amplitude=1.0, symbols_mask=DMRS_MASK, crbs=all_crbs,
                                           precoding=wdl)
        self.ofdm_mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(MU, NPRB, NFFT, 0, 1.0, 3.5e9),
                                              device=d)
        self.ofdm_dem = amd.OfdmSlotDemodulator(
            amd.OfdmDemodulatorConfiguration(MU, NPRB, NFFT, 0, 1.0, 3.5e9, 0), device=d)
        self.chest = amd.DmrsPuschEstimator(device=d)
        self.chest_cfg = amd.DmrsPuschEstimatorConfig(
            slot_index=SLOT, numerology=MU, nof_tx_layers=UL_LAYERS, scrambling_id=N_ID, n_scid=False, scaling=1.0,
            symbols_mask=DMRS_MASK, rb_start=0, rb_count=NPRB, first_symbol=UL_START, nof_symbols=UL_NSYM)
        self.demod = amd.PuschDemodulator(device=d)
        self.demod_cfg = amd.PuschDemodulatorConfig(
            rnti=RNTI, crbs=all_crbs, modulation=QM, start_symbol=UL_START, nof_symbols=UL_NSYM,
            dmrs_symb_pos=DMRS_MASK, n_id=N_ID, nof_tx_layers=UL_LAYERS, nof_rx_ports=UL_PORTS,
            nof_cdm_groups_without_data=2)
        self.demod_plan = self.demod.plan(self.demod_cfg, NSUBC)
        assert self.demod_plan.nof_llrs == self.plan_ul.cw_length
        self.dec = amd.PuschDecoder("simd", device=d)
        self.dec_cfg = amd.PuschDecoder.config(nof_ldpc_iterations=iters, use_early_stop=True)
        # PUSCH lanes: the cells are split into UL_LANES contiguous shares, each run by its own processor
        # objects on its own stream (a multi-cell PHY runs independent cells concurrently)
        self.ul_objs = [(self.ofdm_dem, self.chest, self.demod, self.demod_plan, self.dec)]
        for _ in range(1, UL_LANES):
            dem = amd.PuschDemodulator(device=d)
            self.ul_objs.append((amd.OfdmSlotDemodulator(amd.OfdmDemodulatorConfiguration(MU, NPRB, NFFT, 0, 1.0,
                                                                                          3.5e9, 0), device=d),
                                 amd.DmrsPuschEstimator(device=d), dem, dem.plan(self.demod_cfg, NSUBC),
                                 amd.PuschDecoder("simd", device=d)))
        self.ul_bounds = [slots * k // UL_LANES for k in range(UL_LANES + 1)]
        self.res_ul = [None] * UL_LANES

        # ---- resident inputs and buffers --------------------------------------------------------
        S = slots
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + d)
        self.tb_dl = torch.randint(0, 256, (S, self.tbs_dl // 8), device=dev, dtype=torch.uint8, generator=g)
        self.tb_ul = torch.randint(0, 256, (S, self.tbs_ul // 8), device=dev, dtype=torch.uint8, generator=g)
        self.cw_dl = torch.empty((S, (self.plan_dl.cw_length + 7) // 8), dtype=torch.uint8, device=dev)
        self.grid_dl = torch.zeros((S, DL_PORTS, 14, NSUBC), dtype=torch.int32, device=dev)
        stride = self.ofdm_mod.max_slot_size()
        self.samp_dl = torch.empty((S, DL_PORTS, stride), dtype=torch.complex64, device=dev)
        self.grid_ul = torch.zeros((S, UL_PORTS, 14, NSUBC), dtype=torch.int32, device=dev)
        self.est_ul = torch.zeros((S, UL_PORTS, UL_LAYERS, 14, NSUBC), dtype=torch.int32, device=dev)
        self.stats_ul = torch.zeros((S, UL_PORTS, 6), dtype=torch.float32, device=dev)
        self.llr_ul = torch.empty((S, self.plan_ul.cw_length), dtype=torch.int8, device=dev)
        self.tb_rx = torch.zeros((S, self.tbs_ul // 8), dtype=torch.uint8, device=dev)
        self.soft_bytes = amd.soft_buffer_size(self.plan_ul)  # per TB: C rows [LLRs | message | CRC flag]
        self.soft = torch.zeros((S, self.soft_bytes), dtype=torch.int8, device=dev)
        self.samp_ul = self._ue_transmission(amd, g)

    def _ue_transmission(self, amd, g):
        """UE PUSCH TX (2 layers) through a 4x2 channel + AWGN, untimed."""
        torch, dev, S = self.torch, self.dev, self.S
        h = _ul_channel()
        ue_mod_plan = self.mod.plan(amd.PdschModulatorConfig(
            rnti=RNTI, bwp_start=0, bwp_size=NPRB, modulation=QM, crbs=list(range(NPRB)), start_symbol=UL_START,
            nof_symbols=UL_NSYM, dmrs_symb_pos=DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=2, n_id=N_ID,
            precoding=h), NSUBC)
        assert ue_mod_plan.nof_bits == self.plan_ul.cw_length
        cw = self.enc.encode_batch(self.tb_ul, self.plan_ul)
        grid = torch.zeros((S, UL_PORTS, 14, NSUBC), dtype=torch.int32, device=dev)
        self.mod.modulate_batch(grid, cw, ue_mod_plan)
        self.mod.map_dmrs_batch(grid, amd.DmrsPdschConfig(
            slot_index=SLOT, reference_point_k_rb=0, type=1, scrambling_id=N_ID, n_scid=False, amplitude=1.0,
            symbols_mask=DMRS_MASK, crbs=list(range(NPRB)), precoding=h))
        samp = self.ofdm_mod.modulate_batch(grid.view(torch.int16).view(S, UL_PORTS, 14, 2 * NSUBC), SLOT)
        # AWGN at SNR_DB relative to the mean sample power
        p = float(torch.mean(torch.abs(samp) ** 2).item())
        sigma = np.sqrt(p / 10 ** (SNR_DB / 10) / 2)
        noise = torch.complex(torch.randn(samp.shape, device=dev, generator=g),
                              torch.randn(samp.shape, device=dev, generator=g)) * sigma
        out = (samp + noise.to(torch.complex64)).contiguous()
        torch.cuda.synchronize(dev)
        return out

    # ---- the two chains ------------------------------------------------------------------------
    def pdsch(self, stream):
        t = self.torch
        self.enc.encode_batch(self.tb_dl, self.plan_dl, out=self.cw_dl, stream=stream)
        self.mod.modulate_batch(self.grid_dl, self.cw_dl, self.mod_plan_dl, stream=stream)
        self.mod.map_dmrs_batch(self.grid_dl, self.dmrs_dl, stream=stream)
        self.ofdm_mod.modulate_batch(self.grid_dl.view(t.int16).view(self.S, DL_PORTS, 14, 2 * NSUBC), SLOT,
                                     out=self.samp_dl, stream=stream)

    def pusch(self, stream, lane=0):
        """The PUSCH chain of the cells of one lane (a contiguous share of the batch), with that lane's
        own processor objects (each keeps its own device scratch)."""
        t = self.torch
        ofdm_dem, chest, demod, demod_plan, dec = self.ul_objs[lane]
        a, b = self.ul_bounds[lane], self.ul_bounds[lane + 1]
        n = b - a
        grid = self.grid_ul[a:b]
        ofdm_dem.demodulate_batch(self.samp_ul[a:b], SLOT, grid=grid.view(t.int16).view(n, UL_PORTS, 14, 2 * NSUBC),
                                  stream=stream)
        chest.estimate_batch(grid, self.chest_cfg, self.est_ul[a:b], self.stats_ul[a:b], stream=stream)
        demod.demodulate_batch(grid, self.est_ul[a:b], self.stats_ul[a:b], demod_plan, llrs=self.llr_ul[a:b],
                               stream=stream)
        _, self.res_ul[lane] = dec.decode_batch(self.llr_ul[a:b], self.plan_ul, self.dec_cfg, tbs=self.tb_rx[a:b],
                                                soft=self.soft[a:b], stream=stream)

    def step(self, stream):
        """One slot of every cell through both chains. The PDSCH (TX) and PUSCH (RX) chains share no data,
        so they run concurrently on two HIP streams (fork / join with events on `stream`): their small
        per-TB kernels fill each other's idle CUs."""
        t = self.torch
        if self.ul_stream is None:
            self.ul_stream = [t.cuda.Stream(self.dev) for _ in range(UL_LANES)]
            self.ev_fork = t.cuda.Event()
            self.ev_join = [t.cuda.Event() for _ in range(UL_LANES)]
        self.ev_fork.record(stream)
        for st in self.ul_stream:
            st.wait_event(self.ev_fork)
        with t.cuda.stream(stream):
            self.pdsch(stream)
        for k, st in enumerate(self.ul_stream):
            with t.cuda.stream(st):
                self.pusch(st, k)
            self.ev_join[k].record(st)
        for ev in self.ev_join:
            stream.wait_event(ev)

    def check(self):
        """Fraction of PUSCH transport blocks with TB CRC ok and bit-equal to what the UE sent."""
        res = self.torch.cat(self.res_ul).cpu().numpy()
        crc_ok = res[:, 0] != 0
        same = (self.tb_rx.cpu().numpy() == self.tb_ul.cpu().numpy()).all(axis=1)
        return float(np.mean(crc_ok & same)), res

    def ldpc_decoder_ms(self, stream, reps=5):
        """The PUSCH chain's dominant kernel alone: ldpc_decode_kernel over this step's rate-dematched soft
        buffers (same configuration, CRC24B early stop), HIP events on the launch stream."""
        import srsran_project_amd as amd

        t = self.torch
        p = self.plan_ul
        C = p.nof_segments
        row = self.soft_bytes // C
        n_llr = amd.codeblock_length(p.base_graph, p.lifting_size)
        rows = self.soft.view(-1).as_strided((self.S * C, n_llr), (row, 1))
        dec = amd.LdpcDecoder("simd", device=self.dev.index)
        cfg = amd.LdpcDecoderConfiguration(base_graph=p.base_graph, lifting_size=p.lifting_size,
                                           nof_filler_bits=p.nof_filler_bits, nof_crc_bits=24,
                                           max_iterations=6)
        dec.decode_batch(rows, cfg, amd.CrcGeneratorPoly.CRC24B, stream=stream)
        e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            dec.decode_batch(rows, cfg, amd.CrcGeneratorPoly.CRC24B, stream=stream)
        e1.record(stream)
        t.cuda.synchronize(self.dev)
        # algorithmic bytes: every CB reads its soft-buffer row (the decoder trims at the last non-zero
        # LLR) and writes its message + iteration count
        return e0.elapsed_time(e1) / reps, self.S * C * (n_llr + (amd.message_length(p.base_graph, p.lifting_size)
                                                                   + 7) // 8 + 4)

    def stage_ms(self, stream, reps=3):
        """Per-stage device time (HIP events on the launch stream), averaged over reps."""
        t = self.torch
        names = ["pdsch_encode", "pdsch_modulate", "dmrs_pdsch", "ofdm_modulate", "ofdm_demodulate",
                 "pusch_chest", "pusch_demodulate", "pusch_decode"]
        acc = np.zeros(len(names))
        for _ in range(reps):
            ev = [t.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
            ev[0].record(stream)
            self.enc.encode_batch(self.tb_dl, self.plan_dl, out=self.cw_dl, stream=stream)
            ev[1].record(stream)
            self.mod.modulate_batch(self.grid_dl, self.cw_dl, self.mod_plan_dl, stream=stream)
            ev[2].record(stream)
            self.mod.map_dmrs_batch(self.grid_dl, self.dmrs_dl, stream=stream)
            ev[3].record(stream)
            self.ofdm_mod.modulate_batch(self.grid_dl.view(t.int16).view(self.S, DL_PORTS, 14, 2 * NSUBC), SLOT,
                                         out=self.samp_dl, stream=stream)
            ev[4].record(stream)
            self.ofdm_dem.demodulate_batch(self.samp_ul, SLOT,
                                           grid=self.grid_ul.view(t.int16).view(self.S, UL_PORTS, 14, 2 * NSUBC),
                                           stream=stream)
            ev[5].record(stream)
            self.chest.estimate_batch(self.grid_ul, self.chest_cfg, self.est_ul, self.stats_ul, stream=stream)
            ev[6].record(stream)
            self.demod.demodulate_batch(self.grid_ul, self.est_ul, self.stats_ul, self.demod_plan,
                                        llrs=self.llr_ul, stream=stream)
            ev[7].record(stream)
            self.dec.decode_batch(self.llr_ul, self.plan_ul, self.dec_cfg, tbs=self.tb_rx, soft=self.soft,
                                  stream=stream)
            ev[8].record(stream)
            t.cuda.synchronize(self.dev)
            acc += np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(len(names))])
        return dict(zip(names, (acc / reps).tolist()))


def run_pipeline(args, dist, world, rank, dev, timed, hbm_peak, traffic=None):
    import torch

    stream = torch.cuda.current_stream(dev)
    pl = Pipeline(args.slots_pipeline, dev)
    elapsed, step_ms = timed(args, dist, world, dev, stream, lambda: pl.step(stream))
    ok_frac, res = pl.check()
    stages = pl.stage_ms(stream)
    S = pl.S
    cbs_dl, cbs_ul = pl.plan_dl.nof_segments, pl.plan_ul.nof_segments
    cbs = (cbs_dl + cbs_ul) * S * args.steps * world
    bits = (pl.tbs_dl + pl.tbs_ul) * S * args.steps * world
    value = cbs / elapsed
    dec_ms, dec_bytes = pl.ldpc_decoder_ms(stream)
    # algorithmic HBM bytes of each stage per step (inputs read once, outputs written once)
    samp_dl = S * DL_PORTS * pl.ofdm_mod.get_slot_size(SLOT) * 8
    samp_ul = S * UL_PORTS * pl.ofdm_dem.get_slot_size(SLOT) * 8
    grid_b = lambda ports: S * ports * 14 * NSUBC * 4  # noqa: E731
    alg_bytes = {
        "pdsch_encode": S * (pl.tbs_dl // 8 + (pl.plan_dl.cw_length + 7) // 8),
        "pdsch_modulate": S * ((pl.plan_dl.cw_length + 7) // 8) + grid_b(DL_PORTS) * 11 // 14,
        "dmrs_pdsch": grid_b(DL_PORTS) * 2 // 14,
        "ofdm_modulate": grid_b(DL_PORTS) + samp_dl,
        "ofdm_demodulate": samp_ul + grid_b(UL_PORTS),
        "pusch_chest": grid_b(UL_PORTS) * 2 // 14 + grid_b(UL_PORTS) * UL_LAYERS,
        "pusch_demodulate": grid_b(UL_PORTS) * (1 + UL_LAYERS) + S * pl.plan_ul.cw_length,
        "pusch_decode": S * pl.plan_ul.cw_length + S * pl.tbs_ul // 8,
    }
    gbs = {k: alg_bytes[k] / (stages[k] * 1e-3) / 1e9 for k in stages}
    if rank != 0:
        return None
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = pipeline_cpu_baseline(args, pl)
    return {
        "metric": "PDSCH+PUSCH codeblocks/s @ 100 MHz 273-PRB 4x4 MIMO (PDSCH 4 layers, PUSCH 2 layers x 4 rx)",
        "value": value,
        "unit": "codeblocks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8+fp32",
        "data": "synthetic (random transport blocks; PUSCH from a UE transmission through a 4x2 channel + AWGN "
                "%.0f dB)" % SNR_DB,
        "config": {
            "workload": "configs[3]/headline: full PDSCH+PUSCH slot pipeline, 100 MHz numerology-1 273 PRB, "
                        "256QAM R=948/1024",
            "cells_per_step_per_gpu": S,
            "pdsch": {"layers": DL_LAYERS, "ports": DL_PORTS, "tbs": pl.tbs_dl, "codeblocks": cbs_dl},
            "pusch": {"layers": UL_LAYERS, "rx_ports": UL_PORTS, "tbs": pl.tbs_ul, "codeblocks": cbs_ul,
                      "ldpc_max_iterations": 6, "early_stop": True},
            "parallelism": "cells sharded over ranks" if world > 1 else "single GPU",
        },
        "throughput_gbps": bits / elapsed / 1e9,
        "pusch_tb_ok_fraction": ok_frac,
        # srs_amd_pusch_decoder_result: tb_crc_ok, nof_codeblocks_total, ldpc_iterations_sum / min / max, ...
        "pusch_ldpc_iterations_mean": float(res[:, 2].sum() / max(1, res[:, 1].sum())),
        "stage_ms": stages,
        "stage_gbs": gbs,
        "roofline": {
            "bound": "hbm",
            "kernel": "ldpc_decode_kernel (PUSCH codeblocks of one step, BG%d Z=%d, CRC24B early stop, <= 6 it)"
                      % (pl.plan_ul.base_graph, pl.plan_ul.lifting_size),
            "achieved": dec_bytes / (dec_ms * 1e-3) / 1e9,
            "peak": hbm_peak,
            "unit": "GB/s",
            "frac": dec_bytes / (dec_ms * 1e-3) / 1e9 / hbm_peak,
            "traffic": traffic,
            "kernel_ms": dec_ms,
            "algorithmic_bytes_per_launch": dec_bytes,
            "note": "the LDPC decoder is VALU/LDS-latency bound (layered min-sum), the HBM fraction is low by "
                    "nature; per-stage algorithmic GB/s in stage_gbs",
        },
        "cpu_baseline": cpu,
    }


def pipeline_cpu_baseline(args, pl):
    """The reference's own CPU chain (oracle/_ref) per cell-slot: pdsch_encoder_impl, pdsch_modulator_impl +
    dmrs_pdsch_processor_impl, OFDM modulator / demodulator (generic DFT), dmrs_pusch_estimator_impl,
    channel_equalizer_generic_impl + demodulation mapper + descrambling, pusch_decoder_impl (AVX512/AVX2 LDPC).
    Timed single-threaded and on `--cpu-threads` threads (one chain per thread; ctypes releases the GIL),
    cycling over the same slot inputs, for a bounded sample of about `--cpu-seconds`."""
    try:
        import oracle
        from oracle import chest as och
        from oracle import pdsch_mod as opm
        from oracle import sch as osch
        from oracle.pusch_demod import data_re_mask
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "codeblocks/s", "error": "oracle unavailable: %s" % e}
    if oracle.REF is None:
        return {"value": None, "unit": "codeblocks/s", "error": "oracle/_ref not built"}
    from concurrent.futures import ThreadPoolExecutor

    tb = pl.tb_dl[0].cpu().numpy()
    samp = pl.samp_ul[0].cpu().numpy()
    p_dl = osch.plan(pl.tbs_dl, pl.plan_dl.base_graph, 0, QM, 0, DL_LAYERS, pl.plan_dl.nof_ch_symbols)
    p_ul = osch.plan(pl.tbs_ul, pl.plan_ul.base_graph, 0, QM, 0, UL_LAYERS, pl.plan_ul.nof_ch_symbols)
    mask = data_re_mask(NSUBC, range(NPRB), UL_START, UL_NSYM, DMRS_MASK, False, 2)
    ls, ks = np.nonzero(mask)
    wdl = _dl_weights()
    c_ul = oracle.prbs(RNTI * (1 << 15) + N_ID, pl.plan_ul.cw_length)

    def one_slot():
        t = {}
        t0 = time.perf_counter()
        cw = oracle.ref_pdsch_encode(tb, p_dl)
        t1 = time.perf_counter()
        grid = np.zeros((DL_PORTS, 14, NSUBC, 2), np.uint16)
        opm.ref_pdsch_modulate(grid, cw, RNTI, N_ID, QM, np.arange(NPRB), DL_START, DL_NSYM, DMRS_MASK, False, 2,
                               [], wdl, 1.0, bwp=(0, NPRB))
        opm.ref_dmrs_pdsch_map(grid, SLOT, 0, False, N_ID, 0, 1.0, DMRS_MASK, np.arange(NPRB), wdl[None],
                               numerology=MU)
        t2 = time.perf_counter()
        for p in range(DL_PORTS):
            oracle.ref_ofdm_modulate_slot(grid[p].reshape(14, 2 * NSUBC), SLOT, MU, NPRB, NFFT, 1.0, 3.5e9)
        t3 = time.perf_counter()
        g_ul = np.stack([oracle.ref_ofdm_demodulate_slot(samp[p], SLOT, MU, NPRB, NFFT, 1.0, 3.5e9)
                         for p in range(UL_PORTS)])
        t4 = time.perf_counter()
        g32 = np.ascontiguousarray(g_ul.reshape(UL_PORTS, 14, 2 * NSUBC)).view(np.uint32)
        est, st = och.ref_pusch_chest(g32, SLOT, False, UL_LAYERS, N_ID, 0, 1.0, DMRS_MASK, 0, NPRB, UL_START,
                                      UL_NSYM, fd=2, td=1, compensate_cfo=True, numerology=MU)
        t5 = time.perf_counter()
        sym = np.ascontiguousarray(g32[:, ls, ks]).view(np.uint16)
        e16 = np.ascontiguousarray(np.transpose(est[:, :, ls, ks], (1, 0, 2))).view(np.uint16)
        nv = np.array([x["noise_var"] for x in st], np.float32)
        eq, eqv = oracle.ref_equalize(sym, e16, nv, 1.0, UL_LAYERS)
        llr = oracle.ref_demodulate(eq.reshape(-1).astype(np.complex64), eqv.reshape(-1).astype(np.float32), QM)
        llr = np.where(c_ul == 1, -llr.astype(np.int16), llr.astype(np.int16)).astype(np.int8)
        t6 = time.perf_counter()
        rxbuf = oracle.RefRxBuffer(p_ul["nof_segments"])
        tb_out = np.zeros(pl.tbs_ul // 8, np.uint8)
        ok = oracle.ref_pusch_decode(llr, p_ul, rxbuf, tb_out, max_iterations=6)
        t7 = time.perf_counter()
        t = {"pdsch_encode": t1 - t0, "pdsch_modulate+dmrs": t2 - t1, "ofdm_modulate": t3 - t2,
             "ofdm_demodulate": t4 - t3, "pusch_chest": t5 - t4, "pusch_demodulate": t6 - t5,
             "pusch_decode": t7 - t6}
        return t, bool(ok[0])

    cbs = pl.plan_dl.nof_segments + pl.plan_ul.nof_segments
    # single thread: stage breakdown
    stage = None
    n1, t_start = 0, time.perf_counter()
    ok_all = True
    while n1 < 2 or time.perf_counter() - t_start < max(1.0, args.cpu_seconds / 4):
        st, ok = one_slot()
        ok_all &= ok
        stage = st if stage is None else {k: stage[k] + st[k] for k in st}
        n1 += 1
    t_single = time.perf_counter() - t_start
    # all threads
    threads = max(1, args.cpu_threads)
    per_slot = t_single / n1
    nmt = max(threads, int(args.cpu_seconds * threads / per_slot / 2))
    t_start = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as ex:
        res = list(ex.map(lambda _: one_slot()[1], range(nmt)))
    t_multi = time.perf_counter() - t_start
    ok_all &= all(res)
    return {"value": nmt * cbs / t_multi, "unit": "codeblocks/s", "cores": threads, "kind": "reference",
            "single_thread_value": n1 * cbs / t_single,
            "sample": "%d cell-slots on %d threads (%.1f s) and %d on one thread (%.1f s), cycling over one slot's "
                      "inputs, through the reference's own CPU chain compiled from /root/reference (oracle/_ref): "
                      "pdsch_encoder_impl, pdsch_modulator_impl, dmrs_pdsch_processor_impl, OFDM modulator/"
                      "demodulator with the generic DFT (FFTW absent), dmrs_pusch_estimator_impl, "
                      "channel_equalizer_generic_impl, demodulation mapper, pusch_decoder_impl (AVX512 LDPC when "
                      "the host has it); PUSCH TB CRC %s" % (nmt, threads, t_multi, n1, t_single,
                                                            "ok" if ok_all else "FAILED"),
            "stage_s_per_slot": {k: v / n1 for k, v in stage.items()}}

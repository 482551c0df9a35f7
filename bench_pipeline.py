"""bench_pipeline.py -- the `--workload pipeline` leg of bench.py: the full
PDSCH + PUSCH slot chain of one 100 MHz cell per slot (BASELINE.json metric
"PDSCH+PUSCH codeblocks/s (and Gb/s) @ 100 MHz 273-PRB 4x4 MIMO").

Per slot (= one cell; `--slots-pipeline` cells per step and rank, all resident in HBM):
  PDSCH  (gNB TX, 4 layers x 4 ports, 256QAM R = 948/1024, 273 PRB, symbols 1-13)
         transport block -> pdsch_encoder (CRC, segmentation, LDPC, rate matching)
         -> pdsch_modulator (scrambling, modulation, layer mapping, precoding, RE mapping)
         -> dmrs_pdsch_processor (DM-RS +3 dB, 2 CDM groups without data) -> OFDM modulator.
  PUSCH  (gNB RX, UL_LAYERS layers x 4 rx ports, 256QAM R = 948/1024, 273 PRB, symbols 0-13; 4 layers with the
         MMSE 4 x 4 solve by default -- the open reference's equalizer asserts for 4 layers, so that stage is
         parity unpinned; --ul-layers 2 runs the reference-pinned ZF 2 x 4 chain)
         baseband -> OFDM demodulator -> pusch_processor (the C-ABI PUSCH processor:
         DM-RS estimator -> demodulator -> UL-SCH decoder with CRC early stop), configured as
         the reference pusch_processor_impl (DM-RS scaling from the CDM groups, Nref from
         tbs_lbrm_default, ZF, filter FD smoothing, average TD strategy (the reference app's default), CFO
         compensation).
The PUSCH input is a UE transmission synthesised before the timed region through a
fixed UL_LAYERS x 4 MIMO channel plus AWGN; every run checks the decoded TBs against
what the UE sent. A step processes every slot of the batch through both chains;
`value` counts the codeblocks encoded (PDSCH) plus decoded (PUSCH) per second.

Multi-GPU (one process per GPU): each rank runs its own cells (weak scaling, no
data-path collective). With `--ingest`, rank 0 also holds the slot inputs of all
cells and fans them out / gathers the decoded TBs over RCCL every step
(srsran_project_amd/cell_fanout.py); that time is reported separately.
"""
import os
import sys
import time

import numpy as np

NPRB, NSUBC, MU, NFFT = 273, 273 * 12, 1, 4096
QM, RATE = 8, 948.0  # 256QAM, target code rate x 1024 (MCS 27 of the 256QAM table)
DL_LAYERS, DL_PORTS = 4, 4
UL_LAYERS, UL_PORTS, UL_EQ = 4, 4, "mmse"
DMRS_MASK = (1 << 2) | (1 << 11)
NCDM = 2
DL_START, DL_NSYM = 1, 13
UL_START, UL_NSYM = 0, 14
RNTI, N_ID, SLOT = 0x4601, 500, 0
SNR_DB = 35.0
# DM-RS estimator time-domain strategy: average over the DM-RS symbols, the reference application's default
# (du_low_config.h:68 pusch_channel_estimator_td_strategy = "average" -> upper_phy_factories.cpp:596-600);
# --chest-td interpolate selects the per-symbol estimates with linear interpolation in time
UL_TD = {"interpolate": 0, "average": 1}
# near the decoding threshold (tools/snr_sweep.py, mean LDPC iterations ~4): per PUSCH layer count
LOW_SNR_DB = {(2, 4): 23.8, (4, 4): 32.0}  # (PUSCH layers, rx ports)
LDPC_ITERS = 6
# DM-RS amplitude relative to data: convert_dB_to_amplitude(-get_sch_to_dmrs_ratio_dB(2)) = 10^(3/20),
# evaluated in float as the reference (sch_dmrs_power.h, math_utils.h:118)
DMRS_AMP = float(np.power(np.float32(10.0), np.float32(3.0) / np.float32(20.0)))


def base_graph(tbs, r):
    """TS 38.212 7.2.2 base-graph selection (get_ldpc_base_graph)."""
    if tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25:
        return 2
    return 1


# MIMO shapes of the pipeline: "4x4" (the BASELINE.json headline: PDSCH 4 layers x 4 ports, PUSCH 4 layers x 4 rx
# ports) and "2x2" (configs[3]: PDSCH 2 layers x 2 ports, PUSCH 2 layers x 2 rx ports)
MIMO = {"4x4": (4, 4, 4, 4), "2x2": (2, 2, 2, 2)}  # dl layers, dl ports, ul layers, ul rx ports


def shape_kw(args):
    """Pipeline keyword arguments of bench.py's --mimo / --ul-layers."""
    dl_l, dl_p, ul_l, ul_p = MIMO[getattr(args, "mimo", "4x4")]
    if getattr(args, "mimo", "4x4") == "4x4":
        ul_l = args.ul_layers
    return dict(dl_layers=dl_l, dl_ports=dl_p, ul_layers=ul_l, ul_ports=ul_p,
                ul_td=getattr(args, "chest_td", "average"))


def dl_weights(layers=DL_LAYERS, ports=DL_PORTS):
    """[layer][port] DFT precoder, unit power per layer."""
    k = np.arange(ports)
    return (np.exp(-2j * np.pi * np.outer(np.arange(layers), k) / ports) /
            np.sqrt(np.float32(ports))).astype(np.complex64)


def ul_channel(layers, ports=UL_PORTS):
    """[layer][rx port]: the MIMO channel the UE transmission goes through."""
    h = np.array([[1.0, 0.2j, 0.7 + 0.1j, 0.3],
                  [0.1, 0.9, -0.2j, 0.8 - 0.2j],
                  [0.3j, -0.2, 0.9, 0.1 + 0.2j],
                  [0.2, 0.1 - 0.3j, 0.2, 0.9]], np.complex64)
    return h[:layers, :ports] * np.float32(0.8)


def ul_tbs(amd, layers):
    ndmrs = 6 * bin(DMRS_MASK).count("1") * NCDM  # dmrs.nof_dmrs_per_rb() x symbols x CDM groups
    return amd.tbs_calculator_calculate(UL_NSYM, ndmrs, 0, QM, RATE, layers, 0, NPRB)


def ul_pdu(amd, layers, tbs, ports=UL_PORTS):
    return amd.make_pdu(numerology=MU, slot_index=SLOT, rnti=RNTI, bwp_start_rb=0, bwp_size_rb=NPRB, modulation=QM,
                        target_code_rate=RATE, rv=0, base_graph=base_graph(tbs, RATE / 1024), new_data=1, n_id=N_ID,
                        nof_tx_layers=layers, nof_rx_ports=ports, dmrs_symbol_mask=DMRS_MASK, scrambling_id=N_ID,
                        n_scid=0, nof_cdm_groups_without_data=NCDM, rb_start=0, rb_count=NPRB,
                        start_symbol_index=UL_START, nof_symbols=UL_NSYM, tbs=tbs)


def chain_streams(torch, dev):
    """The two streams of a step's PDSCH and PUSCH chains: two consecutive torch pool streams.  HIP maps streams
    onto GPU_MAX_HW_QUEUES (4 on the box) hardware queues round-robin, so two streams created one after the other
    never share a queue, while the caller's stream and a pool stream can -- and then the chains run one after the
    other (tools/overlap_probe.py: 64-cell slot step 1.45 ms serialized, 1.23-1.26 ms overlapped; a high-priority
    PUSCH stream measured 2.7 ms)."""
    return torch.cuda.Stream(dev), torch.cuda.Stream(dev)


class Pipeline:
    def __init__(self, slots, dev, iters=LDPC_ITERS, snr_db=SNR_DB, ul_layers=UL_LAYERS, seed=0, ul_equalizer=None,
                 keep_estimates=False, dl_layers=DL_LAYERS, dl_ports=DL_PORTS, ul_ports=UL_PORTS, ul_td="average"):
        import torch

        import srsran_project_amd as amd

        self.torch, self.dev, self.S = torch, dev, slots
        self.ul_layers, self.snr_db, self.iters = ul_layers, snr_db, iters
        self.dl_layers, self.dl_ports, self.ul_ports = dl_layers, dl_ports, ul_ports
        assert dl_layers <= dl_ports and ul_layers <= ul_ports
        # the reference-pinned ZF for two layers, MMSE (parity unpinned) for four unless asked otherwise
        self.ul_equalizer = ul_equalizer or ("zf" if ul_layers <= 2 else UL_EQ)
        self.ul_td = UL_TD[ul_td]
        self.ul_stream = None
        self._capturing = False
        d = dev.index
        all_crbs = list(range(NPRB))
        # ---- plans -------------------------------------------------------------------------
        self.tbs_dl = amd.tbs_calculator_calculate(DL_NSYM, 24, 0, QM, RATE, dl_layers, 0, NPRB)
        self.tbs_ul = ul_tbs(amd, ul_layers)
        nre_dl = NPRB * 12 * (DL_NSYM - 2)
        self.plan_dl = amd.sch_plan(self.tbs_dl, base_graph(self.tbs_dl, RATE / 1024), 0, QM, 0, dl_layers,
                                    nre_dl * dl_layers)
        self.enc = amd.PdschEncoder(device=d)
        self.mod = amd.PdschModulator(device=d)
        wdl = dl_weights(dl_layers, dl_ports)
        self.mod_plan_dl = self.mod.plan(amd.PdschModulatorConfig(
            rnti=RNTI, bwp_start=0, bwp_size=NPRB, modulation=QM, crbs=all_crbs, start_symbol=DL_START,
            nof_symbols=DL_NSYM, dmrs_symb_pos=DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=NCDM, n_id=N_ID,
            precoding=wdl), NSUBC)
        assert self.mod_plan_dl.nof_bits == self.plan_dl.cw_length, (self.mod_plan_dl.nof_bits,
                                                                      self.plan_dl.cw_length)
        self.dmrs_dl = amd.DmrsPdschConfig(slot_index=SLOT, reference_point_k_rb=0, type=1, scrambling_id=N_ID,
                                           n_scid=False, amplitude=DMRS_AMP, symbols_mask=DMRS_MASK, crbs=all_crbs,
                                           precoding=wdl)
        self.ofdm_mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(MU, NPRB, NFFT, 0, 1.0, 3.5e9),
                                              device=d)
        self.ofdm_dem = amd.OfdmSlotDemodulator(
            amd.OfdmDemodulatorConfiguration(MU, NPRB, NFFT, 0, 1.0, 3.5e9, 0), device=d)
        self.proc = amd.PuschProcessor(amd.PuschProcessorConfig(
            dec_nof_iterations=iters, dec_enable_early_stop=True, fd_smoothing=2, td_interpolation=self.ul_td,
            compensate_cfo=True, equalizer=int(getattr(amd.ChannelEqualizerAlgorithmType, self.ul_equalizer))),
            device=d)
        self.pdu_ul = ul_pdu(amd, ul_layers, self.tbs_ul, ul_ports)
        self.proc_plan = self.proc.plan(self.pdu_ul, NSUBC)
        self.plan_ul = self.proc_plan.sch  # the processor's UL-SCH plan (Nref from tbs_lbrm_default)

        # ---- resident inputs and buffers --------------------------------------------------------
        S = slots
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + d + 7919 * seed)
        self.tb_dl = torch.randint(0, 256, (S, self.tbs_dl // 8), device=dev, dtype=torch.uint8, generator=g)
        self.tb_ul = torch.randint(0, 256, (S, self.tbs_ul // 8), device=dev, dtype=torch.uint8, generator=g)
        self.cw_dl = torch.empty((S, (self.plan_dl.cw_length + 7) // 8), dtype=torch.uint8, device=dev)
        self.grid_dl = torch.zeros((S, dl_ports, 14, NSUBC), dtype=torch.int32, device=dev)
        stride = self.ofdm_mod.max_slot_size()
        self.samp_dl = torch.empty((S, dl_ports, stride), dtype=torch.complex64, device=dev)
        self.grid_ul = torch.zeros((S, ul_ports, 14, NSUBC), dtype=torch.int32, device=dev)
        # keep_estimates: the processor also writes the expanded channel estimates (tests check them); without
        # it the equalizer rebuilds them per RE from the estimator's per-subcarrier output (no HBM tensor)
        self.est_ul = (torch.zeros((S, ul_ports, ul_layers, 14, NSUBC), dtype=torch.int32, device=dev)
                       if keep_estimates else None)
        self.stats_ul = torch.zeros((S, ul_ports, 6), dtype=torch.float32, device=dev)
        self.llr_ul = torch.empty((S, (self.plan_ul.cw_length + 63) // 64 * 64), dtype=torch.int8, device=dev)
        self.tb_rx = torch.zeros((S, self.tbs_ul // 8), dtype=torch.uint8, device=dev)
        self.res_ul = torch.zeros((S, amd.pusch_processor.RESULT_BYTES), dtype=torch.uint8, device=dev)
        self.samp_ul = self._ue_transmission(amd, g)

    def _ue_transmission(self, amd, g):
        """UE PUSCH TX (ul_layers) through a ul_layers x 4 channel + AWGN, untimed. The UL-SCH coding, scrambling,
        modulation and type-1 DM-RS use the same TS 38.211 / 38.212 chains as the PDSCH TX kernels; DM-RS at the
        amplitude the processor's estimator expects (DMRS_AMP)."""
        torch, dev, S = self.torch, self.dev, self.S
        h = ul_channel(self.ul_layers, self.ul_ports)
        ue_mod_plan = self.mod.plan(amd.PdschModulatorConfig(
            rnti=RNTI, bwp_start=0, bwp_size=NPRB, modulation=QM, crbs=list(range(NPRB)), start_symbol=UL_START,
            nof_symbols=UL_NSYM, dmrs_symb_pos=DMRS_MASK, dmrs_type=1, nof_cdm_groups_without_data=NCDM, n_id=N_ID,
            precoding=h), NSUBC)
        assert ue_mod_plan.nof_bits == self.plan_ul.cw_length
        cw = self.enc.encode_batch(self.tb_ul, self.plan_ul)
        grid = torch.zeros((S, self.ul_ports, 14, NSUBC), dtype=torch.int32, device=dev)
        self.mod.modulate_batch(grid, cw, ue_mod_plan)
        self.mod.map_dmrs_batch(grid, amd.DmrsPdschConfig(
            slot_index=SLOT, reference_point_k_rb=0, type=1, scrambling_id=N_ID, n_scid=False, amplitude=DMRS_AMP,
            symbols_mask=DMRS_MASK, crbs=list(range(NPRB)), precoding=h))
        samp = self.ofdm_mod.modulate_batch(grid.view(torch.int16).view(S, self.ul_ports, 14, 2 * NSUBC), SLOT)
        # AWGN at snr_db relative to the mean sample power
        p = float(torch.mean(torch.abs(samp) ** 2).item())
        sigma = np.sqrt(p / 10 ** (self.snr_db / 10) / 2)
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
        self.ofdm_mod.modulate_batch(self.grid_dl.view(t.int16).view(self.S, self.dl_ports, 14, 2 * NSUBC), SLOT,
                                     out=self.samp_dl, stream=stream)

    def pusch(self, stream):
        t = self.torch
        self.ofdm_dem.demodulate_batch(self.samp_ul, SLOT,
                                       grid=self.grid_ul.view(t.int16).view(self.S, self.ul_ports, 14, 2 * NSUBC),
                                       stream=stream)
        self.proc.process_batch(self.grid_ul, self.proc_plan, tbs=self.tb_rx, results=self.res_ul,
                                port_stats=self.stats_ul, estimates=self.est_ul, llrs=self.llr_ul, stream=stream)

    def step(self, stream):
        """One slot of every cell through both chains. The PDSCH (TX) and PUSCH (RX) chains share no data,
        so they run concurrently on two HIP streams (fork / join with events on `stream`): their small
        per-TB kernels fill each other's idle CUs."""
        t = self.torch
        if self.ul_stream is None:
            self.dl_stream, self.ul_stream = chain_streams(t, self.dev)
            self.ev_fork = t.cuda.Event()
            self.ev_join = [t.cuda.Event(), t.cuda.Event()]
        # under HIP-graph capture the PDSCH chain stays on the capturing stream (a capture whose origin stream holds
        # only the fork / join events crashed the capture); the replayed graph's placement is the runtime's
        # (SRSRAN_AMD_GRAPH_FORK=1 captures the forked form anyway: the probe that records the capture's HIP error)
        dl = stream if self._capturing and os.environ.get("SRSRAN_AMD_GRAPH_FORK") != "1" else self.dl_stream
        self.ev_fork.record(stream)
        if dl is not stream:
            dl.wait_event(self.ev_fork)
        self.ul_stream.wait_event(self.ev_fork)
        # the PUSCH chain (the critical path) is enqueued first, so its first kernels get the CUs before the PDSCH
        # chain's: 0.729 vs 0.735 ms per step over three alternating pairs on one box (tools/order_ab.sh,
        # SRSRAN_AMD_UL_FIRST=0 restores the old order); a HIP-graph capture keeps the old order
        if os.environ.get("SRSRAN_AMD_UL_FIRST", "1") == "1" and not self._capturing:
            with t.cuda.stream(self.ul_stream):
                self.pusch(self.ul_stream)
            with t.cuda.stream(dl):
                self.pdsch(dl)
        else:
            with t.cuda.stream(dl):
                self.pdsch(dl)
            with t.cuda.stream(self.ul_stream):
                self.pusch(self.ul_stream)
        if dl is not stream:
            self.ev_join[0].record(dl)
            stream.wait_event(self.ev_join[0])
        self.ev_join[1].record(self.ul_stream)
        stream.wait_event(self.ev_join[1])

    def graph(self, stream):
        """The step (both chains, every C-ABI launch of both streams) captured once as a HIP graph on `stream` (a
        non-default stream) after two warm-up steps, so scratch buffers are sized and the uniform-batch descriptors
        cached: each replay is one graph launch instead of ~20 kernel launches.  Returns the replay callable (it
        launches on `stream`), or None when the capture is refused (the step then runs eagerly)."""
        t = self.torch
        for _ in range(2):
            self.step(stream)
        t.cuda.synchronize(self.dev)
        g = t.cuda.CUDAGraph()
        self._capturing = True
        try:
            with t.cuda.graph(g, stream=stream):
                self.step(stream)
        except Exception as exc:  # noqa: BLE001 -- report and run eagerly
            print("HIP graph capture refused: %s" % exc, file=sys.stderr)
            t.cuda.synchronize(self.dev)
            return None
        finally:
            self._capturing = False
        t.cuda.synchronize(self.dev)
        self._graph = g  # keep the graph (and its captured memory) alive

        def replay():
            with t.cuda.stream(stream):
                g.replay()
        return replay

    def results(self):
        import srsran_project_amd as amd

        return amd.pusch_processor.parse_results(self.res_ul.cpu().numpy())

    def check(self):
        """Fraction of PUSCH transport blocks with TB CRC ok and bit-equal to what the UE sent, and the mean LDPC
        iterations per codeblock."""
        res = self.results()
        crc_ok = np.array([r.data.tb_crc_ok != 0 for r in res])
        same = (self.tb_rx.cpu().numpy() == self.tb_ul.cpu().numpy()).all(axis=1)
        its = sum(r.data.ldpc_iterations_sum for r in res) / max(1, sum(r.data.nof_codeblocks_total for r in res))
        return float(np.mean(crc_ok & same)), float(its)

    def ldpc_decoder_ms(self, stream, reps=5):
        """The PUSCH chain's dominant kernel alone: ldpc_decode_kernel over this step's rate-dematched LLRs
        (same configuration, CRC24B early stop), HIP events on the launch stream."""
        import srsran_project_amd as amd

        t = self.torch
        p = self.plan_ul
        C = p.nof_segments
        n_llr = amd.codeblock_length(p.base_graph, p.lifting_size)
        # soft-buffer rows of one step: rate dematch this step's LLRs into decoder rows once
        dec = amd.PuschDecoder("simd", device=self.dev.index)
        soft_bytes = amd.soft_buffer_size(p)
        soft = t.zeros((self.S, soft_bytes), dtype=t.int8, device=self.dev)
        dec.decode_batch(self.llr_ul, p, amd.PuschDecoder.config(nof_ldpc_iterations=self.iters, use_early_stop=True),
                         tbs=t.zeros_like(self.tb_rx), soft=soft, stream=stream)
        row = soft_bytes // C
        # the LLR prefix the PUSCH decoder hands to the LDPC decoder (the rest of each row is zero)
        n_llr = amd.decoder_llr_prefix(p, new_data=True, fresh=True)
        rows = soft.view(-1).as_strided((self.S * C, n_llr), (row, 1))
        ldpc = amd.LdpcDecoder("simd", device=self.dev.index)
        cfg = amd.LdpcDecoderConfiguration(base_graph=p.base_graph, lifting_size=p.lifting_size,
                                           nof_filler_bits=p.nof_filler_bits, nof_crc_bits=24,
                                           max_iterations=self.iters)
        its = t.empty((self.S * C,), dtype=t.int32, device=self.dev)
        ldpc.decode_batch(rows, cfg, amd.CrcGeneratorPoly.CRC24B, nof_iters=its, stream=stream)
        e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            ldpc.decode_batch(rows, cfg, amd.CrcGeneratorPoly.CRC24B, nof_iters=its, stream=stream)
        e1.record(stream)
        t.cuda.synchronize(self.dev)
        it = its.cpu().numpy()
        # algorithmic bytes: every CB reads the LLR prefix of its soft-buffer row and writes its message +
        # iteration count
        nbytes = self.S * C * (n_llr + (amd.message_length(p.base_graph, p.lifting_size) + 7) // 8 + 4)
        return e0.elapsed_time(e1) / reps, nbytes, self.S * C, float(np.mean(np.where(it < 0, self.iters, it)))

    def stage_ms(self, stream, reps=3):
        """Per-stage device time (HIP events on the launch stream), averaged over reps after one untimed pass (the
        objects last ran on the step's chain streams: the first call on `stream` carries their cross-stream
        ordering wait and is not a stage time).  A spin kernel (~1 ms) queued ahead of the stages lets the host
        enqueue every stage's launches before the GPU reaches them, so an event pair brackets device time only:
        right after a synchronize the GPU would otherwise wait for the host's launch calls inside the first
        stage (the PDSCH encoder measured 0.15-0.18 ms that way, 0.09 ms back to back)."""
        t = self.torch
        names = ["pdsch_encode", "pdsch_modulate", "dmrs_pdsch", "ofdm_modulate", "ofdm_demodulate", "pusch_process"]
        acc = np.zeros(len(names))
        spin = getattr(t.cuda, "_sleep", None)
        for rep in range(reps + 1):
            ev = [t.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
            if spin is not None:
                with t.cuda.stream(stream):
                    spin(2_000_000)
            ev[0].record(stream)
            self.enc.encode_batch(self.tb_dl, self.plan_dl, out=self.cw_dl, stream=stream)
            ev[1].record(stream)
            self.mod.modulate_batch(self.grid_dl, self.cw_dl, self.mod_plan_dl, stream=stream)
            ev[2].record(stream)
            self.mod.map_dmrs_batch(self.grid_dl, self.dmrs_dl, stream=stream)
            ev[3].record(stream)
            self.ofdm_mod.modulate_batch(self.grid_dl.view(t.int16).view(self.S, self.dl_ports, 14, 2 * NSUBC), SLOT,
                                         out=self.samp_dl, stream=stream)
            ev[4].record(stream)
            self.ofdm_dem.demodulate_batch(self.samp_ul, SLOT,
                                           grid=self.grid_ul.view(t.int16).view(self.S, self.ul_ports, 14, 2 * NSUBC),
                                           stream=stream)
            ev[5].record(stream)
            self.proc.process_batch(self.grid_ul, self.proc_plan, tbs=self.tb_rx, results=self.res_ul,
                                    port_stats=self.stats_ul, estimates=self.est_ul, llrs=self.llr_ul, stream=stream)
            ev[6].record(stream)
            t.cuda.synchronize(self.dev)
            if rep > 0:
                acc += np.array([ev[i].elapsed_time(ev[i + 1]) for i in range(len(names))])
        return dict(zip(names, (acc / reps).tolist()))


def chain_config(pl, choice="auto"):
    """oracle/ref_chain.cpp configuration of the same slot (test infrastructure)."""
    from oracle import chain as oc

    return oc.make_config(numerology=MU, slot=SLOT, nof_prb=NPRB, dft_size=NFFT, rnti=RNTI, n_id=N_ID, qm=QM,
                          dmrs_symbol_mask=DMRS_MASK, nof_cdm_groups_without_data=NCDM, dl_layers=pl.dl_layers,
                          dl_ports=pl.dl_ports, dl_start=DL_START, dl_nsym=DL_NSYM, dl_tbs=pl.tbs_dl,
                          dl_bg=pl.plan_dl.base_graph, dl_weights=dl_weights(pl.dl_layers, pl.dl_ports),
                          dl_dmrs_amplitude=DMRS_AMP, ul_layers=pl.ul_layers, ul_ports=pl.ul_ports, ul_start=UL_START, ul_nsym=UL_NSYM,
                          ul_tbs=pl.tbs_ul, ul_bg=pl.plan_ul.base_graph, ul_iterations=pl.iters,
                          ul_target_code_rate=RATE, choice={"generic": 0, "avx2": 1, "auto": 2}[choice],
                          ul_td=pl.ul_td)


def latency_ms(dev, cells, steps=10, warmup=3, graph=False, **shape):
    """Wall time of one step (both chains of `cells` cells) measured step by step (synchronized each step); graph:
    each step a replay of the HIP graph captured once (Pipeline.graph)."""
    import torch

    pl = Pipeline(cells, dev, **shape)
    stream = torch.cuda.Stream(dev) if graph else torch.cuda.current_stream(dev)
    run = pl.graph(stream) if graph else None
    run = run or (lambda: pl.step(stream))
    for _ in range(warmup):
        run()
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def run_pipeline(args, dist, world, rank, dev, timed, hbm_peak, traffic=None):
    import torch

    from srsran_project_amd.cell_fanout import SlotFanout

    stream = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    pl = Pipeline(args.slots_pipeline, dev, snr_db=args.snr_db, **shape_kw(args))
    S = pl.S
    ingest_ms = None
    if args.ingest and world > 1:
        # rank 0 holds every cell's slot inputs; scatter / gather them over RCCL each step
        fan = SlotFanout(dist, world, rank, S * world)
        full_ul = pl.samp_ul.repeat(world, 1, 1) if rank == 0 else None
        full_tb = pl.tb_dl.repeat(world, 1) if rank == 0 else None
        full_rx = torch.empty((S * world,) + tuple(pl.tb_rx.shape[1:]), dtype=pl.tb_rx.dtype,
                              device=dev) if rank == 0 else None
        full_res = torch.empty((S * world,) + tuple(pl.res_ul.shape[1:]), dtype=torch.uint8,
                               device=dev) if rank == 0 else None

        def ingest_step():
            fan.scatter(full_ul, pl.samp_ul)
            fan.scatter(full_tb, pl.tb_dl)
            pl.step(stream)
            fan.gather(pl.tb_rx, full_rx)
            fan.gather(pl.res_ul, full_res)

        elapsed, step_ms = timed(args, dist, world, dev, stream, ingest_step)
        el_compute, _ = timed(args, dist, world, dev, stream, lambda: pl.step(stream))
        ingest_ms = (elapsed - el_compute) / args.steps * 1e3
    else:
        run = None
        if getattr(args, "graph", False) and dev.type == "cuda":
            stream = torch.cuda.Stream(dev)
            run = pl.graph(stream)
        run = run or (lambda: pl.step(stream))
        elapsed, step_ms = timed(args, dist, world, dev, stream, run)
        # the same K steps again with the live kernel probes armed: each probed launch carries timestamped events in
        # its dispatch packet, which costs the step ~4 % (measured, profiles/r05_probe_overhead.json), so the
        # headline value comes from the unprobed pass above and the kernel times from this one
        probes = None
        if dev.type == "cuda" and not getattr(args, "no_probe", False):
            from srsran_project_amd import profiling as prof

            probes = {prof.PROBE_LDPC_HR: None, prof.PROBE_EQUALIZER: None, prof.PROBE_OFDM_DEMOD: None,
                      prof.PROBE_OFDM_MOD: None}
            el_probed, _ = timed(args, dist, world, dev, stream, run, probes=probes)
            probes["probed_ms_per_step"] = el_probed / args.steps * 1e3
    ok_frac, its_mean = pl.check()
    stages = pl.stage_ms(stream)
    cbs_dl, cbs_ul = pl.plan_dl.nof_segments, pl.plan_ul.nof_segments
    cbs = (cbs_dl + cbs_ul) * S * args.steps * world
    bits = (pl.tbs_dl + pl.tbs_ul) * S * args.steps * world
    value = cbs / elapsed
    # the dominant kernel as the timed steps launched it (fused rate dematching: it reads each codeblock's E received
    # LLRs of the codeword, writes its message and iteration count), timed live by the probe on its own stream
    dec_cbs = pl.plan_ul.nof_segments * S
    dec_its = its_mean
    dec_bytes = S * (pl.plan_ul.cw_length + pl.plan_ul.nof_segments *
                     ((__import__("srsran_project_amd").message_length(pl.plan_ul.base_graph, pl.plan_ul.lifting_size)
                       + 7) // 8 + 4))
    in_step = {}
    if probes:
        from srsran_project_amd import profiling as prof

        for k, v in probes.items():
            if isinstance(k, int) and v is not None and v[0]:
                in_step[prof.NAMES[k]] = {"launches": v[0], "mean_ms": v[1], "min_ms": v[2], "max_ms": v[3]}
    hr = probes.get(__import__("srsran_project_amd").profiling.PROBE_LDPC_HR) if probes else None
    dec_ms = hr[1] if hr and hr[0] else None
    alone = None
    if getattr(args, "alone_probe", False) or dec_ms is None:
        a_ms, a_bytes, _, _ = pl.ldpc_decoder_ms(stream)
        alone = {"kernel_ms": a_ms, "algorithmic_bytes": a_bytes,
                 "note": "the decoder alone on pre-dematched soft-buffer rows (a different input form)"}
        dec_ms = dec_ms or a_ms
    # algorithmic HBM bytes of each stage per step (inputs read once, outputs written once)
    samp_dl = S * pl.dl_ports * pl.ofdm_mod.get_slot_size(SLOT) * 8
    samp_ul = S * pl.ul_ports * pl.ofdm_dem.get_slot_size(SLOT) * 8
    grid_b = lambda ports: S * ports * 14 * NSUBC * 4  # noqa: E731
    L = pl.ul_layers
    alg_bytes = {
        "pdsch_encode": S * (pl.tbs_dl // 8 + (pl.plan_dl.cw_length + 7) // 8),
        "pdsch_modulate": S * ((pl.plan_dl.cw_length + 7) // 8) + grid_b(pl.dl_ports) * 11 // 14,
        "dmrs_pdsch": grid_b(pl.dl_ports) * 2 // 14,
        "ofdm_modulate": grid_b(pl.dl_ports) + samp_dl,
        "ofdm_demodulate": samp_ul + grid_b(pl.ul_ports),
        # estimator: DM-RS REs in, estimates out; demodulator: grid + estimates in, LLRs out; decoder: LLRs in, TB out
        "pusch_process": (grid_b(pl.ul_ports) * 2 // 14 + grid_b(pl.ul_ports) * L) + (grid_b(pl.ul_ports) * (1 + L)
                                                                              + S * pl.plan_ul.cw_length)
        + S * pl.plan_ul.cw_length + S * pl.tbs_ul // 8,
    }
    gbs = {k: alg_bytes[k] / (stages[k] * 1e-3) / 1e9 for k in stages}
    # the decoder's VALU-issue bound: measured SQ_INSTS_VALU per wave x waves x 2 cycles per wave64 VALU
    # instruction (MI355X_MICROARCH.md, wave scheduling) over 1024 SIMDs at 2.4 GHz; the PMC figures come
    # from profiles/ (tools/gpu_check.sh ppmc), scaled to this launch's codeblocks and iterations
    valu = valu_bound(dec_cbs, dec_its, dec_ms)
    if rank != 0:
        return None
    lat = None
    if world == 1 and not args.no_latency:
        lat = {"1_cell": latency_ms(dev, 1, **shape_kw(args)), "8_cells": latency_ms(dev, 8, **shape_kw(args)),
               "1_cell_graph": latency_ms(dev, 1, graph=True, **shape_kw(args)),
               "8_cells_graph": latency_ms(dev, 8, graph=True, **shape_kw(args))}
    low = None
    if args.low_snr_db is None:
        args.low_snr_db = LOW_SNR_DB.get((L, pl.ul_ports), -1.0)
    if world == 1 and args.low_snr_db >= 0:
        low = low_snr_line(args, dev, timed, dist)
    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = pipeline_cpu_baseline(args, pl)
    pinned = None
    if world == 1 and L > 2 and not getattr(args, "no_pinned", False):
        pinned = pinned_sibling_line(args, dev, timed, dist, cpu)
    return {
        "metric": "PDSCH+PUSCH codeblocks/s @ 100 MHz 273-PRB %dx%d MIMO (PDSCH %d layers, PUSCH %d layers x %d rx)"
                  % (pl.dl_ports, pl.ul_ports, pl.dl_layers, L, pl.ul_ports),
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
        "data": "synthetic (random transport blocks; PUSCH from a UE transmission through a %dx4 channel + AWGN "
                "%.0f dB)" % (L, pl.snr_db),
        "config": {
            "workload": "BASELINE metric (PDSCH+PUSCH codeblocks/s @ 100 MHz 273-PRB %dx%d MIMO): full PDSCH+PUSCH "
                        "slot pipeline, 100 MHz numerology-1 273 PRB, 256QAM R=948/1024" % (pl.dl_ports, pl.ul_ports)
                        if (pl.dl_ports, pl.ul_ports) == (4, 4) else
                        "configs[3] (%dx%d MIMO): full PDSCH+PUSCH slot pipeline, 100 MHz numerology-1 273 PRB, "
                        "256QAM R=948/1024" % (pl.dl_ports, pl.ul_ports),
            "cells_per_step_per_gpu": S,
            "pdsch": {"layers": pl.dl_layers, "ports": pl.dl_ports, "tbs": pl.tbs_dl, "codeblocks": cbs_dl},
            "pusch": {"layers": L, "rx_ports": pl.ul_ports, "tbs": pl.tbs_ul, "codeblocks": cbs_ul,
                      "equalizer": pl.ul_equalizer,
                      "equalizer_parity": "pinned (reference ZF)" if (L <= 2 and pl.ul_equalizer == "zf") or L == 1
                      else "unpinned: the open reference asserts for this topology; fp64 solve within stated "
                           "tolerance (tests/test_equalizer_mimo_gpu.py)",
                      "ldpc_max_iterations": pl.iters, "early_stop": True,
                      "chest_td": {0: "interpolate", 1: "average"}[pl.ul_td]},
            "parallelism": ("cells sharded over ranks" + (", slot ingest scatter/gather over RCCL"
                                                           if ingest_ms is not None else "")) if world > 1
            else "single GPU",
        },
        "throughput_gbps": bits / elapsed / 1e9,
        "pusch_tb_ok_fraction": ok_frac,
        "pusch_ldpc_iterations_mean": its_mean,
        "stage_ms": stages,
        "stage_gbs": gbs,
        "latency_ms": lat,
        "hip_graph": bool(getattr(args, "graph", False)),
        "ingest_ms_per_step": ingest_ms,
        "low_snr": low,
        "pinned_sibling": pinned,
        "kernel_ms_in_step": in_step,
        "probed_ms_per_step": probes.get("probed_ms_per_step") if probes else None,
        "roofline": {
            "bound": "hbm",
            "kernel": "ldpc_decode_hr_kernel<0,4,1> as the timed steps launch it (PUSCH codeblocks of one step, BG%d "
                      "Z=%d, CRC24B early stop, <= %d it, rate dematching fused into its load: it reads each "
                      "codeblock's E received LLRs from the codeword row)"
                      % (pl.plan_ul.base_graph, pl.plan_ul.lifting_size, pl.iters),
            "achieved": dec_bytes / (dec_ms * 1e-3) / 1e9,
            "peak": hbm_peak,
            "unit": "GB/s",
            "frac": dec_bytes / (dec_ms * 1e-3) / 1e9 / hbm_peak,
            "traffic": traffic,
            "kernel_ms": dec_ms,
            "kernel_ms_source": "live probe: HIP events around every launch of the kernel on its own stream over the "
                                "timed steps (srs_amd_probe_*, include/srsran_amd/profiling.h)" if hr and hr[0]
                                else "alone on pre-dematched rows (no live probe)",
            "algorithmic_bytes_per_launch": dec_bytes,
            "alone": alone,
            "limiter": "valu",
            "valu": valu,
            "note": "bound/achieved/peak/frac: the decoder's HBM roofline (algorithmic bytes = the codeword's LLR bytes "
                    "+ 1,060 B of message and iteration count per codeblock, / the live in-step launch time, / 8 TB/s); "
                    "traffic = HBM bytes per launch of the same in-step kernel from separate FETCH_SIZE / WRITE_SIZE "
                    "passes over this command, each counter scaled by its calibration in the kernel's own access "
                    "forms (profiles/r05_traffic.json, tools/traffic_calib.hip).  Its limiter is VALU issue, not latency "
                    "(valu: r06 PMC of the same launch, profiles/r06_ldpc_valu_model.json: SQ_ACTIVE_INST_VALU busy "
                    "0.76 over its wave-instructions = 1.71 ns each, inside the measured cost of the slow opcode class "
                    "-- v_pk_*, 32-bit min/max, med3, perm, bfe: 1.72-1.85 ns per wave-instruction per SIMD against "
                    "1.06-1.16 ns for 32-bit add / logic, tools/valu_rate_probe.hip; higher-occupancy variants ran "
                    "slower, profiles/r06_ldpc_hr_ab.json).",
        },
        "cpu_baseline": cpu,
    }


def valu_bound(cbs, its_mean, kernel_ms):
    """VALU-issue roofline of ldpc_decode_hr_kernel.  r05: the PMC of the in-step launch itself
    (profiles/r05_ldpc_valu_model.json, tools/pmc_valu_r05.py over the bench command's rocprofv3 --pmc passes):
    SQ_INSTS_VALU wave-instructions per codeblock at the measured mean iterations, issued at the guide's 2 cycles per
    wave64 VALU instruction (MI355X_MICROARCH.md wave scheduling) on 1,024 SIMDs at 2.4 GHz -> issue bound; frac =
    issue bound / live kernel time.  The measured SQ_ACTIVE_INST_VALU busy fraction of the same launches is reported
    beside it.  Without the r05 model: the r03 model (profiles/ldpc_valu_model.json), labelled as such."""
    import json
    import os

    prof = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    path = os.path.join(prof, "r06_ldpc_valu_model.json")
    if not os.path.exists(path):
        path = os.path.join(prof, "r05_ldpc_valu_model.json")
    if os.path.exists(path):
        m = json.load(open(path))
        insts = cbs * m["valu_insts_per_cb"] * (its_mean / m["iterations_mean"]) if m.get("scale_by_iterations") \
            else cbs * m["valu_insts_per_cb"]
        cycles = insts * m.get("cycles_per_valu_insn", 2.0)
        issue_s = cycles / (1024 * 2.4e9)
        return {"achieved_frac_of_peak_issue": issue_s * 1e3 / kernel_ms, "issue_bound_ms": issue_s * 1e3,
                "kernel_ms": kernel_ms, "valu_insts": insts, "cycles_per_valu_insn": m.get("cycles_per_valu_insn", 2.0),
                "valu_busy_pmc": m.get("valu_busy"),
                "basis": ("SQ_INSTS_VALU of the in-step launch at the mean issue cost of its opcode mix (r06 PMC + "
                          "per-opcode microbenchmark)" if "r06" in os.path.basename(path)
                          else "SQ_INSTS_VALU of the in-step launch (r05 PMC)"),
                "model": os.path.basename(path), "iterations_mean": its_mean}
    path = os.path.join(prof, "ldpc_valu_model.json")
    if not os.path.exists(path):
        return None
    m = json.load(open(path))
    if "valu_cycles_per_cb_fixed" in m:
        cycles = cbs * (m["valu_cycles_per_cb_fixed"] + m["valu_cycles_per_cb_iteration"] * its_mean)
        basis = "SQ_ACTIVE_INST_VALU issue cycles (r03 model, before the r04 kernel changes)"
    else:  # older model: instruction counts at 2 cycles per wave64 VALU instruction
        cycles = 2 * cbs * (m["valu_per_cb_fixed"] + m["valu_per_cb_iteration"] * its_mean)
        basis = "SQ_INSTS_VALU x 2 cycles (r03 model)"
    issue_s = cycles / (1024 * 2.4e9)
    return {"achieved_frac_of_peak_issue": issue_s * 1e3 / kernel_ms, "issue_bound_ms": issue_s * 1e3,
            "kernel_ms": kernel_ms, "valu_issue_cycles": cycles, "basis": basis, "model": os.path.basename(path),
            "iterations_mean": its_mean}


def pinned_sibling_line(args, dev, timed, dist, cpu):
    """The reference-runnable form of the headline's 4x4-port slot: the same cells with the PUSCH at 2 layers x 4 rx
    ports and the reference's ZF equalizer (every stage pinned to the compiled reference; the headline's 4-layer MMSE
    solve has no open-reference counterpart).  Its CPU comparison is exactly the cpu_baseline of the main line, whose
    reference chain runs this 2-layer PUSCH: the same work on both sides."""
    import torch

    pl = Pipeline(args.slots_pipeline, dev, snr_db=args.snr_db, ul_layers=2, dl_layers=DL_LAYERS, dl_ports=DL_PORTS,
                  ul_ports=UL_PORTS)
    stream = torch.cuda.current_stream(dev)
    elapsed, _ = timed(args, dist, 1, dev, stream, lambda: pl.step(stream))
    ok, its = pl.check()
    cbs_cell = pl.plan_dl.nof_segments + pl.plan_ul.nof_segments
    value = cbs_cell * pl.S * args.steps / elapsed
    cpu_value = cpu.get("value") if isinstance(cpu, dict) else None
    return {"metric": "PDSCH+PUSCH codeblocks/s @ 100 MHz 273-PRB 4x4 ports (PDSCH 4 layers, PUSCH 2 layers x 4 rx, "
                      "reference ZF)",
            "value": value, "unit": "codeblocks/s", "ms_per_step": elapsed / args.steps * 1e3,
            "cells_per_step": pl.S, "codeblocks_per_cell": cbs_cell, "pusch_ldpc_iterations_mean": its,
            "pusch_tb_ok_fraction": ok, "equalizer": pl.ul_equalizer, "parity": "every stage pinned to the compiled "
            "reference (tests/test_pipeline_gpu.py::test_pipeline_vs_reference_chain)",
            "cpu_baseline_same_work": cpu_value,
            "speedup_vs_cpu_baseline": (value / cpu_value) if cpu_value else None}


def low_snr_line(args, dev, timed, dist):
    """The same pipeline at an SNR near the 256QAM R=0.93 decoding threshold, where the decoder runs several
    iterations per codeblock (the headline runs at 35 dB, ~2 iterations)."""
    import torch

    pl = Pipeline(args.slots_pipeline, dev, snr_db=args.low_snr_db, seed=1, **shape_kw(args))
    stream = torch.cuda.current_stream(dev)
    elapsed, _ = timed(args, dist, 1, dev, stream, lambda: pl.step(stream))
    ok, its = pl.check()
    cbs = (pl.plan_dl.nof_segments + pl.plan_ul.nof_segments) * pl.S * args.steps
    return {"snr_db": args.low_snr_db, "value": cbs / elapsed, "unit": "codeblocks/s",
            "ms_per_step": elapsed / args.steps * 1e3, "pusch_ldpc_iterations_mean": its,
            "pusch_tb_ok_fraction": ok}


def pipeline_cpu_baseline(args, pl):
    """The reference's own CPU chain (oracle/_ref, ref_chain.cpp) per cell-slot with the implementations the
    reference's "auto" factories pick on this host: pdsch_encoder_impl, pdsch_modulator_impl +
    dmrs_pdsch_processor_impl, OFDM modulator / demodulator (generic DFT), pusch_processor_impl. One chain per
    worker thread, one worker per physical core of this process's CPU share (at most --cpu-threads), cycling over
    one slot's inputs for a bounded sample of about --cpu-seconds."""
    try:
        import oracle
        from oracle import chain as oc
        from oracle import pusch_proc as opp
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "codeblocks/s", "error": "oracle unavailable: %s" % e}
    if oracle.REF is None or not hasattr(oracle.REF, "srs_ref_chain_many"):
        return {"value": None, "unit": "codeblocks/s", "error": "oracle/_ref not built"}
    import os

    # The open reference's PUSCH processor runs at most two layers (its equalizer asserts for 3 / 4,
    # channel_equalizer_generic_impl.cpp:197-247): for a 4-layer GPU line the CPU chain processes the same cell
    # with a 2-layer PUSCH (inputs from a 1-cell 2-layer pipeline); codeblocks/s is normalised per codeblock.
    ref_pl = pl if pl.ul_layers <= 2 else Pipeline(1, pl.dev, snr_db=pl.snr_db, ul_layers=2, dl_layers=pl.dl_layers,
                                                   dl_ports=pl.dl_ports, ul_ports=pl.ul_ports)
    cfg = chain_config(ref_pl)
    tb = ref_pl.tb_dl[0].cpu().numpy()
    n = oc.slot_size(cfg)
    samp = np.ascontiguousarray(ref_pl.samp_ul[0, :, :n].cpu().numpy())
    logical, physical = oc.host_cores()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or logical
    threads = max(1, min(physical, share, args.cpu_threads))
    cbs = ref_pl.plan_dl.nof_segments + ref_pl.plan_ul.nof_segments
    # single thread: per-stage breakdown
    w1, st1, ok1, _ = oc.many(cfg, tb, samp, 2, 1)
    n1 = max(2, int(args.cpu_seconds / 4 / max(w1 / 2, 1e-6)))
    w1, st1, ok1, _ = oc.many(cfg, tb, samp, n1, 1)
    per_slot = w1 / n1
    nmt = max(2 * threads, int(args.cpu_seconds * threads / per_slot / 2))
    wm, stm, okm, itm = oc.many(cfg, tb, samp, nmt, threads)
    value = nmt * cbs / wm
    return {"value": value, "unit": "codeblocks/s", "cores": threads, "kind": "reference",
            "cores_used": threads, "host_logical_cpus": logical, "host_physical_cores": physical,
            "os_cpu_count": os.cpu_count(),
            "per_gpu_share_rationale": "%d threads = this process's CPU share on the GPU box (OMP_NUM_THREADS; the "
                                       "harness gives each GPU of an 8-GPU node 1/8 of the host), i.e. the host cores "
                                       "that stand beside ONE MI355X; the whole host is not this process's to use"
                                       % threads,
            "whole_host_extrapolated_value": value / threads * physical,
            "whole_host_extrapolation": "measured %d-thread rate scaled linearly to all %d physical host cores (an "
                                        "upper bound: no memory-bandwidth contention)" % (threads, physical),
            "single_thread_value": n1 * cbs / w1,
            "impl": opp.describe("auto") + ", precoder " + ("avx512" if "avx512" in opp.describe("auto") else "avx2")
                    + ", LDPC encoder avx2, DFT generic (FFTW absent)",
            "sample": "%d cell-slots on %d threads (one reference chain each, %.1f s) and %d on one thread (%.1f s), "
                      "cycling over one slot's inputs, through the reference's own CPU chain compiled from "
                      "/root/reference (oracle/_ref/ref_chain.cpp): pdsch_encoder_impl, pdsch_modulator_impl, "
                      "dmrs_pdsch_processor_impl, ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl, "
                      "pusch_processor_impl (dmrs_pusch_estimator_impl, pusch_demodulator_impl, "
                      "ulsch_demultiplex_impl, pusch_decoder_impl) with the \"auto\" factory implementations "
                      "(%s); PUSCH TB CRC ok in %d of %d slots; per cell PDSCH %d layers x %d ports and PUSCH "
                      "%d layers x %d rx (%d codeblocks)%s"
                      % (nmt, threads, wm, n1, w1, opp.describe("auto"), okm, nmt, ref_pl.dl_layers, ref_pl.dl_ports,
                         ref_pl.ul_layers, ref_pl.ul_ports, cbs,
                         "" if ref_pl is pl else "; the open reference cannot run the GPU line's %d-layer PUSCH "
                         "(its equalizer asserts), so its chain runs the 2-layer PUSCH of the same cell"
                         % pl.ul_layers),
            "pusch_layers": ref_pl.ul_layers,
            "stage_s_per_slot": {k: v / n1 for k, v in st1.items()}}

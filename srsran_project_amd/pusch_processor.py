"""Host-side mirror of srsRAN's PUSCH processor over the MI355X C-ABI
(include/srsran_amd/pusch_processor.h).

Reference interface:
  pusch_processor.h:181   process(span<uint8_t> data, unique_rx_buffer rm_buffer,
                                  pusch_processor_result_notifier& notifier,
                                  const resource_grid_reader& grid, const pdu_t& pdu)
  pusch_processor.h:117   pdu_t (slot, rnti, bwp, mcs_descr, codeword {rv, base graph, new_data}, n_id,
                                 nof_tx_layers, rx_ports, dmrs_symbol_mask, dmrs, freq_alloc, time allocation,
                                 tbs_lbrm)
  factories.h:107         pusch_processor_factory_sw_configuration (decoder iterations, early stop, ...)
The notifier's pusch_processor_result_data (decoder result + CSI) comes back as a
PuschProcessorResult per transport block.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .pusch_chest import ChestPortStats
from .sch import PuschDecoderResult, SchPlan


class PuschProcessorConfig(ctypes.Structure):
    """``srs_amd_pusch_processor_config`` (pusch_processor_factory_sw_configuration + component choices). The
    defaults are the reference PUSCH processor benchmark's (pusch_processor_benchmark.cpp:133-140, 637-638)."""

    _fields_ = [("dec_nof_iterations", ctypes.c_uint32), ("dec_enable_early_stop", ctypes.c_int32),
                ("dec_force_decoding", ctypes.c_int32), ("equalizer", ctypes.c_int32),
                ("fd_smoothing", ctypes.c_int32), ("td_interpolation", ctypes.c_int32),
                ("compensate_cfo", ctypes.c_int32), ("ldpc_arith", ctypes.c_int32)]

    def __init__(self, dec_nof_iterations=2, dec_enable_early_stop=True, dec_force_decoding=False, equalizer=0,
                 fd_smoothing=2, td_interpolation=0, compensate_cfo=True, ldpc_arith=0):
        super().__init__(dec_nof_iterations, int(dec_enable_early_stop), int(dec_force_decoding), equalizer,
                         fd_smoothing, td_interpolation, int(compensate_cfo), ldpc_arith)


class UciPart2Parameter(ctypes.Structure):
    """``srs_amd_uci_part2_parameter``."""

    _fields_ = [("offset", ctypes.c_uint16), ("width", ctypes.c_uint16)]


class UciPart2Entry(ctypes.Structure):
    """``srs_amd_uci_part2_entry``."""

    _fields_ = [("nof_parameters", ctypes.c_uint32), ("parameters", UciPart2Parameter * 2),
                ("map_size", ctypes.c_uint32), ("map", ctypes.c_uint16 * 16)]


class UciPart2SizeDescription(ctypes.Structure):
    """``srs_amd_uci_part2_size_description`` (uci_part2_size_description)."""

    _fields_ = [("nof_entries", ctypes.c_uint32), ("entries", UciPart2Entry * 2)]


def uci_part2_description(entries):
    """entries: [([(offset, width), ...], [size per index]), ...] -> UciPart2SizeDescription."""
    d = UciPart2SizeDescription()
    d.nof_entries = len(entries)
    for e, (params, sizes) in enumerate(entries):
        d.entries[e].nof_parameters = len(params)
        for q, (off, w) in enumerate(params):
            d.entries[e].parameters[q].offset = off
            d.entries[e].parameters[q].width = w
        d.entries[e].map_size = len(sizes)
        for m, v in enumerate(sizes):
            d.entries[e].map[m] = v
    return d


def uci_part2_get_size(part1, descr):
    """srs_amd_uci_part2_get_size: the CSI part 2 size of a CSI part 1 payload (one bit per byte)."""
    import numpy as np

    lib = _L()
    b = np.ascontiguousarray(part1, np.uint8)
    return int(lib.srs_amd_uci_part2_get_size(b.ctypes.data, b.size, ctypes.byref(descr)))


class PuschPdu(ctypes.Structure):
    """``srs_amd_pusch_pdu`` (pusch_processor::pdu_t, data-only subset)."""

    _fields_ = [(n, ctypes.c_uint32) for n in ("numerology", "slot_index", "rnti", "bwp_start_rb", "bwp_size_rb")] + \
        [("modulation", ctypes.c_int32), ("target_code_rate", ctypes.c_float), ("rv", ctypes.c_uint32),
         ("base_graph", ctypes.c_uint32), ("new_data", ctypes.c_int32)] + \
        [(n, ctypes.c_uint32) for n in ("n_id", "nof_tx_layers", "nof_rx_ports", "dmrs_symbol_mask", "dmrs_type",
                                        "scrambling_id", "n_scid", "nof_cdm_groups_without_data", "rb_start",
                                        "rb_count", "start_symbol_index", "nof_symbols", "tbs_lbrm_bytes", "tbs",
                                        "transform_precoding", "n_rs_id", "nof_harq_ack", "nof_csi_part1")] + \
        [("alpha_scaling", ctypes.c_float), ("beta_offset_harq_ack", ctypes.c_float),
         ("beta_offset_csi_part1", ctypes.c_float), ("beta_offset_csi_part2", ctypes.c_float),
         ("csi_part2_size", UciPart2SizeDescription), ("has_dc_position", ctypes.c_uint32),
         ("dc_position", ctypes.c_uint32)]


class PuschProcessorResult(ctypes.Structure):
    """``srs_amd_pusch_processor_result``: pusch_decoder_result + channel state information."""

    _fields_ = [("data", PuschDecoderResult), ("sinr_db", ctypes.c_float), ("epre_db", ctypes.c_float),
                ("rsrp_db", ctypes.c_float), ("time_alignment_s", ctypes.c_float),
                ("harq_ack_status", ctypes.c_int32), ("csi_part1_status", ctypes.c_int32),
                ("csi_part2_status", ctypes.c_int32), ("nof_csi_part2", ctypes.c_uint32), ("cfo_hz", ctypes.c_float)]


RESULT_BYTES = ctypes.sizeof(PuschProcessorResult)


class PuschIntermediates(ctypes.Structure):
    """``srs_amd_pusch_intermediates``: caller-owned buffers for the processor's intermediate results."""

    _fields_ = [("d_estimates", ctypes.c_void_p), ("est_stride", ctypes.c_uint64), ("d_port_stats", ctypes.c_void_p),
                ("d_llrs", ctypes.c_void_p), ("llr_stride", ctypes.c_uint32),
                ("d_harq_ack", ctypes.c_void_p), ("harq_ack_stride", ctypes.c_uint32),
                ("d_csi_part1", ctypes.c_void_p), ("csi_part1_stride", ctypes.c_uint32),
                ("d_csi_part2", ctypes.c_void_p), ("csi_part2_stride", ctypes.c_uint32),
                ("d_cb_iterations", ctypes.c_void_p)]


class PuschSlotPdu(ctypes.Structure):
    """``srs_amd_pusch_slot_pdu``: one PDU of srs_amd_pusch_process_slot."""

    _fields_ = [("plan", ctypes.c_void_p), ("grid", ctypes.c_uint32), ("cb_offset", ctypes.c_uint32),
                ("tb_offset", ctypes.c_uint64), ("d_soft", ctypes.c_void_p), ("uci_offset", ctypes.c_uint64),
                ("has_slot", ctypes.c_uint32), ("numerology", ctypes.c_uint32), ("slot_index", ctypes.c_uint32),
                ("d_grid", ctypes.c_void_p), ("soft_on_failure", ctypes.c_uint32)]


class PuschSlotIo(ctypes.Structure):
    """``srs_amd_pusch_slot_io``: optional outputs of srs_amd_pusch_process_slot_ex."""

    _fields_ = [("d_cb_iterations", ctypes.c_void_p), ("d_uci", ctypes.c_void_p), ("d_port_stats", ctypes.c_void_p)]


def make_pdu(**kw):
    """PuschPdu with the reference benchmark's defaults (pusch_processor_benchmark.cpp:396-431)."""
    d = dict(numerology=1, slot_index=0, rnti=1, bwp_start_rb=0, bwp_size_rb=51, modulation=2,
             target_code_rate=679.0, rv=0, base_graph=1, new_data=1, n_id=0, nof_tx_layers=1, nof_rx_ports=1,
             dmrs_symbol_mask=(1 << 2) | (1 << 11), dmrs_type=1, scrambling_id=0, n_scid=0,
             nof_cdm_groups_without_data=2, rb_start=0, rb_count=None, start_symbol_index=0, nof_symbols=14,
             tbs_lbrm_bytes=0, tbs=0, transform_precoding=0, n_rs_id=0, nof_harq_ack=0, nof_csi_part1=0,
             alpha_scaling=1.0, beta_offset_harq_ack=5.0, beta_offset_csi_part1=5.0, beta_offset_csi_part2=5.0,
             csi_part2_size=None, dc_position=None)
    d.update(kw)
    dc = d.pop("dc_position")
    if dc is not None:  # pdu_t::dc_position (unset: None)
        d["has_dc_position"], d["dc_position"] = 1, int(dc)
    if d["rb_count"] is None:
        d["rb_count"] = d["bwp_size_rb"] - d["rb_start"]
    p = PuschPdu()
    for k, v in d.items():
        if k == "csi_part2_size":
            if v is not None:
                p.csi_part2_size = v if isinstance(v, UciPart2SizeDescription) else uci_part2_description(v)
            continue
        setattr(p, k, v)
    return p


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_pusch_processor_create": (c.c_int, [c.POINTER(P), c.POINTER(PuschProcessorConfig), c.c_int]),
        "srs_amd_pusch_processor_destroy": (None, [P]),
        "srs_amd_pusch_processor_plan_create": (c.c_int, [P, c.POINTER(PuschPdu), u, c.POINTER(P),
                                                          c.POINTER(SchPlan), c.POINTER(c.c_uint64)]),
        "srs_amd_pusch_processor_plan_destroy": (None, [P]),
        "srs_amd_pusch_process_batch": (c.c_int, [P, P, P, c.c_uint64, u, P, u, P, P, P, P]),
        "srs_amd_pusch_process": (c.c_int, [P, P, P, P, c.POINTER(PuschProcessorResult), P]),
        "srs_amd_pusch_process_slot": (c.c_int, [P, c.POINTER(PuschSlotPdu), u, P, c.c_uint64, u, P, P, P]),
        "srs_amd_pusch_process_slot_ex": (c.c_int, [P, c.POINTER(PuschSlotPdu), u, P, c.c_uint64, u, P, P,
                                                    c.POINTER(PuschSlotIo), P]),
        "srs_amd_pusch_processor_plan_set_slot": (c.c_int, [P, u, u]),
        "srs_amd_pusch_processor_plan_info": (c.c_int, [P, c.POINTER(u), c.POINTER(u), c.POINTER(c.c_uint64)]),
        "srs_amd_uci_part2_get_size": (c.c_int32, [P, u, c.POINTER(UciPart2SizeDescription)]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_declared = False


def _L():
    global _declared
    lib = _lib.lib()
    if not _declared:
        _declare(lib)
        _declared = True
    return lib


class PuschProcessorPlan:
    def __init__(self, proc, pdu, nof_subc):
        self._lib = proc._lib
        h = ctypes.c_void_p()
        self.sch = SchPlan()
        sb = ctypes.c_uint64()
        self.pdu = pdu
        _lib.check(self._lib.srs_amd_pusch_processor_plan_create(proc._h, ctypes.byref(pdu), nof_subc,
                                                                ctypes.byref(h), ctypes.byref(self.sch),
                                                                ctypes.byref(sb)), "pusch_processor plan")
        self._h = h
        self.nof_subc = nof_subc
        self.soft_bytes = sb.value
        self.tb_bytes = pdu.tbs // 8
        nc, m2 = ctypes.c_uint32(), ctypes.c_uint32()
        _lib.check(self._lib.srs_amd_pusch_processor_plan_info(h, ctypes.byref(nc), ctypes.byref(m2), None),
                   "pusch_processor plan info")
        self.nof_codeblocks = nc.value
        self.max_csi_part2 = m2.value
        self.uci_bytes = pdu.nof_harq_ack + pdu.nof_csi_part1 + self.max_csi_part2

    def set_slot(self, numerology, slot_index):
        """srs_amd_pusch_processor_plan_set_slot: the same configuration in another slot."""
        _lib.check(self._lib.srs_amd_pusch_processor_plan_set_slot(self._h, numerology, slot_index),
                   "pusch_processor plan set_slot")
        self.pdu.numerology, self.pdu.slot_index = numerology, slot_index

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_processor_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PuschProcessor:
    """pusch_processor over the MI355X chain (estimator -> demodulator -> decoder)."""

    def __init__(self, config=None, device=-1):
        self._lib = _L()
        self.config = config or PuschProcessorConfig()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pusch_processor_create(ctypes.byref(h), ctypes.byref(self.config), int(device)),
                   "pusch_processor create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_processor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, pdu, nof_subc):
        return PuschProcessorPlan(self, pdu, nof_subc)

    def process(self, grid, plan, soft_buffer=None):
        """Host: grid uint32 [P][14][nsubc] -> (tb bytes, PuschProcessorResult). soft_buffer: int8 numpy HARQ
        buffer of plan.soft_bytes kept between transmissions (None: new data only)."""
        g = np.ascontiguousarray(grid, dtype=np.uint32)
        tb = np.zeros(plan.tb_bytes, np.uint8)
        res = PuschProcessorResult()
        sb = None
        if soft_buffer is not None:
            if soft_buffer.dtype != np.int8 or soft_buffer.size != plan.soft_bytes:
                raise ValueError("soft buffer must be int8 of %d bytes" % plan.soft_bytes)
            sb = soft_buffer.ctypes.data
        _lib.check(self._lib.srs_amd_pusch_process(self._h, plan._h, g.ctypes.data, tb.ctypes.data,
                                                   ctypes.byref(res), sb), "pusch_process")
        return tb, res

    def process_batch(self, grids, plan, tbs=None, results=None, soft=None, port_stats=None, estimates=None,
                      llrs=None, stream=None, harq_ack=None, csi_part1=None, csi_part2=None):
        """Device: grids int32 [n][P][14][nsubc] -> tbs uint8 [n][tbs/8], results uint8 [n][RESULT_BYTES].
        Optional caller buffers for the intermediates: port_stats float32 [n][P][6], estimates int32
        [n][P][L][14][nsubc], llrs int8 [n][>= UL-SCH codeword length]; UCI payloads harq_ack uint8
        [n][nof_harq_ack], csi_part1 uint8 [n][nof_csi_part1], csi_part2 uint8 [n][largest CSI part 2 size] (one bit
        per byte; the size each grid's CSI part 1 selected is in its result's nof_csi_part2)."""
        import torch

        n = grids.shape[0]
        dev = grids.device
        if tbs is None:
            tbs = torch.zeros((n, plan.tb_bytes), dtype=torch.uint8, device=dev)
        if results is None:
            results = torch.zeros((n, RESULT_BYTES), dtype=torch.uint8, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        io = None
        if any(x is not None for x in (port_stats, estimates, llrs, harq_ack, csi_part1, csi_part2)):
            io = PuschIntermediates(
                None if estimates is None else estimates.data_ptr(), 0 if estimates is None else estimates.stride(0),
                None if port_stats is None else port_stats.data_ptr(), None if llrs is None else llrs.data_ptr(),
                0 if llrs is None else llrs.stride(0), None if harq_ack is None else harq_ack.data_ptr(),
                0 if harq_ack is None else harq_ack.stride(0), None if csi_part1 is None else csi_part1.data_ptr(),
                0 if csi_part1 is None else csi_part1.stride(0), None if csi_part2 is None else csi_part2.data_ptr(),
                0 if csi_part2 is None else csi_part2.stride(0))
        _lib.check(self._lib.srs_amd_pusch_process_batch(
            self._h, plan._h, grids.data_ptr(), grids.stride(0), n, tbs.data_ptr(), tbs.stride(0),
            results.data_ptr(), None if soft is None else soft.data_ptr(),
            None if io is None else ctypes.byref(io), ctypes.c_void_p(stream.cuda_stream)),
            "pusch_process_batch")
        return tbs, results

    def process_slot(self, grids, pdus, tbs=None, results=None, stream=None, cb_iterations=None, uci=None,
                     port_stats=None):
        """Device: every PDU of a slot in one launch sequence (uplink_processor_impl::process_pusch per PDU).
        grids int32 [n][P][14][nsubc]; pdus: a PuschSlot or a list of (plan, grid index[, soft buffer tensor]).
        Optional outputs: cb_iterations int32 [slot.cb_total] (per-codeblock iteration counts, PDU u's from
        slot.cb_offsets[u]), uci uint8 [slot.uci_total] (UCI payload rows at slot.uci_offsets[u]), port_stats float32
        [len(pdus)][4][6] (estimator measurements per PDU and receive port).  Returns (tbs
        uint8 flat, tb offsets, results uint8 [len(pdus)][RESULT_BYTES])."""
        import torch

        slot = pdus if isinstance(pdus, PuschSlot) else PuschSlot(pdus)
        dev = grids.device
        if tbs is None:
            tbs = torch.zeros(max(slot.tb_total, 1), dtype=torch.uint8, device=dev)
        if results is None:
            results = torch.zeros((slot.n, RESULT_BYTES), dtype=torch.uint8, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        io = None
        if cb_iterations is not None or uci is not None or port_stats is not None:
            io = PuschSlotIo(None if cb_iterations is None else cb_iterations.data_ptr(),
                             None if uci is None else uci.data_ptr(),
                             None if port_stats is None else port_stats.data_ptr())
        _lib.check(self._lib.srs_amd_pusch_process_slot_ex(
            self._h, slot.arr, slot.n, grids.data_ptr(), grids.stride(0), grids.shape[0], tbs.data_ptr(),
            results.data_ptr(), None if io is None else ctypes.byref(io), ctypes.c_void_p(stream.cuda_stream)),
            "pusch_process_slot")
        return tbs, slot.offsets, results


class PuschSlot:
    """The srs_amd_pusch_slot_pdu array of a slot, built once per slot configuration: pdus = list of
    (plan, grid index) or (plan, grid index, device soft buffer); transport block u at byte offsets[u] (64-byte
    aligned) of a tb_total-byte buffer, its codeblock iteration counts at cb_offsets[u] of cb_total, its UCI payload
    row at uci_offsets[u] of uci_total."""

    def __init__(self, pdus, slots=None):
        """slots: optional per-PDU (numerology, slot_index) (srs_amd_pusch_slot_pdu has_slot), None: the plans'."""
        self.plans = [p[0] for p in pdus]  # keep the plans alive
        self.soft = [p[2] if len(p) > 2 else None for p in pdus]
        self.n = len(pdus)
        self.offsets, self.cb_offsets, self.uci_offsets = [], [], []
        total = cbs = ucis = 0
        for p in pdus:
            plan = p[0]
            self.offsets.append(total)
            self.cb_offsets.append(cbs)
            self.uci_offsets.append(ucis)
            total += (plan.tb_bytes + 63) // 64 * 64
            cbs += plan.nof_codeblocks
            ucis += plan.uci_bytes
        self.tb_total, self.cb_total, self.uci_total = total, cbs, ucis
        self.arr = (PuschSlotPdu * max(self.n, 1))()
        for i, p in enumerate(pdus):
            soft = self.soft[i]
            self.arr[i] = PuschSlotPdu(p[0]._h.value, int(p[1]), self.cb_offsets[i], self.offsets[i],
                                       None if soft is None else soft.data_ptr(), self.uci_offsets[i])
            if slots is not None and slots[i] is not None:
                self.arr[i].has_slot = 1
                self.arr[i].numerology, self.arr[i].slot_index = slots[i]


def parse_results(results):
    """uint8 [n][RESULT_BYTES] (host numpy) -> list of PuschProcessorResult."""
    arr = np.ascontiguousarray(results, np.uint8)
    return [PuschProcessorResult.from_buffer_copy(arr[i].tobytes()) for i in range(arr.shape[0])]

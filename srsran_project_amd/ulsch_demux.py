"""Host mirror of the MI355X UL-SCH demultiplexer (include/srsran_amd/ulsch_demux.h):
ulsch_demultiplex::demultiplex (include/srsran/phy/upper/channel_processors/pusch/ulsch_demultiplex.h:97)."""
import ctypes

import numpy as np

from . import _lib

_FIELDS = ["modulation", "nof_layers", "nof_prb", "start_symbol_index", "nof_symbols", "nof_harq_ack_rvd", "dmrs_type",
           "dmrs_symbol_mask", "nof_cdm_groups_without_data", "nof_harq_ack_bits", "nof_enc_harq_ack_bits",
           "nof_csi_part1_bits", "nof_enc_csi_part1_bits", "c_init", "nof_csi_part2_bits", "nof_enc_csi_part2_bits"]


class UlschDemuxConfig(ctypes.Structure):
    """``srs_amd_ulsch_demux_config``."""

    _fields_ = [(n, ctypes.c_int32 if n == "modulation" else ctypes.c_uint32) for n in _FIELDS]


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    u64 = c.c_uint64
    sigs = {
        "srs_amd_ulsch_demux_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_ulsch_demux_destroy": (None, [P]),
        "srs_amd_ulsch_demux_plan_create": (c.c_int, [P, c.POINTER(UlschDemuxConfig), c.POINTER(P), c.POINTER(u),
                                                      c.POINTER(u)]),
        "srs_amd_ulsch_demux_plan_destroy": (None, [P]),
        "srs_amd_ulsch_demultiplex_batch": (c.c_int, [P, P, P, u64, P, u64, P, u64, P, u64, u, P]),
        "srs_amd_ulsch_demultiplex": (c.c_int, [P, P, P, P, P, P]),
        "srs_amd_ulsch_demultiplex_csi2_batch": (c.c_int, [P, P, P, u64, P, u64, P, u64, P, u64, P, u64, u, P]),
        "srs_amd_ulsch_demultiplex_csi2": (c.c_int, [P, P, P, P, P, P, P]),
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


class UlschDemuxPlan:
    def __init__(self, demux, cfg):
        self._lib = demux._lib
        h = ctypes.c_void_p()
        ncw, nsch = ctypes.c_uint32(), ctypes.c_uint32()
        _lib.check(self._lib.srs_amd_ulsch_demux_plan_create(demux._h, ctypes.byref(cfg), ctypes.byref(h),
                                                            ctypes.byref(ncw), ctypes.byref(nsch)), "ulsch_demux plan")
        self._h = h
        self.cfg = cfg
        self.nof_codeword_bits = ncw.value
        self.nof_sch_bits = nsch.value

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_ulsch_demux_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class UlschDemux:
    """ulsch_demultiplex on one device."""

    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_ulsch_demux_create(ctypes.byref(h), int(device)), "ulsch_demux create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_ulsch_demux_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, cfg):
        return UlschDemuxPlan(self, cfg)

    def demultiplex(self, codeword, plan):
        """Host: int8 codeword LLRs -> (UL-SCH, HARQ-ACK, CSI part 1) int8 arrays."""
        cw = np.ascontiguousarray(codeword, np.int8)
        if cw.size != plan.nof_codeword_bits:
            raise ValueError("codeword length %d, plan expects %d" % (cw.size, plan.nof_codeword_bits))
        c = plan.cfg
        sch = np.zeros(plan.nof_sch_bits, np.int8)
        ack = np.zeros(c.nof_enc_harq_ack_bits if c.nof_harq_ack_bits else 0, np.int8)
        csi1 = np.zeros(c.nof_enc_csi_part1_bits if c.nof_csi_part1_bits else 0, np.int8)
        if c.nof_csi_part2_bits and c.nof_csi_part1_bits:
            csi2 = np.zeros(c.nof_enc_csi_part2_bits, np.int8)
            _lib.check(self._lib.srs_amd_ulsch_demultiplex_csi2(self._h, plan._h, cw.ctypes.data, sch.ctypes.data,
                                                                ack.ctypes.data, csi1.ctypes.data, csi2.ctypes.data),
                       "ulsch_demultiplex_csi2")
            return sch, ack, csi1, csi2
        _lib.check(self._lib.srs_amd_ulsch_demultiplex(self._h, plan._h, cw.ctypes.data, sch.ctypes.data,
                                                       ack.ctypes.data, csi1.ctypes.data), "ulsch_demultiplex")
        return sch, ack, csi1

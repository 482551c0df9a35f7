"""Host mirror of the UL-SCH / UCI multiplexing geometry (include/srsran_amd/ulsch_info.h):
get_ulsch_information (include/srsran/ran/pusch/ulsch_info.h:163, lib/ran/pusch/ulsch_info.cpp)."""
import ctypes

from . import _lib

_F = [("tbs", ctypes.c_uint32), ("modulation", ctypes.c_int32), ("target_code_rate", ctypes.c_float),
      ("nof_harq_ack_bits", ctypes.c_uint32), ("nof_csi_part1_bits", ctypes.c_uint32),
      ("nof_csi_part2_bits", ctypes.c_uint32), ("alpha_scaling", ctypes.c_float),
      ("beta_offset_harq_ack", ctypes.c_float), ("beta_offset_csi_part1", ctypes.c_float),
      ("beta_offset_csi_part2", ctypes.c_float), ("nof_rb", ctypes.c_uint32), ("start_symbol_index", ctypes.c_uint32),
      ("nof_symbols", ctypes.c_uint32), ("dmrs_type", ctypes.c_uint32), ("dmrs_symbol_mask", ctypes.c_uint32),
      ("nof_cdm_groups_without_data", ctypes.c_uint32), ("nof_layers", ctypes.c_uint32), ("contains_dc", ctypes.c_int32)]


class UlschConfig(ctypes.Structure):
    """``srs_amd_ulsch_config`` (ulsch_configuration)."""

    _fields_ = _F

    def __init__(self, **kw):
        d = dict(alpha_scaling=1.0, beta_offset_harq_ack=5.0, beta_offset_csi_part1=5.0, beta_offset_csi_part2=5.0)
        d.update(kw)
        super().__init__(**d)

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class UlschInfo(ctypes.Structure):
    """``srs_amd_ulsch_info`` (ulsch_information)."""

    _fields_ = [(n, ctypes.c_uint32) for n in (
        "nof_ul_sch_bits", "nof_harq_ack_bits", "nof_harq_ack_rvd", "nof_csi_part1_bits", "nof_csi_part2_bits",
        "nof_harq_ack_re", "nof_csi_part1_re", "nof_csi_part2_re", "nof_dc_overlap_bits", "sch_tb_crc_size",
        "sch_base_graph", "sch_nof_cb", "sch_lifting_size", "sch_nof_bits_per_cb", "sch_nof_filler_bits_per_cb")]


def ulsch_information(cfg):
    """get_ulsch_information: dict of the ulsch_information fields."""
    lib = _lib.lib()
    f = lib.srs_amd_ulsch_information
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(UlschConfig), ctypes.POINTER(UlschInfo)]
    out = UlschInfo()
    _lib.check(f(ctypes.byref(cfg), ctypes.byref(out)), "ulsch_information")
    return {k: getattr(out, k) for k, _ in out._fields_}

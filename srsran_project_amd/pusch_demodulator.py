"""Host-side mirror of srsRAN's PUSCH demodulator over the MI355X C-ABI
(include/srsran_amd/pusch_demodulator.h).

Reference interface:
  pusch_demodulator.h:95    demodulate(pusch_codeword_buffer&, pusch_demodulator_notifier&,
                                       const resource_grid_reader&, const channel_estimate&, const configuration&)
  pusch_demodulator.h:51    configuration {rnti, rb_mask, modulation, start_symbol_index, nof_symbols,
                                           dmrs_symb_pos, dmrs_config_type, nof_cdm_groups_without_data, n_id,
                                           nof_tx_layers, enable_transform_precoding, rx_ports}
The channel estimate is the DmrsPuschEstimator's output (estimates + per-port stats).
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .pdsch_modulator import MASK_BYTES, _mask_bytes
from .pusch_chest import ChestPortStats


class _Config(ctypes.Structure):
    _fields_ = [("rnti", ctypes.c_uint32), ("n_id", ctypes.c_uint32), ("modulation", ctypes.c_int32),
                ("crb_mask", ctypes.c_uint8 * MASK_BYTES), ("reserved0", ctypes.c_uint8),
                ("start_symbol", ctypes.c_uint32), ("nof_symbols", ctypes.c_uint32),
                ("dmrs_symbol_mask", ctypes.c_uint32), ("dmrs_type", ctypes.c_uint32),
                ("nof_cdm_groups_without_data", ctypes.c_uint32), ("nof_tx_layers", ctypes.c_uint32),
                ("nof_rx_ports", ctypes.c_uint32), ("equalizer", ctypes.c_int32),
                ("transform_precoding", ctypes.c_uint32)]


@dataclass
class PuschDemodulatorConfig:
    """pusch_demodulator::configuration (rb_mask as CRB indices)."""

    rnti: int
    crbs: list
    modulation: int
    start_symbol: int
    nof_symbols: int
    dmrs_symb_pos: int
    n_id: int
    nof_tx_layers: int
    nof_rx_ports: int
    dmrs_type: int = 1
    nof_cdm_groups_without_data: int = 2
    equalizer: int = 0  # ChannelEqualizerAlgorithmType
    enable_transform_precoding: bool = False

    def _c(self):
        return _Config(self.rnti, self.n_id, self.modulation, _mask_bytes(self.crbs), 0, self.start_symbol,
                       self.nof_symbols, self.dmrs_symb_pos, self.dmrs_type, self.nof_cdm_groups_without_data,
                       self.nof_tx_layers, self.nof_rx_ports, int(self.equalizer),
                       int(self.enable_transform_precoding))


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_pusch_demodulator_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_pusch_demodulator_destroy": (None, [P]),
        "srs_amd_pusch_demod_plan_create": (c.c_int, [P, c.POINTER(_Config), u, c.POINTER(P), c.POINTER(u)]),
        "srs_amd_pusch_demod_plan_destroy": (None, [P]),
        "srs_amd_pusch_demodulate": (c.c_int, [P, P, P, P, P, P]),
        "srs_amd_pusch_demodulate_batch": (c.c_int, [P, P, P, c.c_uint64, P, c.c_uint64, P, P, c.c_uint64, u, P]),
        "srs_amd_pusch_demap_descramble_batch": (c.c_int, [P, P, P, P, P, c.c_uint64, u, P]),
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


class PuschDemodPlan:
    def __init__(self, dem, config, nof_subc):
        self._lib = dem._lib
        c = config._c()
        h = ctypes.c_void_p()
        n = ctypes.c_uint32()
        _lib.check(self._lib.srs_amd_pusch_demod_plan_create(dem._h, ctypes.byref(c), nof_subc, ctypes.byref(h),
                                                            ctypes.byref(n)), "pusch_demodulator plan")
        self._h = h
        self.nof_re = n.value
        self.nof_subc = nof_subc
        self.config = config
        self.nof_llrs = self.nof_re * config.nof_tx_layers * (1 if config.modulation < 2 else config.modulation)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_demod_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PuschDemodulator:
    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pusch_demodulator_create(ctypes.byref(h), int(device)),
                   "pusch_demodulator create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_demodulator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, config, nof_subc):
        return PuschDemodPlan(self, config, nof_subc)

    def demodulate(self, grid, estimates, stats, config):
        """grid uint32 [P][14][nsubc]; estimates uint32 [P][L][14][nsubc]; stats: per-port dicts (noise_var ...)
        or ChestPortStats array. Returns int8 LLRs."""
        g = np.ascontiguousarray(grid, dtype=np.uint32)
        e = np.ascontiguousarray(estimates, dtype=np.uint32)
        plan = config if isinstance(config, PuschDemodPlan) else self.plan(config, g.shape[2])
        st = (ChestPortStats * g.shape[0])()
        for i, s in enumerate(stats):
            for k, _ in ChestPortStats._fields_:
                setattr(st[i], k, float(s[k] if isinstance(s, dict) else getattr(s, k)))
        out = np.zeros(plan.nof_llrs, np.int8)
        _lib.check(self._lib.srs_amd_pusch_demodulate(self._h, plan._h, g.ctypes.data, e.ctypes.data, st,
                                                      out.ctypes.data), "pusch_demodulate")
        return out

    def demodulate_batch(self, grids, estimates, stats, plan, llrs=None, stream=None):
        """Device: grids int32 [n][P][14][nsubc], estimates int32 [n][P][L][14][nsubc], stats float32 [n][P][6]."""
        import torch

        n = grids.shape[0]
        if llrs is None:
            llrs = torch.empty((n, plan.nof_llrs), dtype=torch.int8, device=grids.device)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pusch_demodulate_batch(
            self._h, plan._h, grids.data_ptr(), grids.stride(0), estimates.data_ptr(), estimates.stride(0),
            stats.data_ptr(), llrs.data_ptr(), llrs.stride(0), n, ctypes.c_void_p(stream.cuda_stream)),
            "pusch_demodulate_batch")
        return llrs

    def demap_descramble_batch(self, eq_symbols, eq_noise_vars, plan, llrs=None, stream=None):
        """Device: the demodulator's soft demapping (per OFDM symbol) + descrambling of equalized symbols
        complex64 [n][nof_re * layers] and noise variances float32 [n][nof_re * layers]."""
        import torch

        n = eq_symbols.shape[0]
        if eq_symbols.shape[1] != plan.nof_re * plan.config.nof_tx_layers or eq_noise_vars.shape != eq_symbols.shape:
            raise ValueError("equalized symbols must be [n][nof_re * layers]")
        if not (eq_symbols.is_contiguous() and eq_noise_vars.is_contiguous()):
            raise ValueError("equalized symbols must be contiguous")
        if llrs is None:
            llrs = torch.empty((n, plan.nof_llrs), dtype=torch.int8, device=eq_symbols.device)
        if stream is None:
            stream = torch.cuda.current_stream(eq_symbols.device)
        _lib.check(self._lib.srs_amd_pusch_demap_descramble_batch(
            self._h, plan._h, eq_symbols.data_ptr(), eq_noise_vars.data_ptr(), llrs.data_ptr(), llrs.stride(0), n,
            ctypes.c_void_p(stream.cuda_stream)), "pusch_demap_descramble_batch")
        return llrs

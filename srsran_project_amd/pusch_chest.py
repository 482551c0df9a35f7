"""Host-side mirror of srsRAN's PUSCH DM-RS channel estimator over the MI355X
C-ABI (include/srsran_amd/pusch_chest.h).

Reference interface:
  dmrs_pusch_estimator.h:135   estimate(channel_estimate&, dmrs_pusch_estimator_notifier&,
                                        const resource_grid_reader&, const configuration&)
  dmrs_pusch_estimator.h:73    configuration {slot, sequence_config {type, nof_tx_layers, scrambling_id,
                                              n_scid}, scaling, c_prefix, symbols_mask, rb_mask,
                                              first_symbol, nof_symbols, rx_ports}
  port_channel_estimator_average_impl.h:59  (fd_smoothing_strategy, td_interpolation_strategy, compensate_cfo)
Grids: uint32 [ports][14][nof_subc] complex bf16 (host) or torch int32 tensors
[n][ports][14][nof_subc] (device batch); estimates [ports][layers][14][nof_subc].
"""
import ctypes
import enum
from dataclasses import dataclass

import numpy as np

from . import _lib


class FdSmoothingStrategy(enum.IntEnum):
    """port_channel_estimator_fd_smoothing_strategy."""

    none = 0
    mean = 1
    filter = 2


class TdInterpolationStrategy(enum.IntEnum):
    """port_channel_estimator_td_interpolation_strategy."""

    interpolate = 0
    average = 1


class _Config(ctypes.Structure):
    _fields_ = [("numerology", ctypes.c_uint32), ("slot_index", ctypes.c_uint32), ("scrambling_id", ctypes.c_uint32),
                ("n_scid", ctypes.c_uint32), ("nof_tx_layers", ctypes.c_uint32), ("scaling", ctypes.c_float),
                ("symbols_mask", ctypes.c_uint32), ("rb_start", ctypes.c_uint32), ("rb_count", ctypes.c_uint32),
                ("first_symbol", ctypes.c_uint32), ("nof_symbols", ctypes.c_uint32),
                ("fd_smoothing", ctypes.c_int32), ("td_interpolation", ctypes.c_int32),
                ("compensate_cfo", ctypes.c_int32), ("low_papr", ctypes.c_int32), ("n_rs_id", ctypes.c_uint32)]


class ChestPortStats(ctypes.Structure):
    """``srs_amd_chest_port_stats``: the channel_estimate per-port measurements."""

    _fields_ = [("noise_var", ctypes.c_float), ("epre", ctypes.c_float), ("rsrp", ctypes.c_float),
                ("snr", ctypes.c_float), ("time_alignment_s", ctypes.c_float), ("cfo_hz", ctypes.c_float)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


@dataclass
class DmrsPuschEstimatorConfig:
    """dmrs_pusch_estimator::configuration (pseudo-random sequence, DM-RS type 1, contiguous rb_mask)."""

    slot_index: int
    numerology: int
    nof_tx_layers: int
    scrambling_id: int
    n_scid: bool
    scaling: float
    symbols_mask: int
    rb_start: int
    rb_count: int
    first_symbol: int
    nof_symbols: int
    fd_smoothing: FdSmoothingStrategy = FdSmoothingStrategy.filter
    td_interpolation: TdInterpolationStrategy = TdInterpolationStrategy.average
    compensate_cfo: bool = True
    low_papr: bool = False  # transform precoding: low-PAPR sequence of n_rs_id (one layer)
    n_rs_id: int = 0

    def _c(self):
        return _Config(self.numerology, self.slot_index, self.scrambling_id, int(bool(self.n_scid)),
                       self.nof_tx_layers, self.scaling, self.symbols_mask, self.rb_start, self.rb_count,
                       self.first_symbol, self.nof_symbols, int(self.fd_smoothing), int(self.td_interpolation),
                       int(bool(self.compensate_cfo)), int(bool(self.low_papr)), self.n_rs_id)


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_pusch_chest_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_low_papr_length_valid": (c.c_int, [u]),
        "srs_amd_low_papr_sequence": (c.c_int, [P, u, u, u]),
        "srs_amd_pusch_chest_destroy": (None, [P]),
        "srs_amd_pusch_chest_estimate": (c.c_int, [P, c.POINTER(_Config), P, u, u, P, P]),
        "srs_amd_pusch_chest_estimate_batch": (c.c_int, [P, c.POINTER(_Config), P, c.c_uint64, u, u, u, P,
                                                         c.c_uint64, P, P]),
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


def low_papr_sequence(M, u, v=0):
    """low_papr_sequence_generator::generate(sequence, u, v, 0, 1) (include/srsran_amd/low_papr.h): complex64 [M]."""
    import numpy as np

    lib = _L()
    out = np.zeros(M, np.complex64)
    _lib.check(lib.srs_amd_low_papr_sequence(out.ctypes.data, M, u, v), "low_papr_sequence")
    return out


def low_papr_length_valid(M):
    return bool(_L().srs_amd_low_papr_length_valid(M))


class DmrsPuschEstimator:
    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pusch_chest_create(ctypes.byref(h), int(device)), "dmrs_pusch_estimator create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_chest_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def estimate(self, grid, config, estimates=None):
        """grid: uint32 [ports][14][nof_subc]. Returns (estimates uint32 [ports][layers][14][nof_subc],
        list of per-port stats dicts)."""
        g = np.ascontiguousarray(grid, dtype=np.uint32)
        if g.ndim != 3 or g.shape[1] != 14:
            raise ValueError("grid must be [ports][14][nof_subc]")
        P, _, nsubc = g.shape
        L = config.nof_tx_layers
        est = np.zeros((P, L, 14, nsubc), np.uint32) if estimates is None else \
            np.ascontiguousarray(estimates, dtype=np.uint32).copy()
        st = (ChestPortStats * P)()
        c = config._c()
        _lib.check(self._lib.srs_amd_pusch_chest_estimate(self._h, ctypes.byref(c), g.ctypes.data, P, nsubc,
                                                          est.ctypes.data, st), "dmrs_pusch_estimator estimate")
        return est, [s.as_dict() for s in st]

    def estimate_batch(self, grids, config, estimates, stats, stream=None):
        """grids torch int32 [n][ports][14][nof_subc]; estimates torch int32 [n][ports][layers][14][nof_subc];
        stats torch float32 [n][ports][6]."""
        import torch

        n, P, _, nsubc = grids.shape
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        c = config._c()
        _lib.check(self._lib.srs_amd_pusch_chest_estimate_batch(
            self._h, ctypes.byref(c), grids.data_ptr(), grids.stride(0), P, nsubc, n, estimates.data_ptr(),
            estimates.stride(0), stats.data_ptr(), ctypes.c_void_p(stream.cuda_stream)), "estimate_batch")
        return estimates, stats

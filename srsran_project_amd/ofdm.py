"""Host-side mirror of srsRAN's OFDM modulator / demodulator and DFT processor
over the MI355X C-ABI (include/srsran_amd/ofdm.h).

Reference interfaces:
  include/srsran/phy/lower/modulation/ofdm_modulator.h:33   ofdm_modulator_configuration
  include/srsran/phy/lower/modulation/ofdm_modulator.h:98   ofdm_slot_modulator::get_slot_size
  include/srsran/phy/lower/modulation/ofdm_modulator.h:108  ofdm_slot_modulator::modulate(output, grid, port, slot)
  include/srsran/phy/lower/modulation/ofdm_demodulator.h:34, :100, :110  (demodulator counterparts)
  include/srsran/phy/generic_functions/dft_processor.h:48-72  dft_processor {configuration, get_input, run}

Resource grids are complex bfloat16 arrays (uint16 [nsymb, 2*rg], re/im
interleaved, the reference's resource_grid_impl storage); baseband samples are
complex64.  ``*_batch`` methods take torch device tensors.
"""
import ctypes
import enum
from dataclasses import dataclass

import numpy as np

from . import _lib


class OfdmConfig(ctypes.Structure):
    _fields_ = [
        ("numerology", ctypes.c_uint32),
        ("bw_rb", ctypes.c_uint32),
        ("dft_size", ctypes.c_uint32),
        ("cp_extended", ctypes.c_uint32),
        ("nof_samples_window_offset", ctypes.c_uint32),
        ("scale", ctypes.c_float),
        ("center_freq_hz", ctypes.c_double),
    ]


class CyclicPrefix(enum.IntEnum):
    NORMAL = 0
    EXTENDED = 1


class DftDirection(enum.IntEnum):
    """dft_processor::direction (dft_processor.h:36)."""

    DIRECT = 0
    INVERSE = 1


@dataclass
class OfdmModulatorConfiguration:
    numerology: int = 0
    bw_rb: int = 0
    dft_size: int = 0
    cp: CyclicPrefix = CyclicPrefix.NORMAL
    scale: float = 1.0
    center_freq_Hz: float = 0.0

    def to_c(self, window_offset=0):
        return OfdmConfig(int(self.numerology), int(self.bw_rb), int(self.dft_size), int(self.cp), int(window_offset),
                          float(self.scale), float(self.center_freq_Hz))


@dataclass
class OfdmDemodulatorConfiguration(OfdmModulatorConfiguration):
    nof_samples_window_offset: int = 0

    def to_c(self, window_offset=None):
        return super().to_c(self.nof_samples_window_offset)


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_ofdm_modulator_create": (c.c_int, [c.POINTER(P), c.POINTER(OfdmConfig), c.c_int]),
        "srs_amd_ofdm_modulator_destroy": (None, [P]),
        "srs_amd_ofdm_modulator_get_slot_size": (c.c_uint32, [P, c.c_uint32]),
        "srs_amd_ofdm_modulate_slot": (c.c_int, [P, P, P, c.c_uint32]),
        "srs_amd_ofdm_modulate_batch": (c.c_int, [P, P, c.c_uint32, c.c_uint32, c.c_uint32, P, c.c_uint32, P]),
        "srs_amd_ofdm_demodulator_create": (c.c_int, [c.POINTER(P), c.POINTER(OfdmConfig), c.c_int]),
        "srs_amd_ofdm_demodulator_destroy": (None, [P]),
        "srs_amd_ofdm_demodulator_get_slot_size": (c.c_uint32, [P, c.c_uint32]),
        "srs_amd_ofdm_demodulate_slot": (c.c_int, [P, P, P, c.c_uint32]),
        "srs_amd_ofdm_demodulate_batch": (c.c_int, [P, P, c.c_uint32, c.c_uint32, c.c_uint32, c.c_uint32, P, P]),
        "srs_amd_dft_create": (c.c_int, [c.POINTER(P), c.c_uint32, c.c_int, c.c_int]),
        "srs_amd_dft_destroy": (None, [P]),
        "srs_amd_dft_run": (c.c_int, [P, P, P]),
        "srs_amd_dft_run_batch": (c.c_int, [P, P, P, c.c_uint32, P]),
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


def _stream(stream, t):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return ctypes.c_void_p(stream.cuda_stream)


class _Engine:
    _create = _destroy = _slot_size = None

    def __init__(self, config, device=-1):
        self._lib = _L()
        self.config = config
        c = config.to_c()
        h = ctypes.c_void_p()
        _lib.check(getattr(self._lib, self._create)(ctypes.byref(h), ctypes.byref(c), int(device)), self._create)
        self._h = h
        self.nsymb = 12 if int(config.cp) == 1 else 14
        self.rg_size = int(config.bw_rb) * 12

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            getattr(self._lib, self._destroy)(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_slot_size(self, slot_index):
        return int(getattr(self._lib, self._slot_size)(self._h, int(slot_index)))

    @property
    def slots_per_subframe(self):
        return 1 << int(self.config.numerology)

    def max_slot_size(self):
        return max(self.get_slot_size(s) for s in range(self.slots_per_subframe))


class OfdmSlotModulator(_Engine):
    """ofdm_slot_modulator on the MI355X."""

    _create, _destroy = "srs_amd_ofdm_modulator_create", "srs_amd_ofdm_modulator_destroy"
    _slot_size = "srs_amd_ofdm_modulator_get_slot_size"

    def modulate(self, grid: np.ndarray, slot_index: int) -> np.ndarray:
        """grid: uint16 [nsymb, 2*rg] cbf16 of one port; returns complex64 [slot size]."""
        g = np.ascontiguousarray(grid, dtype=np.uint16)
        if g.size != self.nsymb * 2 * self.rg_size:
            raise ValueError("grid must hold %d x %d cbf16 values" % (self.nsymb, self.rg_size))
        n = self.get_slot_size(slot_index)
        if n == 0:
            raise ValueError("invalid slot index %d" % slot_index)
        out = np.zeros(n, np.complex64)
        _lib.check(self._lib.srs_amd_ofdm_modulate_slot(self._h, out.ctypes.data, g.ctypes.data, int(slot_index)),
                   "ofdm modulate")
        return out

    def modulate_batch(self, grid, first_slot=0, out=None, sample_stride=None, stream=None):
        """grid: torch int16/uint16-compatible device tensor [nof_slots, nof_ports, nsymb, 2*rg]
        (cbf16).  Returns complex64 samples [nof_slots, nof_ports, sample_stride]."""
        import torch

        if grid.dim() != 4 or grid.shape[2] != self.nsymb or grid.shape[3] != 2 * self.rg_size:
            raise ValueError("grid must be [nof_slots, nof_ports, %d, %d]" % (self.nsymb, 2 * self.rg_size))
        if not grid.is_contiguous() or grid.element_size() != 2 or not grid.is_cuda:
            raise ValueError("grid must be a contiguous 16-bit device tensor")
        nslots, nports = grid.shape[0], grid.shape[1]
        stride = sample_stride or self.max_slot_size()
        if out is None:
            out = torch.empty((nslots, nports, stride), dtype=torch.complex64, device=grid.device)
        _lib.check(self._lib.srs_amd_ofdm_modulate_batch(self._h, grid.data_ptr(), nports, int(first_slot), nslots,
                                                         out.data_ptr(), out.shape[-1], _stream(stream, grid)),
                   "ofdm modulate_batch")
        return out


class OfdmSlotDemodulator(_Engine):
    """ofdm_slot_demodulator on the MI355X."""

    _create, _destroy = "srs_amd_ofdm_demodulator_create", "srs_amd_ofdm_demodulator_destroy"
    _slot_size = "srs_amd_ofdm_demodulator_get_slot_size"

    def demodulate(self, samples: np.ndarray, slot_index: int) -> np.ndarray:
        """samples: complex64 [slot size]; returns the cbf16 grid uint16 [nsymb, 2*rg]."""
        x = np.ascontiguousarray(samples, dtype=np.complex64)
        n = self.get_slot_size(slot_index)
        if n == 0:
            raise ValueError("invalid slot index %d" % slot_index)
        if x.size != n:
            raise ValueError("The input buffer size (%d) does not match the slot size (%d)" % (x.size, n))
        grid = np.zeros((self.nsymb, 2 * self.rg_size), np.uint16)
        _lib.check(self._lib.srs_amd_ofdm_demodulate_slot(self._h, grid.ctypes.data, x.ctypes.data, int(slot_index)),
                   "ofdm demodulate")
        return grid

    def demodulate_batch(self, samples, first_slot=0, grid=None, stream=None):
        """samples: complex64 device tensor [nof_slots, nof_ports, sample_stride].
        Returns the cbf16 grid int16 [nof_slots, nof_ports, nsymb, 2*rg]."""
        import torch

        if samples.dim() != 3 or samples.dtype != torch.complex64 or not samples.is_cuda:
            raise ValueError("samples must be a complex64 device tensor [nof_slots, nof_ports, stride]")
        nslots, nports, stride = samples.shape
        if grid is None:
            grid = torch.empty((nslots, nports, self.nsymb, 2 * self.rg_size), dtype=torch.int16,
                               device=samples.device)
        _lib.check(self._lib.srs_amd_ofdm_demodulate_batch(self._h, samples.data_ptr(), stride, nports,
                                                           int(first_slot), nslots, grid.data_ptr(),
                                                           _stream(stream, samples)), "ofdm demodulate_batch")
        return grid


class DftProcessor:
    """dft_processor on the MI355X: run() transforms get_input() into the output."""

    def __init__(self, size, direction=DftDirection.DIRECT, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_dft_create(ctypes.byref(h), int(size), int(direction), int(device)),
                   "dft create")
        self._h = h
        self.size = int(size)
        self.direction = DftDirection(direction)
        self._input = np.zeros(self.size, np.complex64)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_dft_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_size(self):
        return self.size

    def get_direction(self):
        return self.direction

    def get_input(self):
        return self._input

    def run(self):
        out = np.zeros(self.size, np.complex64)
        _lib.check(self._lib.srs_amd_dft_run(self._h, out.ctypes.data, self._input.ctypes.data), "dft run")
        return out

    def run_batch(self, x, out=None, stream=None):
        """x: complex64 device tensor [nof, size] (contiguous)."""
        import torch

        if x.dtype != torch.complex64 or not x.is_cuda or not x.is_contiguous() or x.shape[-1] != self.size:
            raise ValueError("input must be a contiguous complex64 device tensor [..., %d]" % self.size)
        if out is None:
            out = torch.empty_like(x)
        _lib.check(self._lib.srs_amd_dft_run_batch(self._h, x.data_ptr(), out.data_ptr(), x.numel() // self.size,
                                                   _stream(stream, x)), "dft run_batch")
        return out


def create_ofdm_modulator_factory_hip():
    class _F:
        def create_ofdm_slot_modulator(self, config, device=-1):
            return OfdmSlotModulator(config, device)

    return _F()


def create_ofdm_demodulator_factory_hip():
    class _F:
        def create_ofdm_slot_demodulator(self, config, device=-1):
            return OfdmSlotDemodulator(config, device)

    return _F()


def create_dft_processor_factory_hip():
    class _F:
        def create(self, size, direction, device=-1):
            return DftProcessor(size, direction, device)

    return _F()

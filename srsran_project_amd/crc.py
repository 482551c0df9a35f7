"""Host-side mirror of srsRAN's CRC calculator over the MI355X C-ABI
(include/srsran_amd/crc.h).

Reference interface (include/srsran/phy/upper/channel_coding/crc_calculator.h):
  :71 calculate_byte(span<const uint8_t> data)   -- whole bytes, MSB first
  :76 calculate_bit(span<const uint8_t> data)    -- one bit per byte
  :81 calculate(const bit_buffer& data)          -- packed bits
  :84 get_generator_poly()
Batch forms compute (or attach) the CRCs of many rows on the device.
"""
import ctypes

import numpy as np

from . import _lib
from .ldpc import CrcGeneratorPoly


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_crc_calculator_create": (c.c_int, [c.POINTER(P), c.c_int, u, c.c_int]),
        "srs_amd_crc_calculator_destroy": (None, [P]),
        "srs_amd_crc_order": (u, [P]),
        "srs_amd_crc_calculate": (c.c_int, [P, c.POINTER(u), P, u]),
        "srs_amd_crc_calculate_batch": (c.c_int, [P, P, P, u, u, u, P]),
        "srs_amd_crc_attach_batch": (c.c_int, [P, P, u, u, u, P]),
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


class CrcCalculator:
    """crc_calculator on the MI355X: ``max_bits`` bounds the message length."""

    def __init__(self, poly, max_bits=1 << 20, device=-1):
        self._lib = _L()
        self.poly = CrcGeneratorPoly(int(poly))
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_crc_calculator_create(ctypes.byref(h), int(self.poly), int(max_bits),
                                                           int(device)), "crc calculator create")
        self._h = h
        self.order = int(self._lib.srs_amd_crc_order(h))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_crc_calculator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_generator_poly(self):
        return self.poly

    def calculate(self, packed, nof_bits):
        b = np.ascontiguousarray(packed, dtype=np.uint8)
        if b.size * 8 < nof_bits:
            raise ValueError("buffer holds fewer than %d bits" % nof_bits)
        r = ctypes.c_uint32()
        _lib.check(self._lib.srs_amd_crc_calculate(self._h, ctypes.byref(r), b.ctypes.data, int(nof_bits)),
                   "crc calculate")
        return int(r.value)

    def calculate_byte(self, data):
        b = np.ascontiguousarray(data, dtype=np.uint8)
        return self.calculate(b, 8 * b.size)

    def calculate_bit(self, bits):
        b = np.ascontiguousarray(bits, dtype=np.uint8)
        return self.calculate(np.packbits(b & 1), b.size)

    def calculate_batch(self, rows, nof_bits, out=None, stream=None):
        """CRCs (uint32 view in an int32 tensor) of each row of a uint8 [rows, stride] tensor."""
        import torch

        if rows.dim() != 2 or rows.dtype != torch.uint8 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous uint8 [rows, stride] tensor")
        if out is None:
            out = torch.empty(rows.shape[0], dtype=torch.int32, device=rows.device)
        _lib.check(self._lib.srs_amd_crc_calculate_batch(self._h, out.data_ptr(), rows.data_ptr(), rows.shape[1],
                                                         int(nof_bits), rows.shape[0], _stream(stream, rows)),
                   "crc calculate_batch")
        return out

    def attach_batch(self, rows, nof_bits, stream=None):
        """Writes each row's CRC into bits [nof_bits, nof_bits + order), in place."""
        import torch

        if rows.dim() != 2 or rows.dtype != torch.uint8 or not rows.is_contiguous():
            raise ValueError("rows must be a contiguous uint8 [rows, stride] tensor")
        _lib.check(self._lib.srs_amd_crc_attach_batch(self._h, rows.data_ptr(), rows.shape[1], int(nof_bits),
                                                      rows.shape[0], _stream(stream, rows)), "crc attach_batch")
        return rows


def create_crc_calculator_factory_hip(device=-1):
    """create_crc_calculator_factory_sw equivalent: a callable poly -> CrcCalculator."""

    def create(poly, max_bits=1 << 20):
        return CrcCalculator(poly, max_bits=max_bits, device=device)

    return create

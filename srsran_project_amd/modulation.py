"""Host-side mirror of srsRAN's modulation mapper, soft demodulation mapper and
pseudo-random (Gold) sequence scrambling over the MI355X C-ABI
(include/srsran_amd/modulation.h).

Reference interfaces:
  modulation_mapper.h:52        modulate(span<cf_t> symbols, const bit_buffer& input, modulation_scheme)
  demodulation_mapper.h:66      demodulate_soft(span<log_likelihood_ratio>, span<const cf_t>, span<const float>,
                                                modulation_scheme)
  pseudo_random_generator.h:54  init(c_init); :79 apply_xor(bit_buffer&, const bit_buffer&);
                                :102 apply_xor(span<log_likelihood_ratio>, span<const log_likelihood_ratio>)
Modulation codes: 0 pi/2-BPSK, 1 BPSK, 2 QPSK, 4 16QAM, 6 64QAM, 8 256QAM.
"""
import ctypes

import numpy as np

from . import _lib

MODULATION = {"pi/2-BPSK": 0, "BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_modulator_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_modulator_destroy": (None, [P]),
        "srs_amd_modulate": (c.c_int, [P, P, P, u, c.c_int]),
        "srs_amd_demodulate_soft": (c.c_int, [P, P, P, P, u, c.c_int]),
        "srs_amd_scramble_bits": (c.c_int, [P, P, P, u, u]),
        "srs_amd_descramble_llrs": (c.c_int, [P, P, P, u, u]),
        "srs_amd_modulate_batch": (c.c_int, [P, P, P, u, c.c_int, P]),
        "srs_amd_demodulate_soft_batch": (c.c_int, [P, P, P, P, u, c.c_int, P]),
        "srs_amd_scramble_bits_batch": (c.c_int, [P, P, P, u, u, P]),
        "srs_amd_descramble_llrs_batch": (c.c_int, [P, P, P, u, u, P]),
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


def _bps(qm):
    return 1 if qm in (0, 1) else qm


def _stream(stream, t):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return ctypes.c_void_p(stream.cuda_stream)


class Modulator:
    """Modulation mapper + soft demodulation mapper + scrambler on the MI355X."""

    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_modulator_create(ctypes.byref(h), int(device)), "modulator create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_modulator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host forms ------------------------------------------------------
    def modulate(self, bits_packed, nof_symbols, qm):
        b = np.ascontiguousarray(bits_packed, dtype=np.uint8)
        if b.size * 8 < nof_symbols * _bps(qm):
            raise ValueError("not enough bits for %d symbols" % nof_symbols)
        out = np.zeros(nof_symbols, np.complex64)
        _lib.check(self._lib.srs_amd_modulate(self._h, out.ctypes.data, b.ctypes.data, int(nof_symbols), int(qm)),
                   "modulate")
        return out

    def demodulate_soft(self, symbols, noise_vars, qm):
        s = np.ascontiguousarray(symbols, dtype=np.complex64)
        nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
        if s.size != nv.size:
            raise ValueError("Inputs symbols and noise_vars must have the same length.")
        out = np.zeros(s.size * _bps(qm), np.int8)
        _lib.check(self._lib.srs_amd_demodulate_soft(self._h, out.ctypes.data, s.ctypes.data, nv.ctypes.data, s.size,
                                                     int(qm)), "demodulate_soft")
        return out

    def scramble_bits(self, bits_packed, nof_bits, c_init):
        b = np.ascontiguousarray(bits_packed, dtype=np.uint8)
        out = np.zeros((nof_bits + 7) // 8, np.uint8)
        _lib.check(self._lib.srs_amd_scramble_bits(self._h, out.ctypes.data, b.ctypes.data, int(nof_bits),
                                                   int(c_init)), "scramble_bits")
        return out

    def descramble_llrs(self, llrs, c_init):
        x = np.ascontiguousarray(llrs, dtype=np.int8)
        out = np.zeros_like(x)
        _lib.check(self._lib.srs_amd_descramble_llrs(self._h, out.ctypes.data, x.ctypes.data, x.size, int(c_init)),
                   "descramble_llrs")
        return out

    # -- device forms ----------------------------------------------------
    def modulate_batch(self, bits, nof_symbols, qm, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty(nof_symbols, dtype=torch.complex64, device=bits.device)
        _lib.check(self._lib.srs_amd_modulate_batch(self._h, out.data_ptr(), bits.data_ptr(), int(nof_symbols),
                                                    int(qm), _stream(stream, bits)), "modulate_batch")
        return out

    def demodulate_soft_batch(self, symbols, noise_vars, qm, out=None, stream=None):
        import torch

        n = symbols.numel()
        if out is None:
            out = torch.empty(n * _bps(qm), dtype=torch.int8, device=symbols.device)
        _lib.check(self._lib.srs_amd_demodulate_soft_batch(self._h, out.data_ptr(), symbols.data_ptr(),
                                                           noise_vars.data_ptr(), n, int(qm),
                                                           _stream(stream, symbols)), "demodulate_soft_batch")
        return out

    def scramble_bits_batch(self, bits, nof_bits, c_init, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty((nof_bits + 7) // 8, dtype=torch.uint8, device=bits.device)
        _lib.check(self._lib.srs_amd_scramble_bits_batch(self._h, out.data_ptr(), bits.data_ptr(), int(nof_bits),
                                                         int(c_init), _stream(stream, bits)), "scramble_bits_batch")
        return out

    def descramble_llrs_batch(self, llrs, c_init, out=None, stream=None):
        import torch

        if out is None:
            out = torch.empty_like(llrs)
        _lib.check(self._lib.srs_amd_descramble_llrs_batch(self._h, out.data_ptr(), llrs.data_ptr(), llrs.numel(),
                                                           int(c_init), _stream(stream, llrs)),
                   "descramble_llrs_batch")
        return out

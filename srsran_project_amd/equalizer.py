"""Host-side mirror of srsRAN's channel_equalizer over the MI355X C-ABI
(include/srsran_amd/equalizer.h).

Reference interface: include/srsran/phy/upper/equalization/channel_equalizer.h:65-95
  bool is_supported(nof_ports, nof_layers)
  void equalize(eq_symbols, eq_noise_vars, ch_symbols, ch_estimates, noise_var_estimates, tx_scaling)
and create_channel_equalizer_generic_factory(type) (equalization_factories.cpp:47).

Arrays: ch_symbols uint16 [ports, 2*nof_re] (cbf16), ch_estimates uint16
[layers, ports, 2*nof_re], outputs complex64 [nof_re, layers] and float32
[nof_re, layers].
"""
import ctypes
import enum

import numpy as np

from . import _lib


class ChannelEqualizerAlgorithmType(enum.IntEnum):
    """channel_equalizer_algorithm_type (channel_equalizer_algorithm_type.h)."""

    zf = 0
    mmse = 1


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_channel_equalizer_create": (c.c_int, [c.POINTER(P), c.c_int, c.c_int]),
        "srs_amd_channel_equalizer_destroy": (None, [P]),
        "srs_amd_channel_equalizer_is_supported": (c.c_int, [P, c.c_uint32, c.c_uint32]),
        "srs_amd_channel_equalize": (c.c_int, [P, P, P, P, P, P, c.c_uint32, c.c_uint32, c.c_uint32, c.c_float]),
        "srs_amd_channel_equalize_batch": (
            c.c_int, [P, P, P, P, P, P, c.c_uint32, c.c_uint32, c.c_uint32, c.c_float, P]),
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


class ChannelEqualizer:
    def __init__(self, algorithm=ChannelEqualizerAlgorithmType.zf, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_channel_equalizer_create(ctypes.byref(h), int(algorithm), int(device)),
                   "channel_equalizer create")
        self._h = h
        self.algorithm = ChannelEqualizerAlgorithmType(algorithm)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_channel_equalizer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def is_supported(self, nof_ports, nof_layers):
        return bool(self._lib.srs_amd_channel_equalizer_is_supported(self._h, int(nof_ports), int(nof_layers)))

    def equalize(self, ch_symbols, ch_estimates, noise_var_estimates, tx_scaling=1.0):
        """Returns (eq_symbols complex64 [nof_re, layers], eq_noise_vars float32 [nof_re, layers])."""
        s = np.ascontiguousarray(ch_symbols, dtype=np.uint16)
        h = np.ascontiguousarray(ch_estimates, dtype=np.uint16)
        nv = np.ascontiguousarray(noise_var_estimates, dtype=np.float32)
        if s.ndim != 2 or h.ndim != 3 or h.shape[1:] != s.shape or nv.size != s.shape[0]:
            raise ValueError("inconsistent equalizer input dimensions")
        ports, re2 = s.shape
        layers = h.shape[0]
        nre = re2 // 2
        eq = np.zeros((nre, layers), np.complex64)
        nvo = np.zeros((nre, layers), np.float32)
        _lib.check(self._lib.srs_amd_channel_equalize(self._h, eq.ctypes.data, nvo.ctypes.data, s.ctypes.data,
                                                      h.ctypes.data, nv.ctypes.data, nre, ports, layers,
                                                      float(tx_scaling)), "equalize")
        return eq, nvo

    def equalize_batch(self, ch_symbols, ch_estimates, noise_var_estimates, tx_scaling=1.0, eq=None, nvo=None,
                       stream=None):
        """Device tensors: ch_symbols int16 [ports, 2*nof_re], ch_estimates int16
        [layers, ports, 2*nof_re]; noise_var_estimates a host sequence."""
        import torch

        ports, re2 = ch_symbols.shape
        layers = ch_estimates.shape[0]
        nre = re2 // 2
        if eq is None:
            eq = torch.empty((nre, layers), dtype=torch.complex64, device=ch_symbols.device)
        if nvo is None:
            nvo = torch.empty((nre, layers), dtype=torch.float32, device=ch_symbols.device)
        nv = np.ascontiguousarray(noise_var_estimates, dtype=np.float32)
        if stream is None:
            stream = torch.cuda.current_stream(ch_symbols.device)
        _lib.check(self._lib.srs_amd_channel_equalize_batch(
            self._h, eq.data_ptr(), nvo.data_ptr(), ch_symbols.data_ptr(), ch_estimates.data_ptr(), nv.ctypes.data,
            nre, ports, layers, float(tx_scaling), ctypes.c_void_p(stream.cuda_stream)), "equalize_batch")
        return eq, nvo


def create_channel_equalizer_generic_factory_hip(algorithm=ChannelEqualizerAlgorithmType.zf):
    class _F:
        def create(self, device=-1):
            return ChannelEqualizer(algorithm, device)

    return _F()

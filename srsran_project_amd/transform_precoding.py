"""Host-side mirror of srsRAN's transform precoder (DFT-s-OFDM PUSCH) over the MI355X C-ABI
(include/srsran_amd/transform_precoding.h).

Reference interfaces:
  transform_precoder.h:55   deprecode_ofdm_symbol(span<cf_t> out, span<const cf_t> in)
  transform_precoder.h:63   deprecode_ofdm_symbol_noise(span<float> out, span<const float> in)
  transform_precoding_helpers.h:64   is_nof_prbs_valid(unsigned nof_prb)
"""
import ctypes

import numpy as np

from . import _lib

_declared = False


def _L():
    global _declared
    lib = _lib.lib()
    if not _declared:
        c, P, u = ctypes, ctypes.c_void_p, ctypes.c_uint32
        for name, res, args in [
            ("srs_amd_transform_precoder_create", c.c_int, [c.POINTER(P), c.c_int]),
            ("srs_amd_transform_precoder_destroy", None, [P]),
            ("srs_amd_transform_precoding_nof_prbs_valid", c.c_int, [u]),
            ("srs_amd_transform_deprecode", c.c_int, [P, P, P, u]),
            ("srs_amd_transform_deprecode_noise", c.c_int, [P, P, P, u]),
            ("srs_amd_transform_deprecode_batch", c.c_int, [P, P, c.c_uint64, P, c.c_uint64, u, u, P]),
        ]:
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _declared = True
    return lib


def is_nof_prbs_valid(nof_prb):
    """transform_precoding::is_nof_prbs_valid (host only)."""
    return bool(_L().srs_amd_transform_precoding_nof_prbs_valid(int(nof_prb)))


class TransformPrecoder:
    """``transform_precoder`` (transform_precoder_dft_impl) on the GPU."""

    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_transform_precoder_create(ctypes.byref(h), int(device)),
                   "transform precoder create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.srs_amd_transform_precoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def deprecode_ofdm_symbol(self, symbols):
        """Host form: complex64 [M] -> complex64 [M]."""
        x = np.ascontiguousarray(symbols, np.complex64)
        out = np.empty_like(x)
        _lib.check(self._lib.srs_amd_transform_deprecode(self._h, out.ctypes.data, x.ctypes.data, x.size),
                   "transform deprecode")
        return out

    def deprecode_ofdm_symbol_noise(self, noise_vars):
        x = np.ascontiguousarray(noise_vars, np.float32)
        out = np.empty_like(x)
        _lib.check(self._lib.srs_amd_transform_deprecode_noise(self._h, out.ctypes.data, x.ctypes.data, x.size),
                   "transform deprecode noise")
        return out

    def deprecode_batch(self, symbols, noise_vars=None, nof_subc=None, stream=None):
        """Device form, in place: complex64 [rows, stride] symbols (the first nof_subc of each row, default the
        whole row) and optional float32 [rows, stride] noise variances."""
        import torch

        if symbols.dim() != 2 or symbols.dtype != torch.complex64 or not symbols.is_contiguous():
            raise ValueError("symbols must be a contiguous complex64 [rows, stride] tensor")
        M = symbols.shape[1] if nof_subc is None else int(nof_subc)
        nv_ptr, nv_stride = None, 0
        if noise_vars is not None:
            if noise_vars.dtype != torch.float32 or not noise_vars.is_contiguous() or noise_vars.shape[0] != symbols.shape[0]:
                raise ValueError("noise_vars must be a contiguous float32 [rows, stride] tensor")
            nv_ptr, nv_stride = noise_vars.data_ptr(), noise_vars.shape[1]
        if stream is None:
            stream = torch.cuda.current_stream(symbols.device)
        _lib.check(self._lib.srs_amd_transform_deprecode_batch(
            self._h, symbols.data_ptr(), symbols.shape[1], nv_ptr, nv_stride, M, symbols.shape[0],
            ctypes.c_void_p(stream.cuda_stream)), "transform deprecode batch")
        return symbols, noise_vars

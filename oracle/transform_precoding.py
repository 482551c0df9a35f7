"""CPU oracle of the transform deprecoder (DFT-s-OFDM PUSCH) -- TEST INFRASTRUCTURE ONLY.

Restatement of transform_precoder_dft_impl.cpp:31-84: deprecode_ofdm_symbol is the inverse M-point DFT
scaled by 1/sqrt(M) (x[k] = M^-1/2 sum_n y[n] exp(+j 2 pi n k / M), M = 12 M_rb), computed here in
float64; deprecode_ofdm_symbol_noise replaces every valid (positive, finite) noise variance of the symbol
by their mean.  is_nof_prbs_valid (transform_precoding_helpers.h:64): M_rb = 2^a 3^b 5^c, M_rb <= 275.

Pinned: the `ref_*` functions run the reference's own transform_precoder_dft_impl (oracle/ref_wrapper_tp.cpp,
generic float DFT) on the same inputs; tests/test_oracle_vs_ref.py checks the restatement against them.
"""
import ctypes as _c

import numpy as np

from . import REF, _ptr

MAX_NOF_PRBS = 275


def nof_prbs_valid(n):
    if n < 1 or n > MAX_NOF_PRBS:
        return False
    for f in (2, 3, 5):
        while n % f == 0:
            n //= f
    return n == 1


def deprecode(y):
    y = np.asarray(y, np.complex128)
    M = y.size
    return np.fft.ifft(y) * (M / np.sqrt(M))


def deprecode_noise(nv):
    nv = np.asarray(nv, np.float32)
    valid = (nv > 0) & np.isfinite(nv)
    mean = np.float32(nv[valid].astype(np.float64).mean()) if valid.any() else np.float32(0)
    return np.where(valid, mean, nv).astype(np.float32)


def _need_ref():
    if REF is None:
        raise RuntimeError("oracle/_ref not built")
    REF.srs_ref_transform_deprecode.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint]
    REF.srs_ref_transform_deprecode_noise.argtypes = [_c.c_void_p, _c.c_void_p, _c.c_uint]


def ref_deprecode(y):
    _need_ref()
    x = np.ascontiguousarray(np.asarray(y, np.complex64))
    out = np.zeros_like(x)
    if REF.srs_ref_transform_deprecode(_ptr(out), _ptr(x), x.size) != 0:
        raise ValueError("invalid transform precoding size %d" % x.size)
    return out


def ref_deprecode_noise(nv):
    _need_ref()
    x = np.ascontiguousarray(nv, np.float32)
    out = np.zeros_like(x)
    REF.srs_ref_transform_deprecode_noise(_ptr(out), _ptr(x), x.size)
    return out


def ref_nof_prbs_valid(n):
    _need_ref()
    return bool(REF.srs_ref_transform_nof_prbs_valid(int(n)))

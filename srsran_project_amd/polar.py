"""Host-side mirror of srsRAN's polar coding objects over the MI355X C-ABI
(include/srsran_amd/polar.h).

Reference interfaces (include/srsran/phy/upper/channel_coding/polar/):
  polar_code.h:110  set(K, E, nMax, ibil); get_N / get_n / get_nPC / get_K_set / get_PC_set
  the encode chain of pdcch_encoder_impl (allocator -> encoder -> rate matcher)
  the decode chain of the UCI decoder (rate dematcher -> decoder -> deallocator)
  polar_interleaver.h  interleave(out, in, direction)
Bits are uint8 0/1 arrays, LLRs int8 arrays; *_batch take torch device tensors.
"""
import ctypes
import enum

import numpy as np

from . import _lib


class PolarCodeIbil(enum.IntEnum):
    not_present = 0
    present = 1


class PolarInterleaverDirection(enum.IntEnum):
    tx = 0
    rx = 1


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_polar_code_create": (c.c_int, [c.POINTER(P), c.c_uint32, c.c_uint32, c.c_uint32, c.c_int, c.c_int]),
        "srs_amd_polar_code_destroy": (None, [P]),
        "srs_amd_polar_code_get_N": (c.c_uint32, [P]),
        "srs_amd_polar_code_get_n": (c.c_uint32, [P]),
        "srs_amd_polar_code_get_nPC": (c.c_uint32, [P]),
        "srs_amd_polar_code_get_K_set": (c.c_int, [P, P]),
        "srs_amd_polar_code_get_PC_set": (c.c_int, [P, P]),
        "srs_amd_polar_code_construct": (c.c_uint32, [c.c_uint32, c.c_uint32, c.c_uint32, P, P, c.POINTER(c.c_uint32)]),
        "srs_amd_polar_encode": (c.c_int, [P, P, P]),
        "srs_amd_polar_decode": (c.c_int, [P, P, P]),
        "srs_amd_polar_encode_batch": (c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_polar_decode_batch": (c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_polar_interleave": (c.c_int, [P, P, c.c_uint32, c.c_int]),
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


def polar_code_construct(K, E, nMax):
    """Host-only polar_code::set: (N, K_set mask uint8 [N], PC set uint16 [nPC])."""
    lib = _L()
    mask = np.zeros(1024, np.uint8)
    pc = np.zeros(8, np.uint16)
    npc = ctypes.c_uint32(0)
    N = lib.srs_amd_polar_code_construct(int(K), int(E), int(nMax), mask.ctypes.data, pc.ctypes.data,
                                         ctypes.byref(npc))
    if N == 0:
        raise ValueError(lib.srs_amd_last_error().decode())
    return N, mask[:N].copy(), pc[:npc.value].copy()


class PolarCode:
    """A constructed polar code with its device tables (polar_code on the MI355X)."""

    def __init__(self, K, E, nMax, ibil=PolarCodeIbil.not_present, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_polar_code_create(ctypes.byref(h), int(K), int(E), int(nMax), int(ibil),
                                                       int(device)), "polar_code set")
        self._h = h
        self.K, self.E, self.nMax, self.ibil = int(K), int(E), int(nMax), PolarCodeIbil(ibil)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_polar_code_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_N(self):
        return int(self._lib.srs_amd_polar_code_get_N(self._h))

    def get_n(self):
        return int(self._lib.srs_amd_polar_code_get_n(self._h))

    def get_nPC(self):
        return int(self._lib.srs_amd_polar_code_get_nPC(self._h))

    def get_K_set(self):
        m = np.zeros(self.get_N(), np.uint8)
        _lib.check(self._lib.srs_amd_polar_code_get_K_set(self._h, m.ctypes.data))
        return m

    def get_PC_set(self):
        p = np.zeros(max(self.get_nPC(), 1), np.uint16)
        _lib.check(self._lib.srs_amd_polar_code_get_PC_set(self._h, p.ctypes.data))
        return p[:self.get_nPC()]

    def encode(self, message):
        msg = np.ascontiguousarray(message, dtype=np.uint8)
        if msg.size != self.K:
            raise ValueError("message must hold K=%d bits" % self.K)
        out = np.zeros(self.E, np.uint8)
        _lib.check(self._lib.srs_amd_polar_encode(self._h, out.ctypes.data, msg.ctypes.data), "polar encode")
        return out

    def decode(self, llrs):
        x = np.ascontiguousarray(llrs, dtype=np.int8)
        if x.size != self.E:
            raise ValueError("input must hold E=%d LLRs" % self.E)
        msg = np.zeros(self.K, np.uint8)
        _lib.check(self._lib.srs_amd_polar_decode(self._h, msg.ctypes.data, x.ctypes.data), "polar decode")
        return msg

    def encode_batch(self, messages, out=None, stream=None):
        import torch

        n = messages.shape[0]
        if out is None:
            out = torch.empty((n, self.E), dtype=torch.uint8, device=messages.device)
        if stream is None:
            stream = torch.cuda.current_stream(messages.device)
        _lib.check(self._lib.srs_amd_polar_encode_batch(self._h, messages.data_ptr(), messages.stride(0),
                                                        out.data_ptr(), out.stride(0), n,
                                                        ctypes.c_void_p(stream.cuda_stream)), "polar encode_batch")
        return out

    def decode_batch(self, llrs, out=None, stream=None):
        import torch

        n = llrs.shape[0]
        if out is None:
            out = torch.empty((n, self.K), dtype=torch.uint8, device=llrs.device)
        if stream is None:
            stream = torch.cuda.current_stream(llrs.device)
        _lib.check(self._lib.srs_amd_polar_decode_batch(self._h, llrs.data_ptr(), llrs.stride(0), out.data_ptr(),
                                                        out.stride(0), n, ctypes.c_void_p(stream.cuda_stream)),
                   "polar decode_batch")
        return out


def polar_interleave(bits, direction=PolarInterleaverDirection.tx):
    lib = _L()
    b = np.ascontiguousarray(bits, dtype=np.uint8)
    out = np.zeros_like(b)
    _lib.check(lib.srs_amd_polar_interleave(out.ctypes.data, b.ctypes.data, b.size, int(direction)),
               "polar interleave")
    return out

"""Host mirror of the MI355X UCI decoder (include/srsran_amd/uci_decoder.h):
uci_decoder::decode (include/srsran/phy/upper/channel_processors/uci/uci_decoder.h:59)."""
import ctypes

import numpy as np

from . import _lib

UCI_UNKNOWN, UCI_VALID, UCI_INVALID = 0, 1, 2


class UciDecoder:
    def __init__(self, device=-1):
        lib = _lib.lib()
        c = ctypes
        P = c.c_void_p
        for name, res, args in (
                ("srs_amd_uci_decoder_create", c.c_int, [c.POINTER(P), c.c_int]),
                ("srs_amd_uci_decoder_destroy", None, [P]),
                ("srs_amd_uci_decode", c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.c_int32]),
                ("srs_amd_uci_decode_batch", c.c_int, [P, P, c.c_uint64, c.c_uint32, c.c_uint32, c.c_int32, P,
                                                       c.c_uint64, P, c.c_uint64, c.c_uint32, P])):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        self._lib = lib
        h = ctypes.c_void_p()
        _lib.check(lib.srs_amd_uci_decoder_create(ctypes.byref(h), int(device)), "uci_decoder create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_uci_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, llrs, K, modulation):
        """Host: int8 LLRs -> (message bits uint8 [K], status)."""
        x = np.ascontiguousarray(llrs, np.int8)
        msg = np.zeros(K, np.uint8)
        rc = self._lib.srs_amd_uci_decode(self._h, msg.ctypes.data, K, x.ctypes.data, x.size, modulation)
        if rc < 0:
            _lib.check(rc, "uci_decode")
        return msg, rc

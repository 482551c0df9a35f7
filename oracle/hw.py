"""TEST INFRASTRUCTURE: the reference's hardware-accelerated PUSCH decoder (pusch_decoder_hw_impl, compiled from
/root/reference) driving the MI355X plug-in (integration/hip_accelerator_pusch_dec.cpp) -- oracle/hw_harness.cpp,
built into oracle/_ref/libsrsran_ref_hw.so.  Loading it initialises the GPU (the plug-in allocates its HARQ
buffers in HBM), so only GPU tests use it."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
HW_PATH = os.path.join(_HERE, "_ref", "libsrsran_ref_hw.so")
HAL_PATH = os.path.join(_HERE, "..", "integration", "_build", "libsrsran_amd_hal.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(HW_PATH):
            raise ImportError("oracle/_ref/libsrsran_ref_hw.so not built (make -C integration && make -C oracle)")
        L = ctypes.CDLL(HW_PATH)
        P, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        L.srs_ref_hw_ctx_create.restype = P
        L.srs_ref_hw_ctx_create.argtypes = [i, i]
        L.srs_ref_hw_ctx_destroy.argtypes = [P]
        L.srs_ref_hw_ctx_sibling.restype = P
        L.srs_ref_hw_ctx_sibling.argtypes = [P, i]
        L.srs_ref_hw_rx_buffer_create.restype = P
        L.srs_ref_hw_rx_buffer_create.argtypes = [u, u]
        L.srs_ref_hw_rx_buffer_destroy.argtypes = [P]
        L.srs_ref_hw_pusch_decode.restype = i
        L.srs_ref_hw_pusch_decode.argtypes = [P, P, P, u, P, u] + [u] * 6 + [i, i, P]
        _lib = L
    return _lib


class HwPuschDecoder:
    """pusch_decoder_hw_impl + the MI355X hal::hw_accelerator_pusch_dec (external HARQ in HBM)."""

    def __init__(self, device=0, generic=False, sibling_of=None):
        if sibling_of is not None:  # another accelerator of the same factory (shared HBM HARQ pool)
            self.h = lib().srs_ref_hw_ctx_sibling(sibling_of.h, int(generic))
            self._base = sibling_of  # keeps the factory's owner alive
        else:
            self.h = lib().srs_ref_hw_ctx_create(int(device), int(generic))

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_hw_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HwRxBuffer:
    """rx_buffer of one HARQ process; its codeblocks have absolute ids abs_base + index (HARQ rows in HBM)."""

    def __init__(self, nof_cbs, abs_base):
        self.h = lib().srs_ref_hw_rx_buffer_create(int(nof_cbs), int(abs_base))

    def __del__(self):
        if getattr(self, "h", None):
            lib().srs_ref_hw_rx_buffer_destroy(self.h)
            self.h = None


def hw_pusch_decode(dec, llrs, p, rxbuf, tb_out, max_iterations=6, use_early_stop=True, new_data=True):
    """Returns (tb_crc_ok, nof_cbs, nof_obs, iteration sum, min, max), as oracle.ref_pusch_decode."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    res = np.zeros(6, np.float64)
    r = lib().srs_ref_hw_pusch_decode(dec.h, rxbuf.h, llrs.ctypes.data, llrs.size, tb_out.ctypes.data, tb_out.size,
                                      p["base_graph"], p["rv"], p["modulation_order"], p["Nref"], p["nof_layers"],
                                      max_iterations, int(use_early_stop), int(new_data), res.ctypes.data)
    if r != 0:
        raise RuntimeError("pusch_decoder_hw_impl did not notify")
    return bool(res[0]), int(res[1]), int(res[2]), int(round(res[3])), int(res[4]), int(res[5])

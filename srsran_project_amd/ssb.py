"""Host-side mirror of srsRAN's SS/PBCH block processor over the MI355X C-ABI (include/srsran_amd/ssb.h).

Reference interface: ssb_processor::process(resource_grid_writer&, const pdu_t&)
(include/srsran/phy/upper/channel_processors/ssb/ssb_processor.h:77, impl ssb_processor_impl.cpp:29-109) and its pdu_t
(ssb_processor.h:33-62; the slot_point as numerology, SFN and slot index in the frame).  Grids are cbf16
[port][14][nof_subc]: numpy uint32 for the host form, torch int32 [n][port][14][nof_subc] on the device for the slot
form.
"""
import ctypes
import enum

import numpy as np

from . import _lib

MIB_BITS = 24


class SsbPatternCase(enum.IntEnum):
    """ssb_pattern_case (include/srsran/ran/ssb/ssb_properties.h:45-57)."""
    A = 0
    B = 1
    C = 2
    D = 3
    E = 4


class SsbPdu(ctypes.Structure):
    _fields_ = [("numerology", ctypes.c_uint32), ("sfn", ctypes.c_uint32), ("slot_index", ctypes.c_uint32),
                ("phys_cell_id", ctypes.c_uint32), ("beta_pss_dB", ctypes.c_float), ("ssb_idx", ctypes.c_uint32),
                ("L_max", ctypes.c_uint32), ("common_scs", ctypes.c_uint32), ("subcarrier_offset", ctypes.c_uint32),
                ("offset_to_pointA", ctypes.c_uint32), ("pattern_case", ctypes.c_uint32),
                ("mib_payload", ctypes.c_uint8 * MIB_BITS), ("nof_ports", ctypes.c_uint32),
                ("ports", ctypes.c_uint8 * 4), ("grid", ctypes.c_uint32), ("d_grid", ctypes.c_void_p)]


def make_pdu(mib, *, numerology=0, sfn=0, slot_index=0, phys_cell_id=1, beta_pss_dB=0.0, ssb_idx=0, L_max=4,
             common_scs=0, subcarrier_offset=0, offset_to_pointA=0, pattern_case=SsbPatternCase.A, ports=(0,), grid=0):
    """ssb_processor::pdu_t; mib: the 24 MIB bits (one per element)."""
    p = SsbPdu()
    p.numerology, p.sfn, p.slot_index = int(numerology), int(sfn), int(slot_index)
    p.phys_cell_id, p.beta_pss_dB, p.ssb_idx, p.L_max = int(phys_cell_id), float(beta_pss_dB), int(ssb_idx), int(L_max)
    p.common_scs, p.subcarrier_offset, p.offset_to_pointA = int(common_scs), int(subcarrier_offset), int(offset_to_pointA)
    p.pattern_case = int(pattern_case)
    bits = np.asarray(mib, np.uint8)
    if bits.size != MIB_BITS:
        raise ValueError("the MIB payload has %d bits" % MIB_BITS)
    ctypes.memmove(p.mib_payload, bits.ctypes.data, MIB_BITS)
    if not 1 <= len(ports) <= 4:
        raise ValueError("1 to 4 ports")
    p.nof_ports = len(ports)
    for i, q in enumerate(ports):
        p.ports[i] = int(q)
    p.grid = int(grid)
    return p


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_ssb_processor_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_ssb_processor_destroy": (None, [P]),
        "srs_amd_ssb_position": (c.c_int, [P, P, P]),
        "srs_amd_ssb_process_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32, c.c_uint32,
                                               P]),
        "srs_amd_ssb_process": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32]),
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


def position(pdu):
    """(first OFDM symbol in the slot, first subcarrier) of the block; ValueError with the reference's assertion
    message for a PDU the reference cannot process."""
    l0, k0 = ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(_L().srs_amd_ssb_position(ctypes.byref(pdu), ctypes.byref(l0), ctypes.byref(k0)), "ssb position")
    return l0.value, k0.value


class SsbProcessor:
    """ssb_processor on the MI355X (one per device; thread-safe)."""

    def __init__(self, device=0):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_ssb_processor_create(ctypes.byref(h), int(device)), "ssb_processor create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_ssb_processor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdu):
        """ssb_processor::process onto a host grid (numpy uint32 [ports][14][nof_subc], modified in place)."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        _lib.check(self._lib.srs_amd_ssb_process(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                 grid.shape[2]), "ssb process")
        return grid

    def process_slot(self, grids, pdus, stream=None):
        """Every block of a slot onto device grids (torch int32 [n][ports][14][nof_subc]), asynchronous on stream."""
        import torch

        arr = (SsbPdu * len(pdus))(*pdus)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_ssb_process_slot(
            self._h, arr, len(pdus), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[1],
            grids.shape[-1], ctypes.c_void_p(stream.cuda_stream)), "ssb process_slot")
        return grids

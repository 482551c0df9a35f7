"""Host-side mirror of srsRAN's PDCCH processor over the MI355X C-ABI (include/srsran_amd/pdcch.h).

Reference interface: pdcch_processor::process(resource_grid_writer&, const pdu_t&)
(include/srsran/phy/upper/channel_processors/pdcch/pdcch_processor.h:129, impl pdcch_processor_impl.cpp:79-130), its
pdu_t / coreset_description / dci_description (pdcch_processor.h:55-121) and the validator's checks
(pdcch_processor_validator_impl.cpp:27-85).  Grids are cbf16 [port][14][nof_subc]: numpy uint32 (or uint16 pairs)
for the host form, torch int32 [n][port][14][nof_subc] on the device for the slot form.
"""
import ctypes
import enum

import numpy as np

from . import _lib

MAX_PAYLOAD = 128
CRB_MASK_BYTES = 35


class CceToRegMapping(enum.IntEnum):
    """pdcch_processor::cce_to_reg_mapping_type (pdcch_processor.h:79-86)."""
    CORESET0 = 0
    NON_INTERLEAVED = 1
    INTERLEAVED = 2


class PdcchCoreset(ctypes.Structure):
    _fields_ = [("bwp_size_rb", ctypes.c_uint32), ("bwp_start_rb", ctypes.c_uint32),
                ("start_symbol_index", ctypes.c_uint32), ("duration", ctypes.c_uint32),
                ("frequency_resources", ctypes.c_uint8 * 8), ("cce_to_reg_mapping", ctypes.c_uint32),
                ("reg_bundle_size", ctypes.c_uint32), ("interleaver_size", ctypes.c_uint32),
                ("shift_index", ctypes.c_uint32)]


class PdcchDci(ctypes.Structure):
    _fields_ = [("rnti", ctypes.c_uint32), ("n_id_pdcch_dmrs", ctypes.c_uint32), ("n_id_pdcch_data", ctypes.c_uint32),
                ("n_rnti", ctypes.c_uint32), ("cce_index", ctypes.c_uint32), ("aggregation_level", ctypes.c_uint32),
                ("dmrs_power_offset_dB", ctypes.c_float), ("data_power_offset_dB", ctypes.c_float),
                ("payload_size", ctypes.c_uint32), ("payload", ctypes.c_uint8 * MAX_PAYLOAD),
                ("nof_ports", ctypes.c_uint32), ("weights", (ctypes.c_float * 2) * 4)]


class PdcchPdu(ctypes.Structure):
    _fields_ = [("numerology", ctypes.c_uint32), ("slot_index", ctypes.c_uint32), ("coreset", PdcchCoreset),
                ("dci", PdcchDci), ("grid", ctypes.c_uint32), ("d_grid", ctypes.c_void_p)]


def make_pdu(payload, *, numerology=0, slot_index=0, bwp_size_rb=52, bwp_start_rb=0, start_symbol_index=0,
             duration=1, frequency_resources=None, cce_to_reg_mapping=CceToRegMapping.NON_INTERLEAVED,
             reg_bundle_size=6, interleaver_size=2, shift_index=0, rnti=0x4601, n_id_pdcch_dmrs=1, n_id_pdcch_data=1,
             n_rnti=0, cce_index=0, aggregation_level=1, dmrs_power_offset_dB=0.0, data_power_offset_dB=0.0,
             weights=(1.0,), grid=0):
    """pdcch_processor::pdu_t.  frequency_resources: iterable of the set six-RB group indices (default: every group
    of the BWP); weights: the layer's complex weight per port (wideband, one layer)."""
    p = PdcchPdu()
    p.numerology, p.slot_index = int(numerology), int(slot_index)
    c = p.coreset
    c.bwp_size_rb, c.bwp_start_rb = int(bwp_size_rb), int(bwp_start_rb)
    c.start_symbol_index, c.duration = int(start_symbol_index), int(duration)
    groups = range(min(int(bwp_size_rb) // 6, 45)) if frequency_resources is None else frequency_resources
    for g in groups:
        c.frequency_resources[g // 8] |= 1 << (g % 8)
    c.cce_to_reg_mapping = int(cce_to_reg_mapping)
    c.reg_bundle_size, c.interleaver_size, c.shift_index = int(reg_bundle_size), int(interleaver_size), int(shift_index)
    d = p.dci
    d.rnti, d.n_id_pdcch_dmrs, d.n_id_pdcch_data, d.n_rnti = int(rnti), int(n_id_pdcch_dmrs), int(n_id_pdcch_data), int(n_rnti)
    d.cce_index, d.aggregation_level = int(cce_index), int(aggregation_level)
    d.dmrs_power_offset_dB, d.data_power_offset_dB = float(dmrs_power_offset_dB), float(data_power_offset_dB)
    bits = np.asarray(payload, np.uint8)
    if bits.size > MAX_PAYLOAD:
        raise ValueError("DCI payload of %d bits exceeds %d" % (bits.size, MAX_PAYLOAD))
    d.payload_size = bits.size
    ctypes.memmove(d.payload, bits.ctypes.data, bits.size)
    w = np.asarray(weights, np.complex64).ravel()
    d.nof_ports = w.size
    for a, v in enumerate(w):
        d.weights[a][0], d.weights[a][1] = float(v.real), float(v.imag)
    p.grid = int(grid)
    return p


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_pdcch_processor_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_pdcch_processor_destroy": (None, [P]),
        "srs_amd_pdcch_rb_mask": (c.c_int, [P, P]),
        "srs_amd_pdcch_process_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32, P]),
        "srs_amd_pdcch_process": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32]),
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


def rb_mask(pdu):
    """pdcch_processor_impl::compute_rb_mask: the DCI's CRBs (sorted int array); ValueError on an invalid PDU."""
    mask = np.zeros(CRB_MASK_BYTES, np.uint8)
    n = _L().srs_amd_pdcch_rb_mask(ctypes.byref(pdu), mask.ctypes.data)
    if n < 0:
        _lib.check(n, "pdcch rb_mask")
    return np.flatnonzero(np.unpackbits(mask, bitorder="little"))


class PdcchProcessor:
    """pdcch_processor on the MI355X (one per device; thread-safe)."""

    def __init__(self, device=0):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pdcch_processor_create(ctypes.byref(h), int(device)), "pdcch_processor create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pdcch_processor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdu):
        """pdcch_processor::process onto a host grid (numpy uint32 [ports][14][nof_subc], modified in place)."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        _lib.check(self._lib.srs_amd_pdcch_process(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                   grid.shape[2]), "pdcch process")
        return grid

    def process_slot(self, grids, pdus, stream=None):
        """Every PDU of a slot onto device grids (torch int32 [n][ports][14][nof_subc]), asynchronous on stream."""
        import torch

        arr = (PdcchPdu * len(pdus))(*pdus)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pdcch_process_slot(
            self._h, arr, len(pdus), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[-1],
            ctypes.c_void_p(stream.cuda_stream)), "pdcch process_slot")
        return grids

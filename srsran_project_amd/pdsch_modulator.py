"""Host-side mirror of srsRAN's PDSCH modulator and PDSCH DM-RS processor over
the MI355X C-ABI (include/srsran_amd/pdsch_modulator.h).

Reference interfaces:
  pdsch_modulator.h:97         modulate(resource_grid_writer& grid, span<const bit_buffer> codewords, const config_t&)
  pdsch_modulator.h:50-85      config_t {rnti, bwp, modulation1, modulation2, freq_allocation, time_alloc,
                                         dmrs_symb_pos, dmrs_config_type, nof_cdm_groups_without_data, n_id,
                                         scaling, reserved, precoding}
  dmrs_pdsch_processor.h:65    map(resource_grid_writer& grid, const config_t&)
  dmrs_pdsch_processor.h:38-57 config_t {slot, reference_point_k_rb, type, scrambling_id, n_scid, amplitude,
                                         symbols_mask, rb_mask, precoding}
Grids: uint32 [ports][14][nof_subc] (complex bf16, real in the low half) on the
host, or a torch int32 tensor of the same shape(s) on the device for the batch forms.
The frequency allocation is given resolved to CRB indices (rb_allocation::get_crb_indices);
precoding as complex weights [layer][port] (precoding_configuration, PRG 0).
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib

MAX_RB = 275
MASK_BYTES = 35
MAX_PATTERNS = 8


class RePattern(ctypes.Structure):
    """``srs_amd_re_pattern`` (re_pattern.h:35)."""

    _fields_ = [("crb_mask", ctypes.c_uint8 * MASK_BYTES), ("reserved0", ctypes.c_uint8),
                ("re_mask", ctypes.c_uint16), ("symbols", ctypes.c_uint16)]


class _ModConfig(ctypes.Structure):
    _fields_ = [("rnti", ctypes.c_uint32), ("n_id", ctypes.c_uint32), ("modulation", ctypes.c_int32),
                ("bwp_start", ctypes.c_uint32), ("bwp_size", ctypes.c_uint32),
                ("crb_mask", ctypes.c_uint8 * MASK_BYTES), ("reserved0", ctypes.c_uint8),
                ("start_symbol", ctypes.c_uint32), ("nof_symbols", ctypes.c_uint32),
                ("dmrs_symbol_mask", ctypes.c_uint32), ("dmrs_type", ctypes.c_uint32),
                ("nof_cdm_groups_without_data", ctypes.c_uint32), ("scaling", ctypes.c_float),
                ("nof_layers", ctypes.c_uint32), ("nof_ports", ctypes.c_uint32),
                ("weights", ctypes.c_float * 32), ("nof_reserved", ctypes.c_uint32),
                ("reserved", RePattern * MAX_PATTERNS)]


class _DmrsConfig(ctypes.Structure):
    _fields_ = [("slot_index", ctypes.c_uint32), ("reference_point_k_rb", ctypes.c_uint32),
                ("type", ctypes.c_uint32), ("scrambling_id", ctypes.c_uint32), ("n_scid", ctypes.c_uint32),
                ("amplitude", ctypes.c_float), ("symbols_mask", ctypes.c_uint32),
                ("crb_mask", ctypes.c_uint8 * MASK_BYTES), ("reserved0", ctypes.c_uint8),
                ("nof_layers", ctypes.c_uint32), ("nof_ports", ctypes.c_uint32), ("weights", ctypes.c_float * 32)]


def _mask_bytes(crbs):
    m = (ctypes.c_uint8 * MASK_BYTES)()
    for c in crbs:
        c = int(c)
        if not 0 <= c < MAX_RB:
            raise ValueError("CRB %d out of range" % c)
        m[c // 8] |= 1 << (c % 8)
    return m


def _weights(w, nof_layers, nof_ports):
    w = np.asarray(w, np.complex64).reshape(nof_layers, nof_ports)
    out = (ctypes.c_float * 32)()
    for v in range(nof_layers):
        for p in range(nof_ports):
            out[(v * 4 + p) * 2] = float(w[v, p].real)
            out[(v * 4 + p) * 2 + 1] = float(w[v, p].imag)
    return out


@dataclass
class ReservedPattern:
    """re_pattern: CRB indices, 12-bit RE mask, 14-bit symbol mask."""

    crbs: list
    re_mask: int
    symbols: int


@dataclass
class PdschModulatorConfig:
    """pdsch_modulator::config_t. crbs = rb_allocation::get_crb_indices(bwp)."""

    rnti: int
    bwp_start: int
    bwp_size: int
    modulation: int  # Qm code (modulation.MODULATION)
    crbs: list
    start_symbol: int
    nof_symbols: int
    dmrs_symb_pos: int
    dmrs_type: int = 1
    nof_cdm_groups_without_data: int = 2
    n_id: int = 0
    scaling: float = 1.0
    reserved: list = field(default_factory=list)
    precoding: object = None  # complex [layers][ports]; None = identity 1x1

    def _c(self):
        w = np.ones((1, 1), np.complex64) if self.precoding is None else np.asarray(self.precoding, np.complex64)
        if w.ndim != 2:
            raise ValueError("precoding weights must be [layers][ports]")
        if len(self.reserved) > MAX_PATTERNS:
            raise ValueError("too many reserved patterns")
        c = _ModConfig()
        c.rnti, c.n_id, c.modulation = self.rnti, self.n_id, self.modulation
        c.bwp_start, c.bwp_size = self.bwp_start, self.bwp_size
        c.crb_mask = _mask_bytes(self.crbs)
        c.start_symbol, c.nof_symbols = self.start_symbol, self.nof_symbols
        c.dmrs_symbol_mask, c.dmrs_type = self.dmrs_symb_pos, self.dmrs_type
        c.nof_cdm_groups_without_data = self.nof_cdm_groups_without_data
        c.scaling = self.scaling
        c.nof_layers, c.nof_ports = w.shape
        c.weights = _weights(w, *w.shape)
        c.nof_reserved = len(self.reserved)
        for i, r in enumerate(self.reserved):
            c.reserved[i].crb_mask = _mask_bytes(r.crbs)
            c.reserved[i].re_mask = r.re_mask
            c.reserved[i].symbols = r.symbols
        return c


@dataclass
class DmrsPdschConfig:
    """dmrs_pdsch_processor::config_t (slot as its slot_index)."""

    slot_index: int
    reference_point_k_rb: int
    type: int
    scrambling_id: int
    n_scid: bool
    amplitude: float
    symbols_mask: int
    crbs: list
    precoding: object = None  # complex [layers][ports]

    def _c(self):
        w = np.ones((1, 1), np.complex64) if self.precoding is None else np.asarray(self.precoding, np.complex64)
        if w.ndim != 2:
            raise ValueError("precoding weights must be [layers][ports] (one PRG)")
        c = _DmrsConfig()
        c.slot_index, c.reference_point_k_rb, c.type = self.slot_index, self.reference_point_k_rb, self.type
        c.scrambling_id, c.n_scid, c.amplitude = self.scrambling_id, int(bool(self.n_scid)), self.amplitude
        c.symbols_mask = self.symbols_mask
        c.crb_mask = _mask_bytes(self.crbs)
        c.nof_layers, c.nof_ports = w.shape
        c.weights = _weights(w, *w.shape)
        return c


class PdschSlotPdu(ctypes.Structure):
    """``srs_amd_pdsch_slot_pdu``: one PDU of srs_amd_pdsch_modulate_slot."""

    _fields_ = [("plan", ctypes.c_void_p), ("dmrs", ctypes.c_void_p), ("grid", ctypes.c_uint32),
                ("nof_bits", ctypes.c_uint32), ("cw_offset", ctypes.c_uint64), ("d_grid", ctypes.c_void_p),
                ("ptrs", ctypes.c_void_p)]


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    sigs = {
        "srs_amd_pdsch_modulator_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_pdsch_modulator_destroy": (None, [P]),
        "srs_amd_pdsch_mod_plan_create": (c.c_int, [P, c.POINTER(_ModConfig), u, c.POINTER(P), c.POINTER(u)]),
        "srs_amd_pdsch_mod_plan_destroy": (None, [P]),
        "srs_amd_pdsch_modulate": (c.c_int, [P, P, P, u, P, u]),
        "srs_amd_pdsch_modulate_batch": (c.c_int, [P, P, P, c.c_uint64, P, u, u, u, P]),
        "srs_amd_dmrs_pdsch_map": (c.c_int, [P, c.POINTER(_DmrsConfig), P, u, u]),
        "srs_amd_dmrs_pdsch_map_batch": (c.c_int, [P, c.POINTER(_DmrsConfig), P, c.c_uint64, u, u, P]),
        "srs_amd_pdsch_modulate_slot": (c.c_int, [P, c.POINTER(PdschSlotPdu), u, P, c.c_uint64, u, u, P, P]),
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


class PdschModPlan:
    """RE allocation of one configuration resolved on the device (reusable across batches)."""

    def __init__(self, modulator, config, nof_subc):
        self._lib = modulator._lib
        self._c = config._c()
        h = ctypes.c_void_p()
        n = ctypes.c_uint32()
        _lib.check(self._lib.srs_amd_pdsch_mod_plan_create(modulator._h, ctypes.byref(self._c), nof_subc,
                                                          ctypes.byref(h), ctypes.byref(n)), "pdsch_modulator plan")
        self._h = h
        self.nof_re = n.value
        self.nof_subc = nof_subc
        self.nof_layers = self._c.nof_layers
        self.nof_ports = self._c.nof_ports
        self.qm = config.modulation
        self.nof_bits = self.nof_re * self.nof_layers * (1 if self.qm < 2 else self.qm)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pdsch_mod_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PdschModulator:
    """pdsch_modulator + dmrs_pdsch_processor on one device."""

    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pdsch_modulator_create(ctypes.byref(h), int(device)), "pdsch_modulator create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pdsch_modulator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def plan(self, config, nof_subc):
        return PdschModPlan(self, config, nof_subc)

    def modulate(self, grid, codeword, config):
        """grid: uint32 [ports][14][nof_subc], updated in place; codeword: packed bytes (bit_buffer)
        holding the allocation's nof_re * layers * Qm bits."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a contiguous uint32 [ports][14][nof_subc] array")
        plan = config if isinstance(config, PdschModPlan) else self.plan(config, grid.shape[2])
        cw = np.ascontiguousarray(codeword, dtype=np.uint8)
        if cw.size * 8 < plan.nof_bits:
            raise ValueError("codeword shorter than the allocation")
        _lib.check(self._lib.srs_amd_pdsch_modulate(self._h, plan._h, grid.ctypes.data, grid.shape[0],
                                                    cw.ctypes.data, plan.nof_bits), "pdsch_modulate")
        return grid

    def modulate_batch(self, grids, codewords, plan, stream=None):
        """grids: torch int32 [n][ports][14][nof_subc]; codewords: torch uint8 [n][cw_stride] packed."""
        import torch

        n = codewords.shape[0]
        if grids.shape[0] != n or grids.shape[2] != 14 or grids.shape[3] != plan.nof_subc:
            raise ValueError("grid batch shape does not match the plan")
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pdsch_modulate_batch(
            self._h, plan._h, grids.data_ptr(), grids.stride(0), codewords.data_ptr(), codewords.stride(0),
            plan.nof_bits, n, ctypes.c_void_p(stream.cuda_stream)), "pdsch_modulate_batch")
        return grids

    def map_dmrs(self, grid, config):
        """dmrs_pdsch_processor::map on a host grid uint32 [ports][14][nof_subc] (in place)."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a contiguous uint32 [ports][14][nof_subc] array")
        c = config._c()
        _lib.check(self._lib.srs_amd_dmrs_pdsch_map(self._h, ctypes.byref(c), grid.ctypes.data, grid.shape[0],
                                                    grid.shape[2]), "dmrs_pdsch_map")
        return grid

    def map_dmrs_batch(self, grids, config, stream=None):
        import torch

        c = config._c()
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_dmrs_pdsch_map_batch(self._h, ctypes.byref(c), grids.data_ptr(), grids.stride(0),
                                                          grids.shape[3], grids.shape[0],
                                                          ctypes.c_void_p(stream.cuda_stream)), "dmrs_pdsch_map_batch")
        return grids

    def modulate_slot(self, grids, pdus, codewords=None, stream=None):
        """Every PDSCH PDU of a slot in two launches. grids: torch int32 [n][ports][14][nof_subc].
        pdus: a PdschSlot over the device codeword buffer `codewords` (uint8), or a list of (plan or None,
        DmrsPdschConfig or None, grid index, packed host codeword bytes or None), staged here."""
        import torch

        if isinstance(pdus, PdschSlot):
            slot = pdus
        else:
            offs, total = [], 0
            for plan, _, _, _ in pdus:
                offs.append(total)
                total += 0 if plan is None else (plan.nof_bits // 8 + 64) // 64 * 64
            host = np.zeros(max(total, 1), np.uint8)
            for (plan, _, _, cw), off in zip(pdus, offs):
                if plan is not None:
                    b = np.ascontiguousarray(cw, np.uint8)
                    if b.size * 8 < plan.nof_bits:
                        raise ValueError("codeword shorter than the allocation")
                    host[off:off + b.size] = b
            codewords = torch.from_numpy(host).to(grids.device)
            slot = PdschSlot([(p, d, g, o) for (p, d, g, _), o in zip(pdus, offs)])
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pdsch_modulate_slot(
            self._h, slot.arr, slot.n, grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[3],
            None if codewords is None else codewords.data_ptr(), ctypes.c_void_p(stream.cuda_stream)),
            "pdsch_modulate_slot")
        if not isinstance(pdus, PdschSlot):
            stream.synchronize()  # the staged codewords are released on return
        return grids


class PdschSlot:
    """The srs_amd_pdsch_slot_pdu array of a slot, built once per slot configuration: pdus = list of
    (plan or None, DmrsPdschConfig or None, grid index, codeword byte offset)."""

    def __init__(self, pdus):
        self.plans = [p for p, _, _, _ in pdus]  # keep the plans alive
        self.dmrs = [None if d is None else d._c() for _, d, _, _ in pdus]
        self.n = len(pdus)
        self.arr = (PdschSlotPdu * max(self.n, 1))()
        for i, (plan, _, g, off) in enumerate(pdus):
            d = self.dmrs[i]
            self.arr[i] = PdschSlotPdu(None if plan is None else plan._h.value,
                                       None if d is None else ctypes.addressof(d), int(g),
                                       0 if plan is None else plan.nof_bits, int(off))

"""Host-side mirror of srsRAN's PUCCH Format 0 / Format 1 detectors over the MI355X C-ABI (include/srsran_amd/pucch.h).

Reference interfaces: pucch_detector::detect(const resource_grid_reader&, const format0_configuration&)
(include/srsran/phy/upper/channel_processors/pucch/pucch_detector.h:44-77, impl pucch_detector_format0.cpp:124-246),
the Format 0 branch of pucch_processor::process; pucch_detector::detect(grid, format1_configuration,
pucch_format1_map<unsigned>) (pucch_detector.h:86-118, 155-160, impl pucch_detector_format1.cpp:156-663) behind
pucch_processor::process(grid, format1_batch_configuration) (pucch_processor_impl.cpp:74-138).  Grids are cbf16 [port][14][nof_subc]: numpy uint32 for the host
form, torch int32 [n][port][14][nof_subc] on the device for the slot form.
"""
import ctypes

import numpy as np

from . import _lib

UCI_STATUS_VALID = 1
UCI_STATUS_INVALID = 2


class PucchF0Pdu(ctypes.Structure):
    _fields_ = [("numerology", ctypes.c_uint32), ("slot_index", ctypes.c_uint32), ("starting_prb", ctypes.c_uint32),
                ("second_hop_prb", ctypes.c_int32), ("start_symbol_index", ctypes.c_uint32),
                ("nof_symbols", ctypes.c_uint32), ("initial_cyclic_shift", ctypes.c_uint32),
                ("n_id", ctypes.c_uint32), ("nof_harq_ack", ctypes.c_uint32), ("sr_opportunity", ctypes.c_uint32),
                ("nof_ports", ctypes.c_uint32), ("ports", ctypes.c_uint8 * 4), ("grid", ctypes.c_uint32),
                ("d_grid", ctypes.c_void_p)]


class PucchResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("nof_sr", ctypes.c_uint32), ("nof_harq_ack", ctypes.c_uint32),
                ("sr", ctypes.c_uint8), ("harq_ack", ctypes.c_uint8 * 2), ("reserved", ctypes.c_uint8),
                ("detection_metric", ctypes.c_float), ("sinr_dB", ctypes.c_float), ("rsrp_dB", ctypes.c_float),
                ("epre_dB", ctypes.c_float)]


PucchF0Result = PucchResult


class PucchF1Entry(ctypes.Structure):
    _fields_ = [("initial_cyclic_shift", ctypes.c_uint8), ("time_domain_occ", ctypes.c_uint8),
                ("nof_harq_ack", ctypes.c_uint8), ("reserved", ctypes.c_uint8)]


class PucchF1Batch(ctypes.Structure):
    _fields_ = [("numerology", ctypes.c_uint32), ("slot_index", ctypes.c_uint32), ("starting_prb", ctypes.c_uint32),
                ("second_hop_prb", ctypes.c_int32), ("start_symbol_index", ctypes.c_uint32),
                ("nof_symbols", ctypes.c_uint32), ("n_id", ctypes.c_uint32), ("nof_ports", ctypes.c_uint32),
                ("ports", ctypes.c_uint8 * 4), ("nof_entries", ctypes.c_uint32), ("entries", ctypes.c_void_p),
                ("grid", ctypes.c_uint32), ("d_grid", ctypes.c_void_p)]


class PucchF2Pdu(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("numerology", "slot_index", "bwp_start_rb", "bwp_size_rb",
                                                "starting_prb")] + [("second_hop_prb", ctypes.c_int32)] + \
               [(n, ctypes.c_uint32) for n in ("nof_prb", "start_symbol_index", "nof_symbols", "rnti", "n_id", "n_id_0",
                                                "nof_harq_ack", "nof_sr", "nof_csi_part1", "nof_csi_part2",
                                                "nof_ports")] + \
               [("ports", ctypes.c_uint8 * 4), ("grid", ctypes.c_uint32), ("d_grid", ctypes.c_void_p)]


class PucchUciResult(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("status", "nof_harq_ack", "nof_sr", "nof_csi_part1", "nof_csi_part2")] + \
               [(n, ctypes.c_float) for n in ("sinr_dB", "rsrp_dB", "epre_dB", "time_alignment_s", "cfo_Hz")]


UCI_RESULT_DTYPE = np.dtype([(n, "<u4") for n in ("status", "nof_harq_ack", "nof_sr", "nof_csi_part1",
                                                  "nof_csi_part2")] +
                            [(n, "<f4") for n in ("sinr_dB", "rsrp_dB", "epre_dB", "time_alignment_s", "cfo_Hz")])
assert UCI_RESULT_DTYPE.itemsize == ctypes.sizeof(PucchUciResult)


def make_f2_pdu(*, numerology=0, slot_index=0, bwp_start_rb=0, bwp_size_rb=52, starting_prb=0, second_hop_prb=None,
                nof_prb=1, start_symbol_index=12, nof_symbols=2, rnti=0x4601, n_id=0, n_id_0=0, nof_harq_ack=0,
                nof_sr=0, nof_csi_part1=0, nof_csi_part2=0, ports=(0,), grid=0):
    """pucch_processor::format2_configuration."""
    p = PucchF2Pdu()
    for k, v in dict(numerology=numerology, slot_index=slot_index, bwp_start_rb=bwp_start_rb, bwp_size_rb=bwp_size_rb,
                     starting_prb=starting_prb, nof_prb=nof_prb, start_symbol_index=start_symbol_index,
                     nof_symbols=nof_symbols, rnti=rnti, n_id=n_id, n_id_0=n_id_0, nof_harq_ack=nof_harq_ack,
                     nof_sr=nof_sr, nof_csi_part1=nof_csi_part1, nof_csi_part2=nof_csi_part2, grid=grid).items():
        setattr(p, k, int(v))
    p.second_hop_prb = -1 if second_hop_prb is None else int(second_hop_prb)
    if not 1 <= len(ports) <= 4:
        raise ValueError("1 to 4 ports")
    p.nof_ports = len(ports)
    for i, q in enumerate(ports):
        p.ports[i] = int(q)
    return p


class PucchF34Pdu(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("format", "numerology", "slot_index", "bwp_start_rb", "bwp_size_rb",
                                                "starting_prb")] + [("second_hop_prb", ctypes.c_int32)] + \
               [(n, ctypes.c_uint32) for n in ("nof_prb", "start_symbol_index", "nof_symbols", "rnti", "n_id_hopping",
                                                "n_id_scrambling", "nof_harq_ack", "nof_sr", "nof_csi_part1",
                                                "nof_csi_part2", "additional_dmrs", "pi2_bpsk", "occ_index",
                                                "occ_length", "nof_ports")] + \
               [("ports", ctypes.c_uint8 * 4), ("grid", ctypes.c_uint32), ("d_grid", ctypes.c_void_p)]


def make_f34_pdu(*, format=3, numerology=0, slot_index=0, bwp_start_rb=0, bwp_size_rb=52, starting_prb=0,
                 second_hop_prb=None, nof_prb=1, start_symbol_index=0, nof_symbols=14, rnti=0x4601, n_id_hopping=0,
                 n_id_scrambling=0, nof_harq_ack=0, nof_sr=0, nof_csi_part1=0, nof_csi_part2=0, additional_dmrs=False,
                 pi2_bpsk=False, occ_index=0, occ_length=2, ports=(0,), grid=0):
    """pucch_processor::format3_configuration (format=3) / format4_configuration (format=4)."""
    p = PucchF34Pdu()
    for k, v in dict(format=format, numerology=numerology, slot_index=slot_index, bwp_start_rb=bwp_start_rb,
                     bwp_size_rb=bwp_size_rb, starting_prb=starting_prb, nof_prb=1 if format == 4 else nof_prb,
                     start_symbol_index=start_symbol_index, nof_symbols=nof_symbols, rnti=rnti,
                     n_id_hopping=n_id_hopping, n_id_scrambling=n_id_scrambling, nof_harq_ack=nof_harq_ack,
                     nof_sr=nof_sr, nof_csi_part1=nof_csi_part1, nof_csi_part2=nof_csi_part2,
                     additional_dmrs=bool(additional_dmrs), pi2_bpsk=bool(pi2_bpsk), occ_index=occ_index,
                     occ_length=occ_length, grid=grid).items():
        setattr(p, k, int(v))
    p.second_hop_prb = -1 if second_hop_prb is None else int(second_hop_prb)
    if not 1 <= len(ports) <= 4:
        raise ValueError("1 to 4 ports")
    p.nof_ports = len(ports)
    for i, q in enumerate(ports):
        p.ports[i] = int(q)
    return p


def f34_dmrs_mask(nof_symbols, hop, additional):
    """get_pucch_formats3_4_dmrs_symbol_mask (pucch_formats3_4_helpers.h): allocated symbols carrying DM-RS."""
    t = {4: [0, 2] if hop else [1], 5: [0, 3], 6: [1, 4], 7: [1, 4], 8: [1, 5], 9: [1, 6],
         10: [1, 3, 6, 8] if additional else [2, 7], 11: [1, 3, 6, 9] if additional else [2, 7],
         12: [1, 4, 7, 10] if additional else [2, 8], 13: [1, 4, 7, 11] if additional else [2, 9],
         14: [1, 5, 8, 12] if additional else [3, 10]}
    return t[nof_symbols]


def f34_nof_llrs(pdu):
    nd = len(f34_dmrs_mask(pdu.nof_symbols, pdu.second_hop_prb >= 0, pdu.additional_dmrs))
    M = 12 * (1 if pdu.format == 4 else pdu.nof_prb)
    return (pdu.nof_symbols - nd) * M * (1 if pdu.pi2_bpsk else 2) // (pdu.occ_length if pdu.format == 4 else 1)


def payload_bits(pdu):
    return pdu.nof_harq_ack + pdu.nof_sr + pdu.nof_csi_part1 + pdu.nof_csi_part2


RESULT_DTYPE = np.dtype([("status", "<u4"), ("nof_sr", "<u4"), ("nof_harq_ack", "<u4"), ("sr", "u1"),
                         ("harq_ack", "u1", (2,)), ("reserved", "u1"), ("detection_metric", "<f4"),
                         ("sinr_dB", "<f4"), ("rsrp_dB", "<f4"), ("epre_dB", "<f4")])
assert RESULT_DTYPE.itemsize == ctypes.sizeof(PucchResult)


def make_f0_pdu(*, numerology=0, slot_index=0, starting_prb=0, second_hop_prb=None, start_symbol_index=12,
                nof_symbols=2, initial_cyclic_shift=0, n_id=0, nof_harq_ack=1, sr_opportunity=False, ports=(0,),
                grid=0):
    """pucch_detector::format0_configuration."""
    p = PucchF0Pdu()
    p.numerology, p.slot_index, p.starting_prb = int(numerology), int(slot_index), int(starting_prb)
    p.second_hop_prb = -1 if second_hop_prb is None else int(second_hop_prb)
    p.start_symbol_index, p.nof_symbols = int(start_symbol_index), int(nof_symbols)
    p.initial_cyclic_shift, p.n_id = int(initial_cyclic_shift), int(n_id)
    p.nof_harq_ack, p.sr_opportunity = int(nof_harq_ack), int(bool(sr_opportunity))
    if not 1 <= len(ports) <= 4:
        raise ValueError("1 to 4 ports")
    p.nof_ports = len(ports)
    for i, q in enumerate(ports):
        p.ports[i] = int(q)
    p.grid = int(grid)
    return p


def make_f1_batch(entries, *, numerology=0, slot_index=0, starting_prb=0, second_hop_prb=None,
                  start_symbol_index=0, nof_symbols=14, n_id=0, ports=(0,), grid=0):
    """pucch_processor::format1_batch_configuration: the common allocation and entries = [(initial cyclic shift,
    time-domain OCC, nof_harq_ack)].  The entry array is kept alive by the returned batch (attribute _entries)."""
    b = PucchF1Batch()
    b.numerology, b.slot_index, b.starting_prb = int(numerology), int(slot_index), int(starting_prb)
    b.second_hop_prb = -1 if second_hop_prb is None else int(second_hop_prb)
    b.start_symbol_index, b.nof_symbols, b.n_id = int(start_symbol_index), int(nof_symbols), int(n_id)
    if not 1 <= len(ports) <= 4:
        raise ValueError("1 to 4 ports")
    b.nof_ports = len(ports)
    for i, q in enumerate(ports):
        b.ports[i] = int(q)
    arr = (PucchF1Entry * max(len(entries), 1))()
    for i, (ics, occ, nh) in enumerate(entries):
        arr[i].initial_cyclic_shift, arr[i].time_domain_occ, arr[i].nof_harq_ack = int(ics), int(occ), int(nh)
    b.nof_entries = len(entries)
    b.entries = ctypes.addressof(arr)
    b._entries = arr
    b.grid = int(grid)
    return b


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_pucch_processor_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_pucch_processor_destroy": (None, [P]),
        "srs_amd_pucch_f0_detect_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32,
                                                   c.c_uint32, P, P]),
        "srs_amd_pucch_f0_detect": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_pucch_f1_detect_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32,
                                                   c.c_uint32, P, P]),
        "srs_amd_pucch_f1_detect": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_pucch_f2_process_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32,
                                                    c.c_uint32, P, P, c.c_uint64, P]),
        "srs_amd_pucch_f2_process": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P, P]),
        "srs_amd_pucch_f2_demodulate": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_pucch_f34_process_slot": (c.c_int, [P, P, c.c_uint32, P, c.c_uint64, c.c_uint32, c.c_uint32,
                                                     c.c_uint32, P, P, c.c_uint64, P]),
        "srs_amd_pucch_f34_process": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P, P]),
        "srs_amd_pucch_f34_demodulate": (c.c_int, [P, P, P, c.c_uint32, c.c_uint32, P]),
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


class PucchProcessor:
    """PUCCH Format 0 detection on the MI355X (one per device; thread-safe)."""

    def __init__(self, device=0):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pucch_processor_create(ctypes.byref(h), int(device)), "pucch_processor create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pucch_processor_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def detect_f0(self, grid, pdu):
        """pucch_detector::detect of one Format 0 PDU on a host grid (numpy uint32 [ports][14][nof_subc])."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        r = PucchResult()
        _lib.check(self._lib.srs_amd_pucch_f0_detect(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                     grid.shape[2], ctypes.byref(r)), "pucch f0 detect")
        return r

    def detect_f0_slot(self, grids, pdus, stream=None):
        """Every Format 0 PDU of a slot on device grids (torch int32 [n][ports][14][nof_subc]); returns a torch
        uint8 tensor of nof_pdus RESULT_DTYPE records (asynchronous on stream)."""
        import torch

        arr = (PucchF0Pdu * len(pdus))(*pdus)
        out = torch.zeros((len(pdus), RESULT_DTYPE.itemsize), dtype=torch.uint8, device=grids.device)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pucch_f0_detect_slot(
            self._h, arr, len(pdus), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[1],
            grids.shape[-1], out.data_ptr(), ctypes.c_void_p(stream.cuda_stream)), "pucch f0 detect_slot")
        return out

    def detect_f1(self, grid, batch):
        """pucch_processor::process of one Format 1 batch on a host grid (numpy uint32 [ports][14][nof_subc]);
        returns one PucchResult per entry, in entry order."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        out = (PucchResult * max(batch.nof_entries, 1))()
        _lib.check(self._lib.srs_amd_pucch_f1_detect(self._h, ctypes.byref(batch), grid.ctypes.data, grid.shape[0],
                                                     grid.shape[2], out), "pucch f1 detect")
        return list(out)[:batch.nof_entries]

    def detect_f1_slot(self, grids, batches, stream=None):
        """Every Format 1 batch of a slot on device grids (torch int32 [n][ports][14][nof_subc]); returns a torch
        uint8 tensor of RESULT_DTYPE records, the entries of all batches in order (asynchronous on stream)."""
        import torch

        arr = (PucchF1Batch * len(batches))(*batches)
        total = sum(b.nof_entries for b in batches)
        out = torch.zeros((max(total, 1), RESULT_DTYPE.itemsize), dtype=torch.uint8, device=grids.device)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pucch_f1_detect_slot(
            self._h, arr, len(batches), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[1],
            grids.shape[-1], out.data_ptr(), ctypes.c_void_p(stream.cuda_stream)), "pucch f1 detect_slot")
        return out[:total]

    def process_f2(self, grid, pdu):
        """pucch_processor::process of one Format 2 PDU on a host grid -> (PucchUciResult, payload bits uint8)."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        r = PucchUciResult()
        payload = np.zeros(max(payload_bits(pdu), 1), np.uint8)
        _lib.check(self._lib.srs_amd_pucch_f2_process(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                      grid.shape[2], ctypes.byref(r), payload.ctypes.data),
                   "pucch f2 process")
        return r, payload[:payload_bits(pdu)]

    def demodulate_f2(self, grid, pdu):
        """Estimator + pucch_demodulator of one Format 2 PDU on a host grid -> int8 LLRs [16 nof_prb nof_symbols]."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        llr = np.zeros(16 * pdu.nof_prb * pdu.nof_symbols, np.int8)
        _lib.check(self._lib.srs_amd_pucch_f2_demodulate(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                         grid.shape[2], llr.ctypes.data), "pucch f2 demodulate")
        return llr

    def process_f34(self, grid, pdu):
        """pucch_processor::process of one Format 3 / 4 PDU on a host grid -> (PucchUciResult, payload bits)."""
        if grid.dtype != np.uint32 or grid.ndim != 3 or grid.shape[1] != 14 or not grid.flags.c_contiguous:
            raise ValueError("grid must be a C-contiguous uint32 array [ports][14][nof_subc]")
        r = PucchUciResult()
        payload = np.zeros(max(payload_bits(pdu), 1), np.uint8)
        _lib.check(self._lib.srs_amd_pucch_f34_process(self._h, ctypes.byref(pdu), grid.ctypes.data, grid.shape[0],
                                                       grid.shape[2], ctypes.byref(r), payload.ctypes.data),
                   "pucch f34 process")
        return r, payload[:payload_bits(pdu)]

    def demodulate_f34(self, grid, pdu):
        """Estimator + pucch_demodulator of one Format 3 / 4 PDU on a host grid -> int8 LLRs."""
        llr = np.zeros(f34_nof_llrs(pdu), np.int8)
        _lib.check(self._lib.srs_amd_pucch_f34_demodulate(self._h, ctypes.byref(pdu), grid.ctypes.data,
                                                          grid.shape[0], grid.shape[2], llr.ctypes.data),
                   "pucch f34 demodulate")
        return llr

    def process_f34_slot(self, grids, pdus, payload_stride=1706, stream=None):
        """Every Format 3 / 4 PDU of a slot on device grids -> (torch uint8 result records, payload rows)."""
        import torch

        arr = (PucchF34Pdu * len(pdus))(*pdus)
        res = torch.zeros((max(len(pdus), 1), UCI_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=grids.device)
        pay = torch.zeros((max(len(pdus), 1), payload_stride), dtype=torch.uint8, device=grids.device)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pucch_f34_process_slot(
            self._h, arr, len(pdus), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[1],
            grids.shape[-1], res.data_ptr(), pay.data_ptr(), payload_stride, ctypes.c_void_p(stream.cuda_stream)),
            "pucch f34 process_slot")
        return res[:len(pdus)], pay[:len(pdus)]

    def process_f2_slot(self, grids, pdus, payload_stride=1706, stream=None):
        """Every Format 2 PDU of a slot on device grids (torch int32 [n][ports][14][nof_subc]) -> (torch uint8
        [n][UCI_RESULT_DTYPE record], torch uint8 [n][payload_stride] payload rows), asynchronous on stream."""
        import torch

        arr = (PucchF2Pdu * len(pdus))(*pdus)
        res = torch.zeros((max(len(pdus), 1), UCI_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=grids.device)
        pay = torch.zeros((max(len(pdus), 1), payload_stride), dtype=torch.uint8, device=grids.device)
        if stream is None:
            stream = torch.cuda.current_stream(grids.device)
        _lib.check(self._lib.srs_amd_pucch_f2_process_slot(
            self._h, arr, len(pdus), grids.data_ptr(), grids.stride(0), grids.shape[0], grids.shape[1],
            grids.shape[-1], res.data_ptr(), pay.data_ptr(), payload_stride, ctypes.c_void_p(stream.cuda_stream)),
            "pucch f2 process_slot")
        return res[:len(pdus)], pay[:len(pdus)]


def parse_uci_results(raw):
    """uint8 [n][record] (numpy) -> UCI_RESULT_DTYPE records."""
    return np.ascontiguousarray(raw).view(UCI_RESULT_DTYPE).reshape(-1)


def parse_results(raw):
    """uint8 [n][record] (numpy) -> RESULT_DTYPE records."""
    return np.ascontiguousarray(raw).view(RESULT_DTYPE).reshape(-1)

"""Host-side mirror of srsRAN's shared-channel transport-block processors over the
MI355X C-ABI (include/srsran_amd/sch.h).

Reference interfaces:
  pdsch_encoder.h:61   encode(span<uint8_t> codeword, span<const uint8_t> transport_block, const configuration&)
  pusch_decoder.h:77   new_data(transport_block, rx_buffer, notifier, configuration) + pusch_decoder_buffer
                       on_new_softbits / on_end_softbits -> pusch_decoder_result
  ldpc_segmenter_tx_impl.cpp:53 new_transmission (segmentation geometry, SchPlan)
"""
import ctypes

import numpy as np

from . import _lib

_FIELDS = ["tbs", "base_graph", "rv", "modulation_order", "Nref", "nof_layers", "nof_ch_symbols", "lifting_size",
           "segment_length", "nof_segments", "nof_tb_crc_bits", "nof_crc_bits", "cb_info_bits", "zero_pad",
           "nof_filler_bits", "nof_short_segments", "rm_length_short", "rm_length_long", "cw_length"]


class SchPlan(ctypes.Structure):
    """``srs_amd_sch_plan`` (segment_parameters of ldpc_segmenter_helpers.h:33)."""

    _fields_ = [(f, ctypes.c_uint32) for f in _FIELDS]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f in _FIELDS}


class PuschDecoderConfig(ctypes.Structure):
    """``srs_amd_pusch_decoder_config`` (pusch_decoder::configuration, pusch_decoder.h:49)."""

    _fields_ = [("nof_ldpc_iterations", ctypes.c_uint32), ("force_decoding", ctypes.c_int32),
                ("use_early_stop", ctypes.c_int32), ("new_data", ctypes.c_int32)]


class PuschDecoderResult(ctypes.Structure):
    """``srs_amd_pusch_decoder_result`` (pusch_decoder_result.h:31)."""

    _fields_ = [("tb_crc_ok", ctypes.c_int32), ("nof_codeblocks_total", ctypes.c_uint32),
                ("ldpc_iterations_sum", ctypes.c_uint32), ("ldpc_iterations_min", ctypes.c_uint32),
                ("ldpc_iterations_max", ctypes.c_uint32), ("nof_codeblocks_crc_ok", ctypes.c_uint32)]


RESULT_WORDS = ctypes.sizeof(PuschDecoderResult) // 4


class PdschUe(ctypes.Structure):
    """``srs_amd_pdsch_ue``: one UE's transport block of a heterogeneous slot batch (one PDSCH PDU codeword,
    pdsch_encoder.h:61)."""

    _fields_ = [("plan", SchPlan), ("tb_offset", ctypes.c_uint64), ("cw_offset", ctypes.c_uint64)]


class SlotUes:
    """The C descriptor array of a slot's UEs (PdschUe / PuschUe), built once and reusable across calls:
    ues is a list of (plan, first offset, second offset) as the slot entry points take them."""

    def __init__(self, kind, ues):
        self.n = len(ues)
        self.arr = (kind * max(self.n, 1))()
        self.data_end = self.out_end = 0
        for i, (plan, o1, o2) in enumerate(ues):
            self.arr[i] = kind(plan, int(o1), int(o2))
            if kind is PdschUe:  # (plan, tb_offset, cw_offset)
                self.data_end = max(self.data_end, int(o1) + plan.tbs // 8)
                self.out_end = max(self.out_end, int(o2) + (plan.cw_length + 7) // 8)
            else:  # (plan, llr_offset, tb_offset)
                self.data_end = max(self.data_end, int(o1) + plan.cw_length)
                self.out_end = max(self.out_end, int(o2) + plan.tbs // 8)


class PuschUe(ctypes.Structure):
    """``srs_amd_pusch_ue``: one UE's transport block of a heterogeneous slot batch (its PUSCH PDU,
    pusch_processor_impl.cpp:343)."""

    _fields_ = [("plan", SchPlan), ("llr_offset", ctypes.c_uint64), ("tb_offset", ctypes.c_uint64)]


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u = c.c_uint32
    PP = c.POINTER(SchPlan)
    sigs = {
        "srs_amd_sch_plan_compute": (c.c_int, [PP] + [u] * 7),
        "srs_amd_sch_plan_segments": (c.c_int, [PP, P, P]),
        "srs_amd_tbs_calculate": (u, [u, u, u, u, c.c_float, u, u, u]),
        "srs_amd_pdsch_encoder_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_pdsch_encoder_destroy": (None, [P]),
        "srs_amd_pdsch_encode": (c.c_int, [P, P, P, PP]),
        "srs_amd_pdsch_encode_batch": (c.c_int, [P, PP, P, u, P, u, u, P]),
        "srs_amd_pdsch_encode_slot": (c.c_int, [P, c.POINTER(PdschUe), u, P, P, P]),
        "srs_amd_pusch_decoder_create": (c.c_int, [c.POINTER(P), c.c_int, c.c_int]),
        "srs_amd_pusch_decoder_destroy": (None, [P]),
        "srs_amd_pusch_soft_buffer_size": (c.c_uint64, [PP]),
        "srs_amd_pusch_decoder_llr_prefix": (c.c_uint32, [PP, c.c_int, c.c_int]),
        "srs_amd_pusch_decode": (c.c_int, [P, P, c.POINTER(PuschDecoderResult), P, P, PP,
                                           c.POINTER(PuschDecoderConfig)]),
        "srs_amd_pusch_decode_batch": (c.c_int, [P, PP, c.POINTER(PuschDecoderConfig), P, u, P, P, u, P, P, u, P]),
        "srs_amd_pusch_decode_slot": (c.c_int, [P, c.POINTER(PuschDecoderConfig), c.POINTER(PuschUe), u, P, P, P,
                                                P]),
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


def _stream(stream, t):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return ctypes.c_void_p(stream.cuda_stream)


def sch_plan(tbs, base_graph, rv, modulation_order, Nref, nof_layers, nof_ch_symbols):
    """Segmentation geometry of one transport block (host only)."""
    p = SchPlan()
    _lib.check(_L().srs_amd_sch_plan_compute(ctypes.byref(p), int(tbs), int(base_graph), int(rv),
                                             int(modulation_order), int(Nref), int(nof_layers), int(nof_ch_symbols)),
               "sch plan")
    return p


def tbs_calculator_calculate(nof_symb_sh, nof_dmrs_prb, nof_oh_prb, modulation_order, target_code_rate, nof_layers,
                             tb_scaling_field, n_prb):
    """TS 38.214 5.1.3.2 TBS (tbs_calculator.h); target_code_rate is R x 1024."""
    v = _L().srs_amd_tbs_calculate(int(nof_symb_sh), int(nof_dmrs_prb), int(nof_oh_prb), int(modulation_order),
                                   float(target_code_rate), int(nof_layers), int(tb_scaling_field), int(n_prb))
    if v == 0:
        raise ValueError(_lib.lib().srs_amd_last_error().decode())
    return int(v)


def sch_segments(plan):
    """(rm_lengths, cw_offsets) per segment."""
    C = plan.nof_segments
    E = np.zeros(C, np.uint32)
    off = np.zeros(C, np.uint32)
    _lib.check(_L().srs_amd_sch_plan_segments(ctypes.byref(plan), E.ctypes.data, off.ctypes.data), "sch segments")
    return E, off


def soft_buffer_size(plan):
    return int(_L().srs_amd_pusch_soft_buffer_size(ctypes.byref(plan)))


def decoder_llr_prefix(plan, new_data=True, fresh=True):
    """LLRs of each soft-buffer row the PUSCH decoder hands to the LDPC decoder (srs_amd_pusch_decoder_llr_prefix)."""
    return int(_L().srs_amd_pusch_decoder_llr_prefix(ctypes.byref(plan), int(new_data), int(fresh)))


class PdschEncoder:
    """pdsch_encoder on the MI355X."""

    def __init__(self, device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_pdsch_encoder_create(ctypes.byref(h), int(device)), "pdsch encoder create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pdsch_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, transport_block, plan):
        """Host form: TB bytes -> codeword, one bit per byte (as the reference)."""
        tb = np.ascontiguousarray(transport_block, dtype=np.uint8)
        if tb.size * 8 != plan.tbs:
            raise ValueError("transport block of %d bytes, plan has TBS %d" % (tb.size, plan.tbs))
        cw = np.zeros(plan.cw_length, np.uint8)
        _lib.check(self._lib.srs_amd_pdsch_encode(self._h, cw.ctypes.data, tb.ctypes.data, ctypes.byref(plan)),
                   "pdsch encode")
        return cw

    def encode_batch(self, tbs, plan, out=None, stream=None):
        """Device form: uint8 [n, tb_stride] TB rows -> packed codeword rows [n, cw_stride]."""
        import torch

        if tbs.dim() != 2 or tbs.dtype != torch.uint8 or not tbs.is_contiguous():
            raise ValueError("tbs must be a contiguous uint8 [n, stride] tensor")
        n = tbs.shape[0]
        if out is None:
            out = torch.empty((n, (plan.cw_length + 7) // 8), dtype=torch.uint8, device=tbs.device)
        _lib.check(self._lib.srs_amd_pdsch_encode_batch(self._h, ctypes.byref(plan), out.data_ptr(), out.shape[1],
                                                        tbs.data_ptr(), tbs.shape[1], n, _stream(stream, tbs)),
                   "pdsch encode_batch")
        return out


def _encode_slot(self, tbs, ues, out=None, stream=None):
    """Device form over UEs with different plans (one slot's PDSCH codewords): tbs: uint8 1-D tensor
    holding every UE's transport block; ues: list of (plan, tb_offset, cw_offset).  Returns the uint8
    1-D codeword tensor (packed MSB-first, each UE's codeword at its cw_offset)."""
    import torch

    if tbs.dim() != 1 or tbs.dtype != torch.uint8 or not tbs.is_contiguous():
        raise ValueError("tbs must be a contiguous uint8 1-D tensor")
    arr = ues if isinstance(ues, SlotUes) else SlotUes(PdschUe, ues)
    n = arr.n
    if arr.data_end > tbs.numel():
        raise ValueError("a transport block lies beyond the TB tensor")
    cw_end = arr.out_end
    if out is None:
        out = torch.zeros(cw_end, dtype=torch.uint8, device=tbs.device)
    elif out.numel() < cw_end:
        raise ValueError("codeword tensor too small")
    _lib.check(self._lib.srs_amd_pdsch_encode_slot(self._h, arr.arr, n, tbs.data_ptr(), out.data_ptr(),
                                                   _stream(stream, tbs)), "pdsch encode_slot")
    return out


PdschEncoder.encode_slot = _encode_slot


class PuschDecoder:
    """pusch_decoder on the MI355X; arith 'simd' / 'generic' selects the LDPC rounding."""

    def __init__(self, arith="simd", device=-1):
        self._lib = _L()
        h = ctypes.c_void_p()
        a = {"simd": 0, "avx2": 0, "avx512": 0, "auto": 0, "generic": 1}[arith]
        _lib.check(self._lib.srs_amd_pusch_decoder_create(ctypes.byref(h), a, int(device)), "pusch decoder create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_pusch_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def config(nof_ldpc_iterations=6, force_decoding=False, use_early_stop=True, new_data=True):
        return PuschDecoderConfig(int(nof_ldpc_iterations), int(force_decoding), int(use_early_stop), int(new_data))

    def decode(self, llrs, plan, soft_buffer, transport_block, cfg):
        """Host form. soft_buffer: int8 array of soft_buffer_size(plan) bytes kept per HARQ process;
        transport_block: uint8 array of tbs/8 bytes, updated in place where the reference writes it."""
        x = np.ascontiguousarray(llrs, dtype=np.int8)
        if x.size != plan.cw_length:
            raise ValueError("%d LLRs, plan codeword has %d" % (x.size, plan.cw_length))
        if soft_buffer.dtype != np.int8 or soft_buffer.size < soft_buffer_size(plan):
            raise ValueError("soft buffer too small")
        res = PuschDecoderResult()
        _lib.check(self._lib.srs_amd_pusch_decode(self._h, transport_block.ctypes.data, ctypes.byref(res),
                                                  x.ctypes.data, soft_buffer.ctypes.data, ctypes.byref(plan),
                                                  ctypes.byref(cfg)), "pusch decode")
        return res

    def decode_batch(self, llrs, plan, cfg, tbs=None, soft=None, cb_iterations=None, stream=None):
        """Device form: int8 [n, llr_stride] codeword rows -> (TB rows uint8 [n, tbs/8], results int32 [n, 6])."""
        import torch

        if llrs.dim() != 2 or llrs.dtype != torch.int8 or not llrs.is_contiguous():
            raise ValueError("llrs must be a contiguous int8 [n, stride] tensor")
        n = llrs.shape[0]
        dev = llrs.device
        if tbs is None:
            tbs = torch.zeros((n, plan.tbs // 8), dtype=torch.uint8, device=dev)
        res = torch.empty((n, RESULT_WORDS), dtype=torch.int32, device=dev)  # every field written by the decoder
        _lib.check(self._lib.srs_amd_pusch_decode_batch(
            self._h, ctypes.byref(plan), ctypes.byref(cfg), tbs.data_ptr(), tbs.shape[1], res.data_ptr(),
            llrs.data_ptr(), llrs.shape[1], None if soft is None else soft.data_ptr(),
            None if cb_iterations is None else cb_iterations.data_ptr(), n, _stream(stream, llrs)),
            "pusch decode_batch")
        return tbs, res

    def decode_slot(self, llrs, ues, cfg, tbs=None, stream=None):
        """Device form over UEs with different plans (one slot's PUSCH PDUs, new transmissions):
        llrs: int8 1-D tensor holding every UE's codeword; ues: list of (plan, llr_offset, tb_offset).
        Returns (uint8 1-D TB tensor, results int32 [len(ues), 6])."""
        import torch

        if llrs.dim() != 1 or llrs.dtype != torch.int8 or not llrs.is_contiguous():
            raise ValueError("llrs must be a contiguous int8 1-D tensor")
        arr = ues if isinstance(ues, SlotUes) else SlotUes(PuschUe, ues)
        n = arr.n
        if arr.data_end > llrs.numel():
            raise ValueError("a codeword lies beyond the LLR tensor")
        tb_end = arr.out_end
        dev = llrs.device
        if tbs is None:
            tbs = torch.zeros(tb_end, dtype=torch.uint8, device=dev)
        elif tbs.numel() < tb_end:
            raise ValueError("TB tensor too small")
        res = torch.empty((n, RESULT_WORDS), dtype=torch.int32, device=dev)
        _lib.check(self._lib.srs_amd_pusch_decode_slot(self._h, ctypes.byref(cfg), arr.arr, n, llrs.data_ptr(),
                                                       tbs.data_ptr(), res.data_ptr(), _stream(stream, llrs)),
                   "pusch decode_slot")
        return tbs, res

"""Host-side mirror of srsRAN's LDPC encoder, rate matcher and rate dematcher
over the MI355X C-ABI (include/srsran_amd/ldpc_encoder.h, ldpc_rate_matching.h).

Reference interfaces (include/srsran/phy/upper/channel_coding/ldpc/):
  ldpc_encoder.h:59         const ldpc_encoder_buffer& encode(const bit_buffer& input, const configuration& cfg)
  ldpc_encoder_buffer.h:49  void write_codeblock(span<uint8_t> data, unsigned offset)
  ldpc_rate_matcher.h:47    void rate_match(bit_buffer& output, const ldpc_encoder_buffer& input,
                                            const codeblock_metadata& cfg)
  ldpc_rate_dematcher.h:54  void rate_dematch(span<log_likelihood_ratio> output,
                                              span<const log_likelihood_ratio> input, bool new_data,
                                              const codeblock_metadata& cfg)
  include/srsran/phy/upper/codeblock_metadata.h:44  tb_common / cb_specific fields used here.

Single-codeblock methods take host numpy arrays (the reference's shapes);
``*_batch`` methods take torch device tensors and launch on the current torch
stream.  Invalid arguments raise ``ValueError`` where the reference asserts.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from .ldpc import LdpcBaseGraph, codeblock_length, message_length

# get_bits_per_symbol(modulation_scheme) (include/srsran/ran/sch/modulation_scheme.h)
MODULATION_ORDER = {"pi/2-BPSK": 1, "BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


@dataclass
class LdpcEncoderConfiguration:
    """ldpc_encoder::configuration (ldpc_encoder.h:43)."""

    base_graph: LdpcBaseGraph = LdpcBaseGraph.BG1
    lifting_size: int = 2
    Nref: int = 0

    def to_c(self):
        return _lib.LDPCEncoderConfig(int(self.base_graph), int(self.lifting_size), int(self.Nref))


@dataclass
class CodeblockMetadata:
    """The codeblock_metadata fields the rate (de)matcher reads (codeblock_metadata.h:44-80)."""

    base_graph: LdpcBaseGraph = LdpcBaseGraph.BG1
    lifting_size: int = 2
    rv: int = 0
    modulation_order: int = 2
    Nref: int = 0
    nof_filler_bits: int = 0

    def to_c(self):
        return _lib.CodeblockMetadata(int(self.base_graph), int(self.lifting_size), int(self.rv),
                                      int(self.modulation_order), int(self.Nref), int(self.nof_filler_bits))


class _Handle:
    _create = _destroy = None

    def __init__(self, device=-1):
        self._lib = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(getattr(self._lib, self._create)(ctypes.byref(h), int(device)), self._create)
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            getattr(self._lib, self._destroy)(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _stream_arg(stream, t):
    import torch

    if stream is None:
        stream = torch.cuda.current_stream(t.device)
    return ctypes.c_void_p(stream.cuda_stream)


def _dev_u32(x, device):
    import torch

    if isinstance(x, torch.Tensor):
        if x.dtype != torch.int32 or not x.is_cuda:
            raise ValueError("index arrays must be int32 device tensors")
        return x
    return torch.as_tensor(np.asarray(x, dtype=np.int64).astype(np.int32), device=device)


class LdpcEncoder(_Handle):
    """ldpc_encoder + ldpc_encoder_buffer on the MI355X."""

    _create, _destroy = "srs_amd_ldpc_encoder_create", "srs_amd_ldpc_encoder_destroy"

    def encode(self, message: np.ndarray, cfg: LdpcEncoderConfiguration, packed=False) -> np.ndarray:
        """Encodes one message (K*Z bits: one bit per byte, or ``packed`` MSB-first)
        and returns the whole codeblock (write_codeblock(data, 0)): N_short*Z
        bytes, one bit per byte."""
        K = message_length(cfg.base_graph, cfg.lifting_size)
        N = codeblock_length(cfg.base_graph, cfg.lifting_size)
        if K == 0:
            raise ValueError("Invalid base graph / lifting size (%s, %s)" % (cfg.base_graph, cfg.lifting_size))
        msg = np.ascontiguousarray(message, dtype=np.uint8)
        if packed:
            nbits = K if msg.size == (K + 7) // 8 else msg.size * 8
        else:
            nbits = msg.size
            msg = np.packbits(msg & 1)
        out = np.zeros(N, np.uint8)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_encode(self._h, out.ctypes.data, N, msg.ctypes.data, nbits,
                                                 ctypes.byref(c)), "ldpc encode")
        return out

    def encode_batch(self, messages, cfg: LdpcEncoderConfiguration, out=None, stream=None):
        """messages: uint8 device tensor [nof_cbs, >= ceil(K*Z/8)] (packed).
        Returns packed codeblocks uint8 [nof_cbs, ceil(N_short*Z/8)]."""
        import torch

        if messages.dtype != torch.uint8 or not messages.is_cuda or messages.dim() != 2 or messages.stride(1) != 1:
            raise ValueError("messages must be a 2-D uint8 device tensor with contiguous rows")
        N = codeblock_length(cfg.base_graph, cfg.lifting_size)
        if N == 0:
            raise ValueError("Invalid base graph / lifting size (%s, %s)" % (cfg.base_graph, cfg.lifting_size))
        n = messages.shape[0]
        if out is None:
            out = torch.empty((n, (N + 7) // 8), dtype=torch.uint8, device=messages.device)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_encode_batch(self._h, ctypes.byref(c), messages.data_ptr(),
                                                       messages.stride(0), out.data_ptr(), out.stride(0), n,
                                                       _stream_arg(stream, messages)), "ldpc encode_batch")
        return out


class LdpcRateMatcher(_Handle):
    """ldpc_rate_matcher on the MI355X."""

    _create, _destroy = "srs_amd_ldpc_rate_matcher_create", "srs_amd_ldpc_rate_matcher_destroy"

    def rate_match(self, output_len: int, codeblock: np.ndarray, cfg: CodeblockMetadata) -> np.ndarray:
        """Rate-matches one codeblock (N_short*Z bits, one per byte) into
        ``output_len`` bits; returns them packed MSB-first (bit_buffer layout)."""
        cb = np.ascontiguousarray(codeblock, dtype=np.uint8)
        out = np.zeros((int(output_len) + 7) // 8, np.uint8)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_rate_match(self._h, out.ctypes.data, int(output_len), cb.ctypes.data,
                                                     cb.size, ctypes.byref(c)), "ldpc rate_match")
        return out

    def rate_match_batch(self, codeblocks, rm_lengths, cfg: CodeblockMetadata, out_offsets=None, out=None,
                         stream=None):
        """codeblocks: packed uint8 device tensor [nof_cbs, >= ceil(N/8)] (encode_batch
        output); rm_lengths: E_r per codeblock.  Segments are concatenated
        (offsets = exclusive prefix sum of E_r unless given).  Returns the packed
        codeword (uint8 device tensor)."""
        import torch

        dev = codeblocks.device
        E = np.asarray(rm_lengths.cpu() if isinstance(rm_lengths, torch.Tensor) else rm_lengths, dtype=np.int64)
        n = codeblocks.shape[0]
        if E.size != n:
            raise ValueError("one rate-matched length per codeblock")
        if out_offsets is None:
            out_offsets = np.concatenate([[0], np.cumsum(E)[:-1]]) if n else np.zeros(0, np.int64)
        total = int(np.max(np.asarray(out_offsets.cpu() if isinstance(out_offsets, torch.Tensor) else out_offsets,
                                      dtype=np.int64) + E)) if n else 0
        if out is None:
            out = torch.zeros(((total + 7) // 8,), dtype=torch.uint8, device=dev)
        d_E = _dev_u32(E, dev)
        d_off = _dev_u32(out_offsets, dev)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_rate_match_batch(
            self._h, ctypes.byref(c), codeblocks.data_ptr(), codeblocks.stride(0), d_E.data_ptr(), d_off.data_ptr(),
            int(E.max()) if n else 0, out.data_ptr(), n, _stream_arg(stream, codeblocks)), "ldpc rate_match_batch")
        return out


class LdpcRateDematcher(_Handle):
    """ldpc_rate_dematcher on the MI355X."""

    _create, _destroy = "srs_amd_ldpc_rate_dematcher_create", "srs_amd_ldpc_rate_dematcher_destroy"

    def rate_dematch(self, output: np.ndarray, input: np.ndarray, new_data: bool, cfg: CodeblockMetadata):
        """Recovers a full codeblock from its rate-matched LLRs into ``output``
        (int8, N_short*Z, read and written in place: the HARQ soft buffer)."""
        if output.dtype != np.int8 or not output.flags["C_CONTIGUOUS"]:
            raise ValueError("output must be a contiguous int8 array")
        inp = np.ascontiguousarray(input, dtype=np.int8)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_rate_dematch(self._h, output.ctypes.data, output.size,
                                                       inp.ctypes.data if inp.size else None, inp.size,
                                                       int(bool(new_data)), ctypes.byref(c)), "ldpc rate_dematch")
        return output

    def rate_dematch_batch(self, soft, llrs, rm_lengths, new_data: bool, cfg: CodeblockMetadata, in_offsets=None,
                           stream=None):
        """soft: int8 device tensor [nof_cbs, >= N_short*Z] (updated in place);
        llrs: int8 device tensor holding the concatenated rate-matched codeword."""
        import torch

        if soft.dtype != torch.int8 or not soft.is_cuda or soft.dim() != 2 or soft.stride(1) != 1:
            raise ValueError("soft must be a 2-D int8 device tensor with contiguous rows")
        if llrs.dtype != torch.int8 or not llrs.is_cuda:
            raise ValueError("llrs must be an int8 device tensor")
        dev = soft.device
        n = soft.shape[0]
        E = np.asarray(rm_lengths.cpu() if isinstance(rm_lengths, torch.Tensor) else rm_lengths, dtype=np.int64)
        if E.size != n:
            raise ValueError("one rate-matched length per codeblock")
        if in_offsets is None:
            in_offsets = np.concatenate([[0], np.cumsum(E)[:-1]]) if n else np.zeros(0, np.int64)
        d_E = _dev_u32(E, dev)
        d_off = _dev_u32(in_offsets, dev)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_rate_dematch_batch(
            self._h, ctypes.byref(c), int(bool(new_data)), llrs.data_ptr(), d_off.data_ptr(), d_E.data_ptr(),
            soft.data_ptr(), soft.stride(0), n, _stream_arg(stream, soft)), "ldpc rate_dematch_batch")
        return soft


def create_ldpc_encoder_factory_hip():
    """create_ldpc_encoder_factory_sw analog: factory.create() -> LdpcEncoder."""
    return _Factory(LdpcEncoder)


def create_ldpc_rate_matcher_factory_hip():
    return _Factory(LdpcRateMatcher)


def create_ldpc_rate_dematcher_factory_hip(dematcher_type="auto"):
    """create_ldpc_rate_dematcher_factory_sw analog.  Every reference type
    ("generic", "avx2", "avx512", "neon", "auto") gives the same soft buffer for
    finite LLRs; the MI355X dematcher follows "generic" on all inputs."""
    if dematcher_type not in ("auto", "generic", "avx2", "avx512", "neon"):
        raise ValueError("Invalid rate dematcher type %r" % (dematcher_type,))
    return _Factory(LdpcRateDematcher)


class _Factory:
    def __init__(self, cls):
        self._cls = cls

    def create(self, device=-1):
        return self._cls(device)

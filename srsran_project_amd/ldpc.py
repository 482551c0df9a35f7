"""Host-side mirror of srsRAN's LDPC decoder interface over the MI355X C-ABI.

Reference interface (same names, argument meaning and error behaviour):
  include/srsran/phy/upper/channel_coding/ldpc/ldpc_decoder.h:37  class ldpc_decoder
      struct configuration {base_graph, lifting_size, nof_filler_bits, nof_crc_bits, max_iterations}
      std::optional<unsigned> decode(bit_buffer& output, span<const log_likelihood_ratio> input,
                                     crc_calculator* crc, const configuration& cfg)
  include/srsran/phy/upper/channel_coding/channel_coding_factories.h
      create_ldpc_decoder_factory_sw(dec_type, {force_decoding}) -> factory->create()

``decode`` returns the number of iterations when the CRC passed and ``None``
where the reference returns an empty ``std::optional``.  Invalid
configurations raise ``ValueError`` where the reference asserts.

``decode_batch`` is the accelerator form (many codeblocks, device-resident,
one launch on the current torch stream), mirroring the enqueue/dequeue pair of
``hal::hw_accelerator_pusch_dec``.
"""
import ctypes
import enum
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib


class LdpcBaseGraph(enum.IntEnum):
    """include/srsran/ran/sch/ldpc_base_graph.h:31"""

    BG1 = 1
    BG2 = 2


class CrcGeneratorPoly(enum.IntEnum):
    """include/srsran/phy/upper/channel_coding/crc_calculator.h crc_generator_poly"""

    CRC24A = 0
    CRC24B = 1
    CRC24C = 2
    CRC16 = 3
    CRC11 = 4
    CRC6 = 5


LIFTING_SIZES = (2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44,
                 48, 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256,
                 288, 320, 352, 384)

ARITH = {"auto": 0, "avx512": 0, "avx2": 0, "simd": 0, "generic": 1}


@dataclass
class LdpcDecoderConfiguration:
    """ldpc_decoder::configuration (ldpc_decoder.h:40) -- same defaults."""

    base_graph: LdpcBaseGraph = LdpcBaseGraph.BG1
    lifting_size: int = 2
    nof_filler_bits: int = 0
    nof_crc_bits: int = 16
    max_iterations: int = 6

    def to_c(self):
        return _lib.LDPCDecoderConfig(int(self.base_graph), int(self.lifting_size), int(self.nof_filler_bits),
                                      int(self.nof_crc_bits), int(self.max_iterations))


def message_length(base_graph, lifting_size):
    return _lib.lib().srs_amd_ldpc_message_length(int(base_graph), int(lifting_size))


def codeblock_length(base_graph, lifting_size):
    return _lib.lib().srs_amd_ldpc_codeblock_length(int(base_graph), int(lifting_size))


def _crc_arg(crc):
    return -1 if crc is None else int(crc)


class LdpcDecoder:
    """One decoder instance (owns its device scratch), as one factory product."""

    def __init__(self, arith="auto", force_decoding=False, device=-1):
        if arith not in ARITH:
            raise ValueError("Invalid decoder type %r" % (arith,))
        self._lib = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(self._lib.srs_amd_ldpc_decoder_create(ctypes.byref(h), ARITH[arith], int(bool(force_decoding)),
                                                         int(device)), "ldpc_decoder create")
        self._h = h
        self.arith = arith
        self.force_decoding = bool(force_decoding)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.srs_amd_ldpc_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_max_slots(self, n):
        _lib.check(self._lib.srs_amd_ldpc_decoder_set_max_slots(self._h, int(n)), "set_max_slots")

    # -- reference-shaped single-codeblock call (host buffers) --------------
    def decode(self, output: np.ndarray, input: np.ndarray, crc: Optional[CrcGeneratorPoly],
               cfg: LdpcDecoderConfiguration) -> Optional[int]:
        """ldpc_decoder::decode. ``output``: uint8 packed (MSB-first) buffer of
        ceil(K*Z/8) bytes, written in place; ``input``: int8 LLRs."""
        inp = np.ascontiguousarray(input, dtype=np.int8)
        if output.dtype != np.uint8 or not output.flags["C_CONTIGUOUS"]:
            raise ValueError("output must be a contiguous uint8 array")
        K = message_length(cfg.base_graph, cfg.lifting_size)
        if K == 0:
            raise ValueError("Invalid base graph / lifting size (%s, %s)" % (cfg.base_graph, cfg.lifting_size))
        if output.size != (K + 7) // 8:
            raise ValueError("The output size %d is not equal to the message length %d." % (output.size * 8, K))
        c = cfg.to_c()
        it = ctypes.c_int32(-1)
        _lib.check(self._lib.srs_amd_ldpc_decode(self._h, output.ctypes.data, inp.ctypes.data, inp.size,
                                                 _crc_arg(crc), ctypes.byref(c), ctypes.byref(it)), "ldpc decode")
        return None if it.value < 0 else int(it.value)

    # -- accelerator form: many codeblocks, device buffers -------------------
    def decode_batch(self, llrs, cfg: LdpcDecoderConfiguration, crc: Optional[CrcGeneratorPoly] = None,
                     llr_lens=None, out=None, nof_iters=None, soft_out=None, stream=None):
        """Decodes ``llrs`` (torch int8 CUDA tensor [nof_cbs, L]) asynchronously on
        ``stream`` (default: torch's current stream).  Returns (packed bits
        uint8 [nof_cbs, ceil(K*Z/8)], iterations int32 [nof_cbs])."""
        import torch

        if llrs.dtype != torch.int8 or not llrs.is_cuda or llrs.dim() != 2:
            raise ValueError("llrs must be a 2-D int8 device tensor")
        if llrs.stride(1) != 1:
            raise ValueError("llrs rows must be contiguous")
        n, L = llrs.shape
        K = message_length(cfg.base_graph, cfg.lifting_size)
        if K == 0:
            raise ValueError("Invalid base graph / lifting size (%s, %s)" % (cfg.base_graph, cfg.lifting_size))
        ob = (K + 7) // 8
        if out is None:
            out = torch.empty((n, ob), dtype=torch.uint8, device=llrs.device)
        if nof_iters is None:
            nof_iters = torch.empty((n,), dtype=torch.int32, device=llrs.device)
        if llr_lens is not None and (llr_lens.dtype != torch.int32 or not llr_lens.is_cuda):
            raise ValueError("llr_lens must be an int32 device tensor")
        if stream is None:
            stream = torch.cuda.current_stream(llrs.device)
        c = cfg.to_c()
        _lib.check(self._lib.srs_amd_ldpc_decode_batch(
            self._h, ctypes.byref(c), _crc_arg(crc), llrs.data_ptr(), llrs.stride(0),
            llr_lens.data_ptr() if llr_lens is not None else None, L, out.data_ptr(), out.stride(0),
            nof_iters.data_ptr(), soft_out.data_ptr() if soft_out is not None else None, n,
            ctypes.c_void_p(stream.cuda_stream)), "ldpc decode_batch")
        return out, nof_iters


class LdpcDecoderFactory:
    """create_ldpc_decoder_factory_sw analog for the MI355X decoder."""

    def __init__(self, dec_type="auto", force_decoding=False):
        if dec_type not in ARITH:
            raise ValueError("Invalid decoder type %r" % (dec_type,))
        self.dec_type = dec_type
        self.force_decoding = force_decoding

    def create(self, device=-1):
        return LdpcDecoder(self.dec_type, self.force_decoding, device)


def create_ldpc_decoder_factory_hip(dec_type="auto", force_decoding=False):
    return LdpcDecoderFactory(dec_type, force_decoding)

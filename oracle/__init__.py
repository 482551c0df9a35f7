"""ctypes access to the CPU checkers -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline.  The product
(srsran_project_amd) never imports it.

  ORACLE : oracle/libsrs_oracle.so, our C restatement (srs_oracle.c, srs_oracle_rm.c)
  REF    : oracle/_ref/libsrsran_ref.so, the reference's own sources compiled here
           (oracle/Makefile); may be absent, then REF is None.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_PATH = os.path.join(_HERE, "libsrs_oracle.so")
REF_PATH = os.path.join(_HERE, "_ref", "libsrsran_ref.so")

P = ctypes.c_void_p
c_int, c_uint = ctypes.c_int, ctypes.c_uint


def _ptr(a):
    return None if a is None else a.ctypes.data_as(P)


def _load_oracle():
    if not os.path.exists(ORACLE_PATH):
        raise ImportError("oracle not built: %s (run make -C oracle)" % ORACLE_PATH)
    lib = ctypes.CDLL(ORACLE_PATH)
    lib.srs_oracle_ldpc_decode.restype = c_int
    lib.srs_oracle_ldpc_decode.argtypes = [c_int] * 8 + [P, c_uint, P, P]
    lib.srs_oracle_ldpc_encode.restype = c_int
    lib.srs_oracle_ldpc_encode.argtypes = [c_int, c_int, P, P]
    lib.srs_oracle_ldpc_syndrome.restype = c_int
    lib.srs_oracle_ldpc_syndrome.argtypes = [c_int, c_int, P]
    lib.srs_oracle_crc_bits.restype = ctypes.c_uint32
    lib.srs_oracle_crc_bits.argtypes = [c_int, P, c_uint]
    lib.srs_oracle_lifting_index.restype = c_int
    lib.srs_oracle_lifting_index.argtypes = [c_int]
    lib.srs_oracle_polar_code.restype = c_uint
    lib.srs_oracle_polar_code.argtypes = [c_uint, c_uint, c_uint, P, P, P]
    lib.srs_oracle_polar_encode_chain.restype = c_int
    lib.srs_oracle_polar_encode_chain.argtypes = [c_uint, c_uint, c_uint, c_int, P, P]
    lib.srs_oracle_polar_decode_chain.restype = c_int
    lib.srs_oracle_polar_decode_chain.argtypes = [c_uint, c_uint, c_uint, c_int, P, P]
    lib.srs_oracle_polar_interleave.restype = c_int
    lib.srs_oracle_polar_interleave.argtypes = [P, P, c_uint, c_int]
    lib.srs_oracle_demodulate.restype = c_int
    lib.srs_oracle_demodulate.argtypes = [c_int, P, P, c_uint, P]
    lib.srs_oracle_modulate.restype = c_int
    lib.srs_oracle_modulate.argtypes = [c_int, P, c_uint, P]
    lib.srs_oracle_prbs.restype = c_int
    lib.srs_oracle_prbs.argtypes = [ctypes.c_uint32, c_uint, P]
    lib.srs_oracle_ldpc_rate_match.restype = c_int
    lib.srs_oracle_ldpc_rate_match.argtypes = [c_uint] * 6 + [P, c_uint, P]
    lib.srs_oracle_ldpc_rate_dematch.restype = c_int
    lib.srs_oracle_ldpc_rate_dematch.argtypes = [c_uint] * 6 + [c_int, P, c_uint, P]
    return lib


def _load_ref():
    if not os.path.exists(REF_PATH):
        return None
    lib = ctypes.CDLL(REF_PATH)
    lib.srs_ref_has_impl.restype = c_int
    lib.srs_ref_has_impl.argtypes = [ctypes.c_char_p]
    lib.srs_ref_ldpc_decode.restype = c_int
    lib.srs_ref_ldpc_decode.argtypes = [ctypes.c_char_p] + [c_int] * 7 + [P, c_uint, P]
    lib.srs_ref_ldpc_encode.restype = c_int
    lib.srs_ref_ldpc_encode.argtypes = [ctypes.c_char_p, c_int, c_int, P, P, c_uint]
    lib.srs_ref_crc_bits.restype = c_uint
    lib.srs_ref_crc_bits.argtypes = [c_int, P, c_uint]
    lib.srs_ref_ldpc_encode_rate_match.restype = c_int
    lib.srs_ref_ldpc_encode_rate_match.argtypes = [c_int, c_int] + [c_uint] * 4 + [P, c_uint, P]
    lib.srs_ref_ldpc_rate_dematch.restype = c_int
    lib.srs_ref_ldpc_rate_dematch.argtypes = [ctypes.c_char_p, c_int, c_int] + [c_uint] * 4 + [c_int, P, c_uint, P]
    lib.srs_ref_dft.restype = c_int
    lib.srs_ref_dft.argtypes = [c_uint, c_int, P, P]
    lib.srs_ref_ofdm_slot_size.restype = c_uint
    lib.srs_ref_ofdm_slot_size.argtypes = [c_uint, c_uint, c_uint, c_int, c_uint]
    lib.srs_ref_ofdm_modulate_slot.restype = c_int
    lib.srs_ref_ofdm_modulate_slot.argtypes = [c_uint, c_uint, c_uint, c_int, ctypes.c_float, ctypes.c_double, c_uint,
                                               P, P]
    lib.srs_ref_ofdm_demodulate_slot.restype = c_int
    lib.srs_ref_ofdm_demodulate_slot.argtypes = [c_uint, c_uint, c_uint, c_int, c_uint, ctypes.c_float,
                                                 ctypes.c_double, c_uint, P, P]
    lib.srs_ref_ofdm_roundtrip_many.restype = ctypes.c_double
    lib.srs_ref_ofdm_roundtrip_many.argtypes = [c_uint, c_uint, c_uint, P, c_uint, c_uint, c_uint]
    lib.srs_ref_equalizer_is_supported.restype = c_int
    lib.srs_ref_equalizer_is_supported.argtypes = [c_int, c_uint, c_uint]
    lib.srs_ref_equalize.restype = c_int
    lib.srs_ref_equalize.argtypes = [c_int, c_uint, c_uint, c_uint, P, P, P, ctypes.c_float, P, P]
    lib.srs_ref_equalize_many.restype = ctypes.c_double
    lib.srs_ref_equalize_many.argtypes = [c_uint, c_uint, c_uint, P, P, P, c_uint, c_uint]
    lib.srs_ref_polar_code.restype = c_uint
    lib.srs_ref_polar_code.argtypes = [c_uint, c_uint, c_uint, P, P, P]
    lib.srs_ref_polar_encode_chain.restype = c_int
    lib.srs_ref_polar_encode_chain.argtypes = [c_uint, c_uint, c_uint, c_int, P, P]
    lib.srs_ref_polar_decode_chain.restype = c_int
    lib.srs_ref_polar_decode_chain.argtypes = [c_uint, c_uint, c_uint, c_int, P, P]
    lib.srs_ref_polar_interleave.restype = c_int
    lib.srs_ref_polar_interleave.argtypes = [P, P, c_uint, c_int]
    lib.srs_ref_polar_decode_many.restype = ctypes.c_double
    lib.srs_ref_polar_decode_many.argtypes = [c_uint, c_uint, c_uint, P, c_uint, c_uint, c_uint]
    lib.srs_ref_modulate.restype = c_int
    lib.srs_ref_modulate.argtypes = [c_int, P, c_uint, P]
    lib.srs_ref_demodulate.restype = c_int
    lib.srs_ref_demodulate.argtypes = [c_int, P, P, c_uint, P]
    lib.srs_ref_prbs.restype = c_int
    lib.srs_ref_prbs.argtypes = [ctypes.c_uint32, c_uint, P]
    lib.srs_ref_descramble_llrs.restype = c_int
    lib.srs_ref_descramble_llrs.argtypes = [ctypes.c_uint32, c_uint, P, P]
    lib.srs_ref_scramble_bits.restype = c_int
    lib.srs_ref_scramble_bits.argtypes = [ctypes.c_uint32, c_uint, P, P]
    lib.srs_ref_pdsch_encode.restype = c_int
    lib.srs_ref_pdsch_encode.argtypes = [P, c_uint] + [c_uint] * 6 + [P]
    lib.srs_ref_rx_buffer_create.restype = ctypes.c_void_p
    lib.srs_ref_rx_buffer_create.argtypes = [c_uint]
    lib.srs_ref_rx_buffer_destroy.restype = None
    lib.srs_ref_rx_buffer_destroy.argtypes = [ctypes.c_void_p]
    lib.srs_ref_pusch_decode.restype = c_int
    lib.srs_ref_pusch_decode.argtypes = [ctypes.c_void_p, P, c_uint, P, c_uint] + [c_uint] * 6 + [c_int] * 4 + [P]
    lib.srs_ref_ldpc_decode_many.restype = ctypes.c_double
    lib.srs_ref_ldpc_decode_many.argtypes = [ctypes.c_char_p, c_int, c_int, c_int, c_int, P, c_uint, c_uint, c_uint,
                                             c_int, P, P]
    return lib


ORACLE = _load_oracle()
REF = _load_ref()

BG_K = {1: 22, 2: 10}
BG_N_SHORT = {1: 66, 2: 50}
BG_N_FULL = {1: 68, 2: 52}
ARITH = {"simd": 0, "avx512": 0, "avx2": 0, "auto": 0, "generic": 1}


def ldpc_decode(llrs, bg, Z, max_iterations=6, arith="simd", crc_poly=None, nof_filler_bits=0, nof_crc_bits=16,
                force_decoding=False, want_soft=False):
    """Oracle decode of one codeblock. Returns (iterations or None, packed bits, soft or None)."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    K = BG_K[bg] * Z
    out = np.zeros((K + 7) // 8, np.uint8)
    soft = np.zeros(BG_N_FULL[bg] * Z, np.int8) if want_soft else None
    r = ORACLE.srs_oracle_ldpc_decode(bg, Z, nof_filler_bits, nof_crc_bits, max_iterations, ARITH[arith],
                                      int(force_decoding), -1 if crc_poly is None else int(crc_poly), _ptr(llrs),
                                      llrs.size, _ptr(out), _ptr(soft))
    if r == -2:
        raise ValueError("invalid decoder arguments")
    return (None if r < 0 else r), out, soft


def ldpc_encode(msg_bits, bg, Z):
    """Oracle systematic encode: K message bits -> N_short*Z codeblock bits (one per byte)."""
    msg_bits = np.ascontiguousarray(msg_bits, dtype=np.uint8)
    cw = np.zeros(BG_N_SHORT[bg] * Z, np.uint8)
    if ORACLE.srs_oracle_ldpc_encode(bg, Z, _ptr(msg_bits), _ptr(cw)) != 0:
        raise ValueError("invalid encoder arguments")
    return cw


def crc_bits(poly, bits):
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    return int(ORACLE.srs_oracle_crc_bits(int(poly), _ptr(bits), bits.size))


def ref_ldpc_decode(impl, llrs, bg, Z, max_iterations=6, crc_poly=None, nof_filler_bits=0, nof_crc_bits=16,
                    force_decoding=False, out_init=None):
    """Reference decoder (compiled from /root/reference). Returns (iterations or None, packed bits)."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    K = BG_K[bg] * Z
    out = np.zeros((K + 7) // 8, np.uint8) if out_init is None else out_init.copy()
    r = REF.srs_ref_ldpc_decode(impl.encode(), bg, Z, nof_filler_bits, nof_crc_bits, max_iterations,
                                int(force_decoding), -1 if crc_poly is None else int(crc_poly), _ptr(llrs),
                                llrs.size, _ptr(out))
    if r == -2:
        raise ValueError("reference implementation %r unavailable" % impl)
    return (None if r < 0 else r), out


def ref_ldpc_encode(msg_bits, bg, Z, n_out=None, impl="generic"):
    msg_bits = np.ascontiguousarray(msg_bits, dtype=np.uint8)
    n = BG_N_SHORT[bg] * Z if n_out is None else n_out
    cw = np.zeros(n, np.uint8)
    if REF.srs_ref_ldpc_encode(impl.encode(), bg, Z, _ptr(msg_bits), _ptr(cw), n) != 0:
        raise ValueError("reference encoder %r unavailable" % impl)
    return cw


def pack_bits(bits):
    return np.packbits(np.asarray(bits, dtype=np.uint8))


def unpack_bits(packed, n):
    return np.unpackbits(np.asarray(packed, dtype=np.uint8))[:n]


def rate_match(cw_bits, bg, Z, rv, Qm, E, Nref=0, filler=0):
    """Oracle rate matching of a full codeblock (one bit per byte) -> E packed bits."""
    cw_bits = np.ascontiguousarray(cw_bits, dtype=np.uint8)
    out = np.zeros((E + 7) // 8, np.uint8)
    if ORACLE.srs_oracle_ldpc_rate_match(bg, Z, rv, Qm, Nref, filler, _ptr(cw_bits), E, _ptr(out)) != 0:
        raise ValueError("invalid rate matching arguments")
    return out


def rate_dematch(llrs, bg, Z, rv, Qm, buf, new_data=True, Nref=0, filler=0):
    """Oracle rate dematching of E LLRs into the soft buffer `buf` (modified in place)."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    assert buf.dtype == np.int8 and buf.flags["C_CONTIGUOUS"]
    if ORACLE.srs_oracle_ldpc_rate_dematch(bg, Z, rv, Qm, Nref, filler, int(new_data), _ptr(llrs), llrs.size,
                                           _ptr(buf)) != 0:
        raise ValueError("invalid rate dematching arguments")
    return buf


def ref_encode_rate_match(msg_bits, bg, Z, rv, Qm, E, Nref=0, filler=0):
    msg_bits = np.ascontiguousarray(msg_bits, dtype=np.uint8)
    out = np.zeros((E + 7) // 8, np.uint8)
    REF.srs_ref_ldpc_encode_rate_match(bg, Z, rv, Qm, Nref, filler, _ptr(msg_bits), E, _ptr(out))
    return out


def ref_rate_dematch(llrs, bg, Z, rv, Qm, buf, new_data=True, Nref=0, filler=0, impl="generic"):
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    if REF.srs_ref_ldpc_rate_dematch(impl.encode(), bg, Z, rv, Qm, Nref, filler, int(new_data), _ptr(llrs), llrs.size,
                                     _ptr(buf)) != 0:
        raise ValueError("reference dematcher %r unavailable" % impl)
    return buf


def ref_dft(x, inverse=False):
    x = np.ascontiguousarray(x, dtype=np.complex64)
    out = np.zeros_like(x)
    if REF.srs_ref_dft(x.size, int(inverse), _ptr(x), _ptr(out)) != 0:
        raise ValueError("reference DFT size %d not supported" % x.size)
    return out


def ref_ofdm_modulate_slot(grid_u16, slot, numerology, bw_rb, dft_size, scale, fc, extended_cp=False):
    grid_u16 = np.ascontiguousarray(grid_u16, dtype=np.uint16)
    n = REF.srs_ref_ofdm_slot_size(numerology, bw_rb, dft_size, int(extended_cp), slot)
    out = np.zeros(n, np.complex64)
    REF.srs_ref_ofdm_modulate_slot(numerology, bw_rb, dft_size, int(extended_cp), scale, fc, slot, _ptr(grid_u16),
                                   _ptr(out))
    return out


def ref_ofdm_demodulate_slot(samples, slot, numerology, bw_rb, dft_size, scale, fc, window_offset=0,
                             extended_cp=False):
    samples = np.ascontiguousarray(samples, dtype=np.complex64)
    ns = 12 if extended_cp else 14
    grid = np.zeros((ns, 2 * bw_rb * 12), np.uint16)
    REF.srs_ref_ofdm_demodulate_slot(numerology, bw_rb, dft_size, int(extended_cp), window_offset, scale, fc, slot,
                                     _ptr(samples), _ptr(grid))
    return grid


def ref_equalize(symbols_u16, est_u16, noise_vars, tx_scaling, nof_layers, mmse=False):
    symbols_u16 = np.ascontiguousarray(symbols_u16, dtype=np.uint16)
    est_u16 = np.ascontiguousarray(est_u16, dtype=np.uint16)
    nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
    P = symbols_u16.shape[0]
    R = symbols_u16.shape[1] // 2
    eq = np.zeros((R, nof_layers), np.complex64)
    nvo = np.zeros((R, nof_layers), np.float32)
    if REF.srs_ref_equalize(int(mmse), R, P, nof_layers, _ptr(symbols_u16), _ptr(est_u16), _ptr(nv),
                            float(tx_scaling), _ptr(eq), _ptr(nvo)) != 0:
        raise ValueError("reference equalizer does not support %d ports x %d layers" % (P, nof_layers))
    return eq, nvo


def _polar_code(lib, K, E, nMax):
    kmask = np.zeros(1024, np.uint8)
    pc = np.zeros(8, np.uint16)
    npc = ctypes.c_uint(0)
    N = lib(K, E, nMax, _ptr(kmask), _ptr(pc), ctypes.byref(npc))
    if N == 0:
        raise ValueError("invalid polar code K=%d E=%d nMax=%d" % (K, E, nMax))
    return N, kmask[:N].copy(), pc[:npc.value].copy()


def polar_code(K, E, nMax):
    """(N, K_set mask [N], PC set) as polar_code::set builds them."""
    return _polar_code(ORACLE.srs_oracle_polar_code, K, E, nMax)


def ref_polar_code(K, E, nMax):
    return _polar_code(REF.srs_ref_polar_code, K, E, nMax)


def polar_encode_chain(msg_bits, E, nMax, ibil=False, lib=None):
    msg = np.ascontiguousarray(msg_bits, dtype=np.uint8)
    out = np.zeros(E, np.uint8)
    f = ORACLE.srs_oracle_polar_encode_chain if lib is None else lib.srs_ref_polar_encode_chain
    if f(msg.size, E, nMax, int(ibil), _ptr(msg), _ptr(out)) != 0:
        raise ValueError("invalid polar code")
    return out


def ref_polar_encode_chain(msg_bits, E, nMax, ibil=False):
    return polar_encode_chain(msg_bits, E, nMax, ibil, lib=REF)


def polar_decode_chain(llrs, K, nMax, ibil=False, lib=None):
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    msg = np.zeros(K, np.uint8)
    f = ORACLE.srs_oracle_polar_decode_chain if lib is None else lib.srs_ref_polar_decode_chain
    if f(K, llrs.size, nMax, int(ibil), _ptr(llrs), _ptr(msg)) != 0:
        raise ValueError("invalid polar code")
    return msg


def ref_polar_decode_chain(llrs, K, nMax, ibil=False):
    return polar_decode_chain(llrs, K, nMax, ibil, lib=REF)


def polar_interleave(bits, direction=0, lib=None):
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    out = np.zeros_like(bits)
    f = ORACLE.srs_oracle_polar_interleave if lib is None else lib.srs_ref_polar_interleave
    if f(_ptr(bits), _ptr(out), bits.size, int(direction)) != 0:
        raise ValueError("K > 164")
    return out


QM_CODE = {"pi/2-BPSK": 0, "BPSK": 1, "QPSK": 2, "QAM16": 4, "QAM64": 6, "QAM256": 8}


def _bits_per_symbol(qm):
    return 1 if qm in (0, 1) else qm


def demodulate(symbols, noise_vars, qm, lib=None):
    """Soft demapping: complex64 symbols, float32 noise variances -> int8 LLRs."""
    sym = np.ascontiguousarray(symbols, dtype=np.complex64)
    nv = np.ascontiguousarray(noise_vars, dtype=np.float32)
    out = np.zeros(sym.size * _bits_per_symbol(qm), np.int8)
    f = ORACLE.srs_oracle_demodulate if lib is None else lib.srs_ref_demodulate
    if f(qm, _ptr(sym), _ptr(nv), sym.size, _ptr(out)) != 0:
        raise ValueError("invalid modulation")
    return out


def ref_demodulate(symbols, noise_vars, qm):
    return demodulate(symbols, noise_vars, qm, lib=REF)


def modulate(bits_packed, nsym, qm, lib=None):
    b = np.ascontiguousarray(bits_packed, dtype=np.uint8)
    out = np.zeros(nsym, np.complex64)
    f = ORACLE.srs_oracle_modulate if lib is None else lib.srs_ref_modulate
    if f(qm, _ptr(b), nsym, _ptr(out)) != 0:
        raise ValueError("invalid modulation")
    return out


def ref_modulate(bits_packed, nsym, qm):
    return modulate(bits_packed, nsym, qm, lib=REF)


def prbs(c_init, length, lib=None):
    """Gold sequence c(0..length-1), one bit per byte."""
    out = np.zeros(length, np.uint8)
    f = ORACLE.srs_oracle_prbs if lib is None else lib.srs_ref_prbs
    if f(c_init, length, _ptr(out)) != 0:
        raise ValueError("sequence too long")
    return out


def ref_prbs(c_init, length):
    return prbs(c_init, length, lib=REF)


def ref_pdsch_encode(tb_bytes, p):
    """Reference pdsch_encoder_impl::encode; p: an oracle.sch.plan() dict. Codeword bits, one per byte."""
    tb = np.ascontiguousarray(tb_bytes, dtype=np.uint8)
    cw = np.zeros(p["cw_length"], np.uint8)
    REF.srs_ref_pdsch_encode(_ptr(tb), tb.size, p["base_graph"], p["rv"], p["modulation_order"], p["Nref"],
                             p["nof_layers"], p["nof_ch_symbols"], _ptr(cw))
    return cw


class RefRxBuffer:
    """HARQ soft buffer of the reference PUSCH decoder."""

    def __init__(self, nof_cbs):
        self.h = REF.srs_ref_rx_buffer_create(nof_cbs)

    def __del__(self):
        if getattr(self, "h", None):
            REF.srs_ref_rx_buffer_destroy(self.h)
            self.h = None


def ref_pusch_decode(llrs, p, rxbuf, tb_out, max_iterations=6, generic=False, use_early_stop=True,
                     force_decoding=False, new_data=True):
    """Reference pusch_decoder_impl. Returns (tb_crc_ok, nof_cbs, nof_obs, iteration sum, min, max)."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    res = np.zeros(6, np.float64)
    r = REF.srs_ref_pusch_decode(rxbuf.h, _ptr(llrs), llrs.size, _ptr(tb_out), tb_out.size, p["base_graph"], p["rv"],
                                 p["modulation_order"], p["Nref"], p["nof_layers"], max_iterations,
                                 int(force_decoding), int(use_early_stop), int(new_data), int(generic), _ptr(res))
    if r != 0:
        raise RuntimeError("reference PUSCH decoder did not notify")
    return bool(res[0]), int(res[1]), int(res[2]), int(round(res[3])), int(res[4]), int(res[5])

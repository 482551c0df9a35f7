"""CPU oracle of the shared-channel transport-block chain -- TEST INFRASTRUCTURE ONLY.

Restates (pinned against the reference's own pdsch_encoder_impl / pusch_decoder_impl,
compiled into oracle/_ref by oracle/Makefile, in tests/test_oracle_vs_ref.py):
  plan()         ldpc_segmenter_tx_impl.cpp:53-123, ldpc.h:128-207, ldpc_segmenter_helpers.h:82-94
  pdsch_encode() pdsch_encoder_impl.cpp:28-80 with read_codeblock (ldpc_segmenter_tx_impl.cpp:137-207)
  pusch_decode() pusch_decoder_impl.cpp:87-503 (+ pusch_codeblock_decoder.cpp:35-86)
on top of the codeblock-level oracle (crc_bits, ldpc_encode, rate_match,
rate_dematch, ldpc_decode in oracle/__init__.py).
"""
import numpy as np

from . import (BG_K, BG_N_SHORT, crc_bits, ldpc_decode, ldpc_encode, pack_bits, rate_dematch, rate_match,
               unpack_bits)

LIFTING_SIZES = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48,
                 52, 56, 60, 64, 72, 80, 88, 96, 104, 112, 120, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320,
                 352, 384]
CRC24A, CRC24B, CRC16 = 0, 1, 3


def _ceil(a, b):
    return -(-a // b)


def plan(tbs, bg, rv, qm, Nref, nof_layers, nof_ch_symbols):
    """Segmentation geometry as a dict (the fields of srs_amd_sch_plan)."""
    assert tbs > 0 and tbs % 8 == 0 and tbs + 24 <= 1277992
    assert nof_ch_symbols % nof_layers == 0
    tb_crc = 16 if tbs <= 3824 else 24
    b = tbs + tb_crc
    max_seg = 8448 if bg == 1 else 3840
    C = 1 if b <= max_seg else _ceil(b, max_seg - 24)
    ref = 22
    if bg == 2:
        ref = 10 if b > 640 else 9 if b > 560 else 8 if b > 192 else 6
    b_out = b + (24 * C if C > 1 else 0)
    Z = next(ls for ls in LIFTING_SIZES if ls * C * ref >= b_out)
    K = BG_K[bg] * Z
    L = 24 if C > 1 else 0
    cbi = _ceil(b_out, C) - L
    per_layer = nof_ch_symbols // nof_layers
    p = dict(tbs=tbs, base_graph=bg, rv=rv, modulation_order=qm, Nref=Nref, nof_layers=nof_layers,
             nof_ch_symbols=nof_ch_symbols, lifting_size=Z, segment_length=K, nof_segments=C, nof_tb_crc_bits=tb_crc,
             nof_crc_bits=L, cb_info_bits=cbi, zero_pad=(cbi + L) * C - b_out, nof_filler_bits=K - cbi - L,
             nof_short_segments=C - per_layer % C, rm_length_short=per_layer // C * nof_layers * qm,
             rm_length_long=_ceil(per_layer, C) * nof_layers * qm, cw_length=nof_ch_symbols * qm)
    return p


def segments(p):
    """[(E_r, cw_offset_r)] per segment."""
    out, off = [], 0
    for r in range(p["nof_segments"]):
        E = p["rm_length_short"] if r < p["nof_short_segments"] else p["rm_length_long"]
        out.append((E, off))
        off += E
    return out


def _tb_crc_poly(p):
    return CRC16 if p["nof_tb_crc_bits"] == 16 else CRC24A


def pdsch_encode(tb_bytes, p):
    """TB bytes -> codeword bits (one per byte, cw_length entries)."""
    tb = np.unpackbits(np.asarray(tb_bytes, np.uint8))
    assert tb.size == p["tbs"]
    L_tb = p["nof_tb_crc_bits"]
    c = crc_bits(_tb_crc_poly(p), tb)
    tb_crc = np.array([(c >> (L_tb - 1 - k)) & 1 for k in range(L_tb)], np.uint8)
    stream = np.concatenate([tb, tb_crc])
    C, cbi, K, Z, bg = p["nof_segments"], p["cb_info_bits"], p["segment_length"], p["lifting_size"], p["base_graph"]
    cw = np.zeros(p["cw_length"], np.uint8)
    for r, (E, off) in enumerate(segments(p)):
        msg = np.zeros(K, np.uint8)
        seg = stream[r * cbi:(r + 1) * cbi]       # the last one is short by the zero pad
        msg[:seg.size] = seg
        if C > 1:
            cc = crc_bits(CRC24B, msg[:cbi])
            msg[cbi:cbi + 24] = [(cc >> (23 - k)) & 1 for k in range(24)]
        coded = ldpc_encode(msg, bg, Z)
        rm = rate_match(coded, bg, Z, p["rv"], p["modulation_order"], E, p["Nref"], p["nof_filler_bits"])
        cw[off:off + E] = unpack_bits(rm, E)
    return cw


class HarqBuffer:
    """The rx_buffer of one HARQ process: soft bits, decoded messages and CB CRC flags."""

    def __init__(self, p):
        C, bg, Z = p["nof_segments"], p["base_graph"], p["lifting_size"]
        self.soft = [np.zeros(BG_N_SHORT[bg] * Z, np.int8) for _ in range(C)]
        self.msgs = [np.zeros(_ceil(p["segment_length"], 8), np.uint8) for _ in range(C)]
        self.crc = [False] * C
        self.its = [0] * C  # iterations of the decoding that set crc[r]


def pusch_decode(llrs, p, harq, tb_out, max_iterations=6, arith="simd", use_early_stop=True, force_decoding=False,
                 new_data=True):
    """Codeword LLRs -> tb_out (bytes, written only where the reference writes them).
    Returns (tb_crc_ok, per-CB iterations (None = CRC failed) as decoded now, stats list)."""
    llrs = np.asarray(llrs, np.int8)
    C, cbi, K, Z, bg = p["nof_segments"], p["cb_info_bits"], p["segment_length"], p["lifting_size"], p["base_graph"]
    F = p["nof_filler_bits"]
    crc_poly = CRC24B if C > 1 else _tb_crc_poly(p)
    nof_crc = 24 if C > 1 else p["nof_tb_crc_bits"]
    if new_data:
        harq.crc = [False] * C
    iters, stats = [], []
    for r, (E, off) in enumerate(segments(p)):
        rate_dematch(llrs[off:off + E], bg, Z, p["rv"], p["modulation_order"], harq.soft[r], new_data, p["Nref"], F)
        if harq.crc[r]:
            # not decoded again; the reference's cb_stats[r] is not updated and holds the iterations of the
            # decoding that passed (pusch_decoder_impl.cpp:333-345, for one decoder object serving the process)
            iters.append(None)
            stats.append(harq.its[r])
            continue
        if use_early_stop:
            it, msg, _ = ldpc_decode(harq.soft[r], bg, Z, max_iterations, arith, crc_poly, F, nof_crc, force_decoding)
        else:
            _, msg, _ = ldpc_decode(harq.soft[r], bg, Z, max_iterations, arith, None, F, nof_crc, force_decoding)
            it = max_iterations if crc_bits(crc_poly, unpack_bits(msg, K - F)) == 0 else None
        harq.msgs[r] = msg
        if it is not None:
            harq.crc[r] = True
            harq.its[r] = it
        iters.append(it)
        stats.append(it if it is not None else max_iterations)
    tbs = p["tbs"]
    if C == 1:
        ok = harq.crc[0]
        if ok:
            tb_out[:tbs // 8] = harq.msgs[0][:tbs // 8]
        return ok, iters, stats
    if not all(harq.crc):
        return False, iters, stats
    bits = np.concatenate([unpack_bits(harq.msgs[r], cbi) for r in range(C)])
    tb_bits = bits[:tbs]
    chk = 0
    for k in range(24):
        chk = (chk << 1) | int(bits[tbs + k])
    tb_out[:tbs // 8] = pack_bits(tb_bits)
    ok = crc_bits(CRC24A, tb_bits) == chk
    if not ok:
        harq.crc = [False] * C
    return ok, iters, stats

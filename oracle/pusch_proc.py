"""The REFERENCE's own PUSCH processor and a UE PUSCH transmitter -- TEST
INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg).

ref_pusch_process: pusch_processor_impl::process (pusch_processor_impl.cpp:134-386)
compiled from /root/reference (oracle/ref_wrapper_pusch.cpp, ref_builders.h),
configured as the reference PUSCH processor benchmark (ZF, filter FD smoothing,
interpolate TD, CFO compensation, `iterations` LDPC iterations with early stop).

ue_transmit: a UE PUSCH transmission without transform precoding built from the
reference's own transmit classes (pdsch_encoder_impl for the UL-SCH coding --
identical TS 38.212 6.2 chain --, pdsch_modulator_impl for scrambling with
c_init = rnti * 2^15 + n_id, modulation and RE mapping, dmrs_pdsch_processor_impl
for the type-1 pseudo-random DM-RS of TS 38.211 6.4.1.1 -- the same sequence and
mapping as PDSCH), DM-RS amplitude = the processor's estimator scaling
convert_dB_to_amplitude(-beta_DMRS) (pusch_processor_impl.cpp:193).
"""
import ctypes as _c

import numpy as np

from . import REF, RefRxBuffer, _ptr, ref_pdsch_encode
from . import sch as osch

CHOICE = {"generic": 0, "avx2": 1, "auto": 2}
BETA_DMRS_DB = {1: 0.0, 2: -3.0, 3: -4.77}

if REF is not None and hasattr(REF, "srs_ref_pusch_process"):
    REF.srs_ref_pusch_process.restype = _c.c_int
    REF.srs_ref_pusch_process.argtypes = ([_c.c_void_p] + [_c.c_uint] * 7 + [_c.c_int, _c.c_float, _c.c_uint,
                                                                             _c.c_uint, _c.c_int, _c.c_uint,
                                                                             _c.c_uint, _c.c_uint, _c.c_int, _c.c_uint,
                                                                             _c.c_int, _c.c_uint]
                                          + [_c.c_uint] * 6 + [_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_uint,
                                                               _c.c_void_p, _c.c_void_p]
                                          + [_c.c_uint, _c.c_uint, _c.c_float, _c.c_float, _c.c_float]
                                          + [_c.c_void_p] * 3)
    REF.srs_ref_describe_choice.restype = _c.c_char_p
    REF.srs_ref_describe_choice.argtypes = [_c.c_int]


def dmrs_scaling(nof_cdm_groups_without_data):
    return float(np.power(np.float32(10.0), np.float32(-BETA_DMRS_DB[nof_cdm_groups_without_data]) / np.float32(20.0)))


def nof_codeblocks(tbs, bg):
    b = tbs + (24 if tbs > 3824 else 16)
    m = 8448 if bg == 1 else 3840
    return 1 if b <= m else -(-b // (m - 24))


def nref(tbs, bg, tbs_lbrm_bytes=0):
    lbrm = tbs_lbrm_bytes or 159749
    return min(lbrm * 8 * 3 // (2 * nof_codeblocks(tbs, bg)), 384 * 66)


def describe(choice="auto"):
    return REF.srs_ref_describe_choice(CHOICE[choice]).decode()


def ref_pusch_process(grid, pdu, tb_bytes, iterations=2, choice="auto", rx_buffer=None):
    """grid uint32 [P][14][nsubc]; pdu: dict with the PuschPdu fields (transform_precoding / n_rs_id: the
    dmrs_transform_precoding_configuration; dc_position: pdu_t::dc_position; tbs = 0 / tb_bytes = 0: a PDU without
    codeword, UCI only). Returns (tb, result dict)."""
    if REF is None:
        raise RuntimeError("oracle/_ref not built")
    g = np.ascontiguousarray(grid, np.uint32)
    P, _, nsubc = g.shape
    tp = bool(pdu.get("transform_precoding", 0))
    uci_only = tb_bytes == 0
    C = 1 if uci_only else nof_codeblocks(tb_bytes * 8, pdu["base_graph"])
    buf = rx_buffer or RefRxBuffer(C)
    dc = pdu.get("dc_position")
    if dc is not None or uci_only:
        f = REF.srs_ref_pusch_set_options
        f.restype = None
        f.argtypes = [_c.c_int, _c.c_int]
        f(-1 if dc is None else int(dc), int(uci_only))
    tb = np.zeros(max(tb_bytes, 1), np.uint8)
    res = np.zeros(6, np.float64)
    csi = np.zeros(4, np.float64)
    ack = np.zeros(max(1, pdu.get("nof_harq_ack", 0)), np.uint8)
    csi1 = np.zeros(max(1, pdu.get("nof_csi_part1", 0)), np.uint8)
    ust = np.zeros(2, np.int32)
    part2 = pdu.get("csi_part2_size")
    if part2:
        f = REF.srs_ref_pusch_set_csi_part2
        f.restype = None
        f.argtypes = [_c.c_void_p, _c.c_uint, _c.c_float]
        w = part2_words(part2)
        f(_ptr(w), w.size, float(pdu.get("beta_offset_csi_part2", 5.0)))
    r = REF.srs_ref_pusch_process(
        _ptr(g), P, nsubc, pdu["numerology"], pdu["slot_index"], pdu["rnti"], pdu["bwp_start_rb"], pdu["bwp_size_rb"],
        pdu["modulation"], float(pdu["target_code_rate"]), pdu["rv"], pdu["base_graph"], int(pdu["new_data"]),
        pdu["n_id"], pdu["nof_tx_layers"], pdu["dmrs_symbol_mask"], 2 if tp else 0,
        pdu.get("n_rs_id", 0) if tp else pdu["scrambling_id"], int(pdu["n_scid"]),
        pdu["nof_cdm_groups_without_data"], pdu["rb_start"], pdu["rb_count"], pdu["start_symbol_index"],
        pdu["nof_symbols"], pdu.get("tbs_lbrm_bytes", 0), iterations, CHOICE[choice], buf.h, _ptr(tb), tb_bytes,
        _ptr(res), _ptr(csi), pdu.get("nof_harq_ack", 0), pdu.get("nof_csi_part1", 0),
        float(pdu.get("alpha_scaling", 1.0)), float(pdu.get("beta_offset_harq_ack", 5.0)),
        float(pdu.get("beta_offset_csi_part1", 5.0)), _ptr(ack), _ptr(csi1), _ptr(ust))
    if r != 0:
        raise RuntimeError("reference PUSCH processor did not notify")
    csi2, st2 = np.zeros(4096, np.uint8), np.zeros(1, np.int32)
    g = REF.srs_ref_pusch_get_csi_part2
    g.restype = _c.c_int
    g.argtypes = [_c.c_void_p, _c.c_uint, _c.c_void_p]
    n2 = g(_ptr(csi2), csi2.size, _ptr(st2))
    tb = tb[:tb_bytes]
    return tb, dict(csi_part2=csi2[:n2].copy(), csi_part2_status=int(st2[0]),
                    tb_crc_ok=bool(res[0]), nof_codeblocks_total=int(res[1]), nof_observations=int(res[2]),
                    iterations_sum=int(round(res[3])) if res[2] else 0, iterations_min=int(res[4]) if res[2] else 0,
                    iterations_max=int(res[5]) if res[2] else 0,
                    sinr_db=csi[0], epre_db=csi[1], rsrp_db=csi[2], time_alignment_s=csi[3],
                    harq_ack=ack[:pdu.get("nof_harq_ack", 0)], csi_part1=csi1[:pdu.get("nof_csi_part1", 0)],
                    harq_ack_status=int(ust[0]), csi_part1_status=int(ust[1]))


def ue_transmit(tb, pdu, nsubc, channel=None, snr_db=None, seed=0, nof_rx_ports=None, uci=None):
    """UE PUSCH transmission of transport block bytes `tb` for `pdu` (dict), through `channel`
    (complex [layer][rx port], default identity) plus AWGN at snr_db (None: noiseless).  uci: optional
    (HARQ-ACK bits, CSI part 1 bits) multiplexed with the UL-SCH (ue_multiplex_uci).
    Returns the received grid uint32 [rx ports][14][nsubc] (cbf16) and the UL-SCH plan."""
    from .pdsch_mod import ref_dmrs_pdsch_map, ref_pdsch_modulate, to_bf16
    from .pusch_demod import data_re_mask

    L = pdu["nof_tx_layers"]
    P = nof_rx_ports or pdu["nof_rx_ports"]
    if channel is None:
        channel = np.eye(L, P, dtype=np.complex64)
    channel = np.asarray(channel, np.complex64)
    crb0 = pdu["bwp_start_rb"] + pdu["rb_start"]
    crbs = list(range(crb0, crb0 + pdu["rb_count"]))
    mask = data_re_mask(nsubc, crbs, pdu["start_symbol_index"], pdu["nof_symbols"], pdu["dmrs_symbol_mask"], False,
                        pdu["nof_cdm_groups_without_data"])
    nre = int(mask.sum())
    tbs = len(tb) * 8
    nch = nre * L
    info = None
    if uci is not None:
        info = ref_ulsch_information(pdu, tbs, len(uci[2]) if len(uci) > 2 else 0)
        nch = info["nof_ul_sch_bits"] // pdu["modulation"]
    if tbs == 0:  # UCI only: the codeword is the multiplexed UCI alone
        p, cw = None, np.zeros(0, np.uint8)
    else:
        p = osch.plan(tbs, pdu["base_graph"], pdu["rv"], pdu["modulation"], nref(tbs, pdu["base_graph"],
                                                                                pdu.get("tbs_lbrm_bytes", 0)),
                      L, nch)
        cw = ref_pdsch_encode(np.asarray(tb, np.uint8), p)
    if uci is not None:
        cw = ue_multiplex_uci(cw, pdu, info, nre * L * pdu["modulation"], uci[0], uci[1],
                              uci[2] if len(uci) > 2 else ())
    grid = np.zeros((P, 14, nsubc, 2), np.uint16)
    ref_pdsch_modulate(grid, cw, pdu["rnti"], pdu["n_id"], pdu["modulation"], crbs, pdu["start_symbol_index"],
                       pdu["nof_symbols"], pdu["dmrs_symbol_mask"], False, pdu["nof_cdm_groups_without_data"], [],
                       channel, 1.0, bwp=(0, nsubc // 12))
    ref_dmrs_pdsch_map(grid, pdu["slot_index"], 0, False, pdu["scrambling_id"], pdu["n_scid"],
                       dmrs_scaling(pdu["nof_cdm_groups_without_data"]), pdu["dmrs_symbol_mask"], crbs,
                       channel[None], numerology=pdu["numerology"])
    g = grid.view(np.uint32).reshape(P, 14, nsubc)
    if snr_db is not None:
        f = np.stack([((g & 0xFFFF) << 16).view(np.float32), ((g >> 16) << 16).view(np.float32)], -1)
        z = f[..., 0] + 1j * f[..., 1]
        occ = np.abs(z) > 0
        pw = float(np.mean(np.abs(z[occ]) ** 2))
        rng = np.random.default_rng(seed)
        sigma = np.sqrt(pw / 10 ** (snr_db / 10) / 2)
        z = z + sigma * (rng.normal(size=z.shape) + 1j * rng.normal(size=z.shape))
        g = (to_bf16(z.real.astype(np.float32)).astype(np.uint32)
             | (to_bf16(z.imag.astype(np.float32)).astype(np.uint32) << 16))
    return np.ascontiguousarray(g), p


def ue_transmit_tp(tb, pdu, nsubc, channel=None, snr_db=None, seed=0):
    """UE PUSCH transmission with transform precoding (DFT-s-OFDM, TS 38.211 6.3.1.4 / 6.4.1.1.1.2): the
    reference's PDSCH-style encoder chain for the codeword, the reference's Gold sequence and modulation mapper,
    an M-point forward DFT scaled by 1/sqrt(M) per data OFDM symbol (numpy, float64 then float32), and the
    reference's low-PAPR DM-RS (r_{n_rs_id mod 30, 0}) on the even subcarriers of the DM-RS symbols at the
    two-CDM-group DM-RS amplitude; one layer through `channel` (complex [rx ports]) plus AWGN.
    Returns the received grid uint32 [P][14][nsubc] (cbf16) and the UL-SCH plan."""
    from . import ref_modulate, ref_prbs
    from .chest import ref_low_papr
    from .pdsch_mod import to_bf16

    P = pdu["nof_rx_ports"]
    channel = np.ones(P, np.complex64) if channel is None else np.asarray(channel, np.complex64).reshape(P)
    crb0 = pdu["bwp_start_rb"] + pdu["rb_start"]
    nrb = pdu["rb_count"]
    M = 12 * nrb
    dmrs = pdu["dmrs_symbol_mask"]
    data_syms = [l for l in range(pdu["start_symbol_index"], pdu["start_symbol_index"] + pdu["nof_symbols"])
                 if not (dmrs >> l) & 1]
    qm = pdu["modulation"]
    tbs = len(tb) * 8
    p = osch.plan(tbs, pdu["base_graph"], pdu["rv"], qm, nref(tbs, pdu["base_graph"], pdu.get("tbs_lbrm_bytes", 0)),
                  1, M * len(data_syms))
    cw = ref_pdsch_encode(np.asarray(tb, np.uint8), p)
    scr = cw ^ ref_prbs((pdu["rnti"] << 15) + pdu["n_id"], cw.size)
    x = ref_modulate(np.packbits(scr), cw.size // qm, qm).reshape(len(data_syms), M)
    y = (np.fft.fft(x.astype(np.complex128), axis=1) / np.sqrt(M)).astype(np.complex64)
    z = np.zeros((P, 14, nsubc), np.complex64)
    k0 = 12 * crb0
    for i, l in enumerate(data_syms):
        z[:, l, k0:k0 + M] = channel[:, None] * y[i][None, :]
    amp = np.float32(dmrs_scaling(2))
    r = ref_low_papr(M // 2, pdu.get("n_rs_id", 0) % 30, 0)
    for l in range(14):
        if (dmrs >> l) & 1:
            z[:, l, k0:k0 + M:2] = channel[:, None] * (amp * r)[None, :]
    if snr_db is not None:
        occ = np.abs(z) > 0
        pw = float(np.mean(np.abs(z[occ]) ** 2))
        rng = np.random.default_rng(seed)
        sigma = np.sqrt(pw / 10 ** (snr_db / 10) / 2)
        z = z + sigma * (rng.normal(size=z.shape) + 1j * rng.normal(size=z.shape))
    g = (to_bf16(z.real.astype(np.float32)).astype(np.uint32) | (to_bf16(z.imag.astype(np.float32)).astype(np.uint32) << 16))
    return np.ascontiguousarray(g), p


if REF is not None and hasattr(REF, "srs_ref_ulsch_demultiplex"):
    REF.srs_ref_ulsch_demultiplex.restype = _c.c_int
    REF.srs_ref_ulsch_demultiplex.argtypes = ([_c.c_int] + [_c.c_uint] * 5 + [_c.c_int] + [_c.c_uint] * 7
                                              + [_c.c_void_p, _c.c_uint] + [_c.c_void_p] * 4)


def ref_ulsch_demultiplex(llrs, qm, nof_layers, nof_prb, start_symbol, nof_symbols, nof_harq_ack_rvd, dmrs_type2,
                          dmrs_mask, nof_cdm_groups_without_data, nof_harq_ack_bits, nof_enc_harq_ack_bits,
                          nof_csi_part1_bits, nof_enc_csi_part1_bits, c_init):
    """The reference ulsch_demultiplex_impl over one codeword: (UL-SCH, HARQ-ACK, CSI part 1) int8 streams."""
    x = np.ascontiguousarray(llrs, np.int8)
    sch, ack, csi1 = (np.zeros(x.size, np.int8) for _ in range(3))
    counts = np.zeros(3, np.uint32)
    r = REF.srs_ref_ulsch_demultiplex(qm, nof_layers, nof_prb, start_symbol, nof_symbols, nof_harq_ack_rvd,
                                      int(dmrs_type2), dmrs_mask, nof_cdm_groups_without_data, nof_harq_ack_bits,
                                      nof_enc_harq_ack_bits, nof_csi_part1_bits, nof_enc_csi_part1_bits, c_init,
                                      _ptr(x), x.size, _ptr(sch), _ptr(ack), _ptr(csi1), _ptr(counts))
    if r != 0:
        raise RuntimeError("reference demultiplexer did not end every stream")
    return sch[:counts[0]], ack[:counts[1]], csi1[:counts[2]]


if REF is not None and hasattr(REF, "srs_ref_ulsch_demultiplex2"):
    REF.srs_ref_ulsch_demultiplex2.restype = _c.c_int
    REF.srs_ref_ulsch_demultiplex2.argtypes = ([_c.c_int] + [_c.c_uint] * 5 + [_c.c_int] + [_c.c_uint] * 9
                                               + [_c.c_void_p, _c.c_uint] + [_c.c_void_p] * 5)


def ref_ulsch_demultiplex2(llrs, qm, nof_layers, nof_prb, start_symbol, nof_symbols, nof_harq_ack_rvd, dmrs_type2,
                           dmrs_mask, nof_cdm_groups_without_data, nof_harq_ack_bits, nof_enc_harq_ack_bits,
                           nof_csi_part1_bits, nof_enc_csi_part1_bits, nof_csi_part2_bits, nof_enc_csi_part2_bits,
                           c_init):
    """The reference ulsch_demultiplex_impl with CSI part 2 configured when the CSI part 1 stream ends (as its PUSCH
    processor does): (UL-SCH, HARQ-ACK, CSI part 1, CSI part 2) int8 streams."""
    x = np.ascontiguousarray(llrs, np.int8)
    sch, ack, csi1, csi2 = (np.zeros(x.size, np.int8) for _ in range(4))
    counts = np.zeros(4, np.uint32)
    r = REF.srs_ref_ulsch_demultiplex2(qm, nof_layers, nof_prb, start_symbol, nof_symbols, nof_harq_ack_rvd,
                                       int(dmrs_type2), dmrs_mask, nof_cdm_groups_without_data, nof_harq_ack_bits,
                                       nof_enc_harq_ack_bits, nof_csi_part1_bits, nof_enc_csi_part1_bits,
                                       nof_csi_part2_bits, nof_enc_csi_part2_bits, c_init, _ptr(x), x.size, _ptr(sch),
                                       _ptr(ack), _ptr(csi1), _ptr(csi2), _ptr(counts))
    if r != 0:
        raise RuntimeError("reference demultiplexer did not end every stream")
    return sch[:counts[0]], ack[:counts[1]], csi1[:counts[2]], csi2[:counts[3]]


def part2_words(entries):
    """A uci_part2_size_description [([(offset, width), ...], [sizes]), ...] as the glue's flat uint16 words."""
    w = [len(entries)]
    for params, sizes in entries:
        x = [len(params)] + [0] * 4 + [len(sizes)] + [0] * 16
        for q, (off, wd) in enumerate(params):
            x[1 + 2 * q], x[2 + 2 * q] = off, wd
        x[6:6 + len(sizes)] = sizes
        w += x
    return np.ascontiguousarray(w, np.uint16)


def ref_uci_part2_get_size(part1, entries):
    """The reference uci_part2_get_size."""
    b = np.ascontiguousarray(part1, np.uint8)
    w = part2_words(entries)
    f = REF.srs_ref_uci_part2_get_size
    f.restype = _c.c_uint
    f.argtypes = [_c.c_void_p, _c.c_uint, _c.c_void_p]
    return int(f(_ptr(b), b.size, _ptr(w)))


if REF is not None and hasattr(REF, "srs_ref_uci_decode"):
    REF.srs_ref_uci_decode.restype = _c.c_int
    REF.srs_ref_uci_decode.argtypes = [_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_int, _c.c_void_p]
    REF.srs_ref_short_block_encode.restype = None
    REF.srs_ref_short_block_encode.argtypes = [_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_int, _c.c_void_p]


def ref_uci_decode(llrs, K, qm):
    """The reference uci_decoder_impl: (message bits, uci_status)."""
    x = np.ascontiguousarray(llrs, np.int8)
    msg = np.zeros(K, np.uint8)
    st = REF.srs_ref_uci_decode(_ptr(x), x.size, K, qm, _ptr(msg))
    return msg, st


def _uci_crc(bits, L):
    poly = 0x21 if L == 6 else 0x621
    crc = 0
    for b in bits:
        fb = ((crc >> (L - 1)) & 1) ^ int(b)
        crc = (crc << 1) & ((1 << L) - 1)
        if fb:
            crc ^= poly
    return [(crc >> (L - 1 - i)) & 1 for i in range(L)]


def uci_encode(msg, E, qm):
    """UE-side UCI encoding (TS 38.212 6.3.1.2-6.3.1.4) for test inputs: the reference's short_block_encoder_impl for
    <= 11 bits (placeholders 255 / 254 kept), else code block segmentation with filler bits, CRC6 / CRC11 and the
    reference's polar chain (nMax 10, channel interleaver) per codeblock."""
    msg = np.asarray(msg, np.uint8)
    A = msg.size
    out = np.zeros(E, np.uint8)
    if A <= 11:
        REF.srs_ref_short_block_encode(_ptr(np.ascontiguousarray(msg)), A, E, qm, _ptr(out))
        return out
    from . import ref_polar_encode_chain

    C = 2 if (A >= 360 and E >= 1088) or A >= 1013 else 1
    L = 6 if A < 20 else 11
    F = (-A) % C
    a = np.concatenate([np.zeros(F, np.uint8), msg])
    per = a.size // C
    pos = 0
    for r in range(C):
        cb = a[r * per:(r + 1) * per]
        cb = np.concatenate([cb, np.array(_uci_crc(cb, L), np.uint8)])
        e = E // C
        out[pos:pos + e] = ref_polar_encode_chain(cb, e, 10, ibil=True)
        pos += e
    return out


if REF is not None and hasattr(REF, "srs_ref_ulsch_information"):
    REF.srs_ref_ulsch_information.restype = None
    REF.srs_ref_ulsch_information.argtypes = ([_c.c_uint, _c.c_int, _c.c_float] + [_c.c_uint] * 3 + [_c.c_float] * 4
                                              + [_c.c_uint] * 3 + [_c.c_int] + [_c.c_uint] * 3
                                              + [_c.c_int, _c.c_void_p])

ULSCH_INFO_FIELDS = ["nof_ul_sch_bits", "nof_harq_ack_bits", "nof_harq_ack_rvd", "nof_csi_part1_bits",
                     "nof_csi_part2_bits", "nof_harq_ack_re", "nof_csi_part1_re", "nof_csi_part2_re",
                     "nof_dc_overlap_bits", "sch_tb_crc_size", "sch_base_graph", "sch_nof_cb", "sch_lifting_size",
                     "sch_nof_bits_per_cb", "sch_nof_filler_bits_per_cb"]


def ref_ulsch_information(pdu, tbs, nof_csi_part2=0):
    """The reference get_ulsch_information for a PUSCH pdu dict (type-1 DM-RS, no DC), with nof_csi_part2 CSI part 2
    payload bits."""
    out = np.zeros(15, np.uint32)
    REF.srs_ref_ulsch_information(tbs, pdu["modulation"], float(pdu["target_code_rate"]), pdu.get("nof_harq_ack", 0),
                                  pdu.get("nof_csi_part1", 0), nof_csi_part2, float(pdu.get("alpha_scaling", 1.0)),
                                  float(pdu.get("beta_offset_harq_ack", 5.0)),
                                  float(pdu.get("beta_offset_csi_part1", 5.0)),
                                  float(pdu.get("beta_offset_csi_part2", 5.0)), pdu["rb_count"],
                                  pdu["start_symbol_index"], pdu["nof_symbols"], 0, pdu["dmrs_symbol_mask"],
                                  pdu["nof_cdm_groups_without_data"], pdu["nof_tx_layers"], 0, _ptr(out))
    return dict(zip(ULSCH_INFO_FIELDS, out.tolist()))


def ue_multiplex_uci(sch_cw, pdu, info, nof_cw_bits, ack_bits, csi1_bits, csi2_bits=()):
    """UE-side UL-SCH / UCI multiplexing for test inputs (TS 38.212 6.2.7 + 6.3.2.1): the UCI encoded with
    uci_encode, the RE placement read off the reference's own demultiplexer (three probe passes with the RE index
    coded in the LLR values), the ACK of <= 2 bits puncturing the UL-SCH, and the scrambler's placeholder rules
    (x -> 1, y -> the previous scrambled bit) folded in by pre-XOR-ing the Gold sequence, so that a modulator that
    scrambles every bit produces the UE's symbols.  Returns the codeword to hand to the modulator."""
    from . import ref_prbs

    qm, L = pdu["modulation"], pdu["nof_tx_layers"]
    bpre = qm * L
    nre = nof_cw_bits // bpre
    K_ack, K_csi1, K_csi2 = len(ack_bits), len(csi1_bits), len(csi2_bits)
    enc_ack = uci_encode(ack_bits, info["nof_harq_ack_bits"], qm) if K_ack else np.zeros(0, np.uint8)
    enc_csi1 = uci_encode(csi1_bits, info["nof_csi_part1_bits"], qm) if K_csi1 else np.zeros(0, np.uint8)
    enc_csi2 = (uci_encode(np.asarray(csi2_bits, np.uint8), info["nof_csi_part2_bits"], qm) if K_csi2
                else np.zeros(0, np.uint8))
    c_init = (pdu["rnti"] << 15) + pdu["n_id"]
    args = (qm, L, pdu["rb_count"], pdu["start_symbol_index"], pdu["nof_symbols"], info["nof_harq_ack_rvd"], False,
            pdu["dmrs_symbol_mask"], pdu["nof_cdm_groups_without_data"], K_ack, info["nof_harq_ack_bits"], K_csi1,
            info["nof_csi_part1_bits"])
    src = [None, None, None, None]
    for k in range(3):
        code = (((np.arange(nre) >> (7 * k)) & 0x7F) + 1).astype(np.int8)
        if K_csi2:
            streams = ref_ulsch_demultiplex2(np.repeat(code, bpre), *args, K_csi2, info["nof_csi_part2_bits"], 0)
        else:
            streams = ref_ulsch_demultiplex(np.repeat(code, bpre), *args, 0) + (np.zeros(0, np.int8),)
        for i, st in enumerate(streams):
            a = np.abs(st.astype(np.int64)) - 1  # -1: a zeroed LLR (a RE a 1/2-bit HARQ-ACK punctures)
            v = np.where(a < 0, -(1 << 40), a << (7 * k))
            src[i] = v if src[i] is None else src[i] + v
    out = np.zeros(nof_cw_bits, np.uint8)
    pos = np.arange(bpre)
    # UL-SCH REs (the zero LLRs of the demultiplexer's SCH stream are the REs an ACK of <= 2 bits punctures)
    sch_src = src[0].reshape(-1, bpre)[:, 0]
    for j, r in enumerate(sch_src if len(sch_cw) else ()):  # UCI only: REs no UCI uses carry nothing (zero bits)
        if r >= 0:
            out[r * bpre + pos] = sch_cw[j * bpre + pos]
    # CSI part 2 first: where a 1/2-bit HARQ-ACK shares a reserved RE with it, the HARQ-ACK is what is sent
    for s_i, enc in ((3, enc_csi2), (1, enc_ack), (2, enc_csi1)):
        if enc.size:
            for j, r in enumerate(src[s_i].reshape(-1, bpre)[:, 0]):
                if r >= 0:
                    out[r * bpre + pos] = enc[j * bpre + pos]
    # scrambling with placeholders (TS 38.211 6.3.1.1), expressed as the bits a plain scrambler receives
    c = ref_prbs(c_init, nof_cw_bits)
    scr = np.zeros(nof_cw_bits, np.uint8)
    for i in range(nof_cw_bits):
        b = out[i]
        if b == 255:
            scr[i] = 1
        elif b == 254:
            scr[i] = scr[i - 1]
        else:
            scr[i] = b ^ c[i]
    return scr ^ c

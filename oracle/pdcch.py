"""CPU restatement of srsRAN's PDCCH processor (TEST INFRASTRUCTURE ONLY: tests/ and __graft_entry__.smoke() use it
as the checker of the MI355X PDCCH processor; the product never imports it).

Follows, function by function:
  crbs            lib/ran/pdcch/cce_to_prb_mapping.cpp:30-199 (pdcch_processor_impl.cpp:44-77 picks the mapping)
  encode          lib/phy/upper/channel_processors/pdcch/pdcch_encoder_impl.cpp:33-98 (CRC24C over 24 ones + payload,
                  RNTI over the last 16 parity bits, DCI interleaver, polar chain with nMax = 9)
  process         pdcch_processor_impl.cpp:79-130, pdcch_modulator_impl.cpp:32-106 (scrambling, QPSK, scaling when
                  the amplitude is a normal number, mapping k mod 4 != 1), dmrs_pdcch_processor_impl.cpp:32-130
                  (c_init, M_SQRT1_2 x amplitude, k = 4 n + 1 from the reference point)
Parity pinned by tests/test_oracle_vs_ref.py against the compiled reference (oracle/ref_wrapper_pdcch.cpp).
Grids: uint32 [port][14][nof_subc], cbf16 (real in the low half).
"""
import numpy as np

from . import crc_bits, polar_encode_chain, polar_interleave, prbs
from .pdsch_mod import cmul_simd, to_bf16

NSYMB = 14


def _freq_groups(pdu):
    fr = bytes(pdu.coreset.frequency_resources)
    return [i for i in range(45) if (fr[i // 8] >> (i % 8)) & 1]


def _regs_interleaved(n_rb, n_symb, L, R, n_shift, al, cce):
    n_reg = n_rb * n_symb
    assert n_reg > 0 and n_reg % (L * R) == 0 and L % n_symb == 0, "invalid CORESET configuration"
    C = n_reg // (L * R)
    out = []
    for x in range(cce * (6 // L), (cce + al) * (6 // L)):
        f = ((x % R) * C + x // R + n_shift) % (n_reg // L)
        out += range(f * L, (f + 1) * L)
    return sorted(out)


def _prbs_other(bwp_start, groups, n_symb, regs):
    out, count, reg = [], 0, 0
    for g in groups:
        for prb in range(g * 6 + bwp_start, g * 6 + bwp_start + 6):
            if reg == regs[count]:
                out.append(prb)
                count += n_symb
                if count == len(regs):
                    return out
            reg += n_symb
    return out


def crbs(pdu):
    """The DCI's CRBs in the mapping functions' order (cce_to_prb_mapping_*)."""
    c, d = pdu.coreset, pdu.dci
    al, cce = d.aggregation_level, d.cce_index
    if c.cce_to_reg_mapping == 0:
        regs = _regs_interleaved(c.bwp_size_rb, c.duration, 6, 2, c.shift_index, al, cce)
        return [regs[i] // c.duration + c.bwp_start_rb for i in range(0, len(regs), c.duration)]
    groups = _freq_groups(pdu)
    if c.cce_to_reg_mapping == 1:
        regs = list(range(6 * cce, 6 * (cce + al)))
    else:
        regs = _regs_interleaved(len(groups) * 6, c.duration, c.reg_bundle_size, c.interleaver_size, c.shift_index,
                                 al, cce)
    return _prbs_other(c.bwp_start_rb, groups, c.duration, regs)


def encode(payload, rnti, E):
    """pdcch_encoder_impl::encode: E coded bits (one per byte)."""
    a = np.asarray(payload, np.uint8)
    crc = crc_bits(2, np.concatenate([np.ones(24, np.uint8), a]))  # CRC24C
    parity = np.array([(crc >> (23 - k)) & 1 for k in range(24)], np.uint8)
    parity[8:] ^= np.array([(rnti >> (15 - k)) & 1 for k in range(16)], np.uint8)
    c = np.concatenate([a, parity])
    return polar_encode_chain(polar_interleave(c, 0), E, 9)


def _pack(re, im):
    return to_bf16(re).astype(np.uint32) | (to_bf16(im).astype(np.uint32) << 16)


def process(grid, pdu):
    """pdcch_processor_impl::process onto grid (uint32 [ports][14][nof_subc], modified in place)."""
    c, d = pdu.coreset, pdu.dci
    rbs = sorted(set(crbs(pdu)))  # the rb_mask bitmap
    E = d.aggregation_level * 6 * 9 * 2
    cw = encode(np.frombuffer(bytes(d.payload), np.uint8)[:d.payload_size], d.rnti & 0xFFFF, E)
    c_init = ((d.n_rnti << 16) + d.n_id_pdcch_data) % (1 << 31)
    b = cw ^ prbs(c_init, E)
    s = np.float32(np.sqrt(np.float32(0.5)))
    sym = (np.where(b[0::2] != 0, -s, s) + 1j * np.where(b[1::2] != 0, -s, s)).astype(np.complex64)
    amp = np.float32(10.0) ** (np.float32(d.data_power_offset_dB) / np.float32(20.0))
    if np.isfinite(amp) and amp != 0 and abs(amp) >= np.finfo(np.float32).tiny:
        sym = (sym.real * amp + 1j * (sym.imag * amp)).astype(np.complex64)
    dmrs_amp = np.float32(np.sqrt(0.5) * np.float64(np.float32(10.0) ** (np.float32(d.dmrs_power_offset_dB)
                                                                       / np.float32(20.0))))
    ref = c.bwp_start_rb if c.cce_to_reg_mapping == 0 else 0
    data_k = np.array([k for k in range(12) if k % 4 != 1])
    dmrs_k = np.array([1, 5, 9])
    w = [complex(d.weights[a][0], d.weights[a][1]) for a in range(d.nof_ports)]
    j = 0
    for li in range(c.duration):
        l = c.start_symbol_index + li
        c_dmrs = ((NSYMB * pdu.slot_index + l + 1) * (2 * d.n_id_pdcch_dmrs + 1) * (1 << 17)
                  + 2 * d.n_id_pdcch_dmrs) % (1 << 31)
        seq = prbs(c_dmrs, 2 * 3 * (max(rbs) - ref + 1))
        for rb in rbs:
            x = sym[j:j + 9]
            j += 9
            m = 3 * (rb - ref) + np.arange(3)
            y = (np.where(seq[2 * m] != 0, -dmrs_amp, dmrs_amp)
                 + 1j * np.where(seq[2 * m + 1] != 0, -dmrs_amp, dmrs_amp)).astype(np.complex64)
            for a, wa in enumerate(w):
                re, im = cmul_simd(x, wa)
                grid[a, l, 12 * rb + data_k] = _pack(re, im)
                re, im = cmul_simd(y, wa)
                grid[a, l, 12 * rb + dmrs_k] = _pack(re, im)
    return grid


# ---- the reference itself -------------------------------------------------------------------------------------------
def _ref():
    import ctypes

    from . import REF

    f = REF.srs_ref_pdcch_process
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p, ctypes.c_uint, ctypes.c_char_p,
                  ctypes.c_uint]
    REF.srs_ref_pdcch_prbs.restype = ctypes.c_int
    REF.srs_ref_pdcch_prbs.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    return REF


def ref_process(grid, pdus):
    """The compiled reference pdcch_processor_impl over pdus, in order, onto grid (uint32 [ports][14][nof_subc], in
    place).  Raises ValueError with the reference validator's message for an invalid PDU."""
    import ctypes

    from srsran_project_amd.pdcch import PdcchPdu

    ref = _ref()
    arr = (PdcchPdu * len(pdus))(*pdus)
    g = np.ascontiguousarray(grid)
    msg = ctypes.create_string_buffer(512)
    if ref.srs_ref_pdcch_process(g.ctypes.data, g.shape[0], g.shape[2], ctypes.addressof(arr), len(pdus), msg,
                                 512) != 0:
        raise ValueError(msg.value.decode())
    grid[...] = g
    return grid


def ref_crbs(pdu):
    import ctypes

    out = np.zeros(96, np.uint16)
    n = _ref().srs_ref_pdcch_prbs(ctypes.addressof(pdu), out.ctypes.data)
    return [int(x) for x in out[:n]]

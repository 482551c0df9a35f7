"""CPU oracle of the PDSCH modulator and the PDSCH DM-RS processor -- TEST INFRASTRUCTURE ONLY.

Restates, in numpy (pinned against the reference's own classes compiled into
oracle/_ref by oracle/Makefile, tests/test_oracle_vs_ref.py):
  pdsch_modulate()  pdsch_modulator_impl.cpp:28-115 -- scrambling (c_init = rnti<<15 + q<<14 + n_id),
                    modulation to ci8 + scaling (modulation_mapper_lut_impl.cpp:37-67, 145-149),
                    RE mapping with layer mapping and precoding (resource_grid_mapper_impl.cpp:341-460,
                    channel_precoder_avx2.cpp:55-58, 60-75, 214-330).
  dmrs_pdsch_map()  dmrs_pdsch_processor_impl.cpp:57-234 with dmrs_helper.cpp:58-110 and
                    resource_grid_mapper_impl.cpp:47-131 (per-PRG precoding, apply_precoding_port).
Precoding arithmetic is the reference's SIMD one: per layer a complex multiply
re = fma(x.re, w.re, -(x.im * w.im)), im = fma(x.im, w.re, x.re * w.im)
(_mm256_fmaddsub_ps), layer contributions summed left to right, then
round-half-even to bf16 (ps_to_cbf16).  FMA is emulated in float64 (the
float32 x float32 product is exact there).
"""
import ctypes

import numpy as np

from . import REF, _ptr, prbs

NRE = 12
MAX_RB = 275
NSYMB = 14


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def _fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def cmul_simd(x, w):
    """Complex float32 product as _mm256_fmaddsub_ps(x, w.re, swap(x) * w.im)."""
    xr, xi = _f32(x.real), _f32(x.imag)
    wr, wi = np.float32(w.real), np.float32(w.imag)
    re = _fma(xr, np.full_like(xr, wr), -(xi * wi))
    im = _fma(xi, np.full_like(xi, wr), xr * wi)
    return re, im


def to_bf16(x):
    """Round-half-even float32 -> bf16 bits (uint16), as ps_to_cbf16 / to_bf16."""
    u = _f32(x).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return (u & 0xFFFF).astype(np.uint16)


def ci8_table(qm):
    """Unscaled integer constellation (modulation_mapper_lut_impl.cpp:41-58) and its scaling."""
    if qm in (0, 1):
        return None, np.float32(np.sqrt(0.5))
    L = 1 << qm
    tab = np.zeros((L, 2), np.float32)
    for i in range(L):
        off, re, im = -1.0, 0.0, 0.0
        for j in range(qm // 2):
            re += off
            im += off
            off *= 2
            re *= 1 if (i >> (2 * j + 1)) & 1 else -1
            im *= 1 if (i >> (2 * j)) & 1 else -1
        tab[i] = (re, im)
    avg = np.float32(np.sum(tab.astype(np.float64) ** 2) / L)
    return tab, np.float32(np.sqrt(np.float32(1) / avg))


def modulate_ci8(bits, qm):
    """bits: one per byte. Returns complex64 integer symbols and the scaling."""
    tab, scale = ci8_table(qm)
    bits = np.asarray(bits, np.uint8)
    if qm == 1:
        v = 1.0 - 2.0 * bits
        return (v + 1j * v).astype(np.complex64), scale
    if qm == 0:
        v = 1.0 - 2.0 * bits
        odd = (np.arange(bits.size) & 1) == 1
        re = np.where(odd, -v, v)
        return (re + 1j * v).astype(np.complex64), scale
    b = bits.reshape(-1, qm).astype(np.int64)
    idx = np.zeros(b.shape[0], np.int64)
    for k in range(qm):
        idx = (idx << 1) | b[:, k]
    return (tab[idx, 0] + 1j * tab[idx, 1]).astype(np.complex64), scale


def dmrs_prb_mask(dmrs_type2, nof_cdm_groups_without_data):
    """get_dmrs_prb_mask (dmrs_mapping.h:76-91) as a 12-bit mask (bit k = subcarrier k)."""
    m = 0
    for k in range(NRE):
        if not dmrs_type2:
            if (k % 2) < nof_cdm_groups_without_data:
                m |= 1 << k
        elif (k % 6) < 2 * nof_cdm_groups_without_data:
            m |= 1 << k
    return m


def data_re_mask(nsubc, crbs, start_symbol, nof_symbols, reserved):
    """bool [14][nsubc]: REs carrying PDSCH data. crbs: allocated CRB indices; reserved: list of
    (crb bool[MAX_RB], re_mask 12 bits, symbols 14 bits) (re_pattern_list::get_exclusion_mask)."""
    base = np.zeros(nsubc, bool)
    for c in crbs:
        base[c * NRE:(c + 1) * NRE] = True
    out = np.zeros((NSYMB, nsubc), bool)
    for l in range(start_symbol, start_symbol + nof_symbols):
        m = base.copy()
        for crb_mask, re_mask, symbols in reserved:
            if not (symbols >> l) & 1:
                continue
            for c in np.nonzero(crb_mask)[0]:
                for k in range(NRE):
                    if (re_mask >> k) & 1 and c * NRE + k < nsubc:
                        m[c * NRE + k] = False
        out[l] = m
    return out


def precode(layers, weights):
    """layers: complex64 [L][n]; weights complex [L][P] (already scaled). Returns bf16 bits [P][n][2]."""
    L, n = layers.shape
    P = weights.shape[1]
    out = np.zeros((P, n, 2), np.uint16)
    for p in range(P):
        re, im = cmul_simd(layers[0], weights[0, p])
        for v in range(1, L):
            r, i = cmul_simd(layers[v], weights[v, p])
            re, im = _f32(re + r), _f32(im + i)
        out[p, :, 0] = to_bf16(re)
        out[p, :, 1] = to_bf16(im)
    return out


def pdsch_modulate(grid, codeword_bits, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                   nof_cdm_groups_without_data, reserved, weights, scaling=1.0, bwp=(0, MAX_RB)):
    """grid: uint16 [ports][14][nsubc][2] (bf16 re, im), modified in place. codeword_bits one per byte.
    weights complex [layers][ports]."""
    weights = np.asarray(weights, np.complex64)
    L = weights.shape[0]
    bits = np.asarray(codeword_bits, np.uint8)
    c_init = (rnti << 15) + n_id
    scr = bits ^ prbs(c_init, bits.size)
    sym, mod_scale = modulate_ci8(scr, qm)
    s = np.float32(mod_scale)
    if np.isfinite(scaling) and scaling != 0 and abs(scaling) >= np.finfo(np.float32).tiny:
        s = np.float32(s * np.float32(scaling))
    w = (weights.real.astype(np.float32) * s) + 1j * (weights.imag.astype(np.float32) * s)
    dmrs = dmrs_prb_mask(dmrs_type2, nof_cdm_groups_without_data)
    bwp_crbs = np.zeros(MAX_RB, bool)
    bwp_crbs[bwp[0]:bwp[0] + bwp[1]] = True
    res = list(reserved) + [(bwp_crbs, dmrs, dmrs_symb_mask)]
    mask = data_re_mask(grid.shape[2], crbs, start_symbol, nof_symbols, res)
    ls, ks = np.nonzero(mask)  # row-major: symbol then subcarrier ascending = mapping order
    nre = ls.size
    assert sym.size == nre * L, "codeword does not fill the allocation"
    layers = sym.reshape(nre, L).T
    out = precode(layers, w)
    for p in range(weights.shape[1]):
        grid[p, ls, ks] = out[p]
    return grid


def dmrs_params(dmrs_type2, port):
    """(cdm group, w_f odd sign, w_t second-symbol sign) of a DM-RS port (dmrs_helper.cpp:34-56)."""
    if not dmrs_type2:
        return (port // 2) % 2, (-1 if port % 2 else 1), (-1 if port >= 4 else 1)
    return (port // 2) % 3, (-1 if port % 2 else 1), (-1 if port >= 6 else 1)


def dmrs_pdsch_map(grid, slot_index, reference_point_k_rb, dmrs_type2, scrambling_id, n_scid, amplitude,
                   symbols_mask, crbs, weights, prg_size=MAX_RB):
    """grid uint16 [ports][14][nsubc][2] modified in place; weights complex [prg][layers][ports]."""
    weights = np.asarray(weights, np.complex64)
    nprg, L, P = weights.shape
    crbs = np.sort(np.asarray(crbs))
    nd = 4 if dmrs_type2 else 6
    amp = np.float32(np.sqrt(0.5) * np.float64(np.float32(amplitude)))  # M_SQRT1_2 (double) * float
    for l in range(NSYMB):
        if not (symbols_mask >> l) & 1:
            continue
        c_init = ((NSYMB * slot_index + l + 1) * (2 * scrambling_id + 1) * (1 << 17) + (2 * scrambling_id + n_scid)) \
            % (1 << 31)
        pos = ((crbs[:, None] - reference_point_k_rb) * nd + np.arange(nd)[None, :]).reshape(-1)
        c = prbs(c_init, 2 * int(pos.max()) + 2)
        base = (np.where(c[2 * pos] == 0, amp, -amp) + 1j * np.where(c[2 * pos + 1] == 0, amp, -amp)).astype(
            np.complex64)
        lprime = 1 if l > 0 and (symbols_mask >> (l - 1)) & 1 else 0
        prg = (np.repeat(crbs, nd)) // prg_size
        for g in range((L + 1) // 2):
            ports = [p for p in range(2 * g, min(2 * g + 2, L))]
            seqs = []
            for p in ports:
                _, wf, wt = dmrs_params(dmrs_type2, p)
                s = base.copy()
                if lprime == 1 and wt < 0:
                    s = -s
                if wf < 0:
                    s[1::2] = -s[1::2]
                seqs.append(s)
            if not dmrs_type2:
                off = np.tile(np.arange(0, NRE, 2) + g, crbs.size)
            else:
                off = np.tile(np.array([0, 1, 6, 7]) + 2 * g, crbs.size)
            sc = np.repeat(crbs, nd) * NRE + off
            for a in range(P):
                re = np.zeros(sc.size, np.float32)
                im = np.zeros(sc.size, np.float32)
                for i, p in enumerate(ports):
                    r = np.zeros(sc.size, np.float32)
                    q = np.zeros(sc.size, np.float32)
                    for gi in np.unique(prg):
                        sel = prg == gi
                        rr, qq = cmul_simd(seqs[i][sel], weights[gi, p, a])
                        r[sel], q[sel] = rr, qq
                    if i == 0:
                        re, im = r, q
                    else:
                        re, im = _f32(re + r), _f32(im + q)
                grid[a, l, sc, 0] = to_bf16(re)
                grid[a, l, sc, 1] = to_bf16(im)
    return grid


# ---- the reference itself -------------------------------------------------------------------------------------------
_c = ctypes
if REF is not None and hasattr(REF, "srs_ref_pdsch_modulate"):
    REF.srs_ref_pdsch_modulate.restype = _c.c_int
    REF.srs_ref_pdsch_modulate.argtypes = ([_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_void_p] + [_c.c_uint] * 4
                                           + [_c.c_int, _c.c_void_p, _c.c_uint, _c.c_uint, _c.c_uint, _c.c_int,
                                              _c.c_uint, _c.c_uint, _c.c_float, _c.c_void_p, _c.c_void_p,
                                              _c.c_void_p, _c.c_uint, _c.c_uint, _c.c_uint, _c.c_void_p, _c.c_int])
    REF.srs_ref_dmrs_pdsch_map.restype = _c.c_int
    REF.srs_ref_dmrs_pdsch_map.argtypes = ([_c.c_void_p] + [_c.c_uint] * 5 + [_c.c_int, _c.c_uint, _c.c_int,
                                                                              _c.c_float, _c.c_uint, _c.c_void_p]
                                           + [_c.c_uint] * 4 + [_c.c_void_p, _c.c_int])

PRECODER = {"generic": 0, "avx2": 1, "avx512": 2}


def ref_pdsch_modulate(grid, codeword_bits, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask,
                       dmrs_type2, nof_cdm_groups_without_data, reserved, weights, scaling=1.0, bwp=(0, MAX_RB),
                       precoder="avx2"):
    """Reference pdsch_modulator_impl (same arguments as pdsch_modulate; crbs must lie in the BWP)."""
    weights = np.asarray(weights, np.complex64)
    L, P = weights.shape
    g = np.ascontiguousarray(grid)
    bits = np.asarray(codeword_bits, np.uint8)
    packed = np.packbits(bits)
    vrbs = np.zeros(bwp[1], np.uint8)
    vrbs[np.asarray(crbs) - bwp[0]] = 1
    nres = len(reserved)
    rc = np.zeros((max(nres, 1), MAX_RB), np.uint8)
    rre = np.zeros(max(nres, 1), np.uint16)
    rsy = np.zeros(max(nres, 1), np.uint16)
    for i, (cm, rm, sm) in enumerate(reserved):
        rc[i] = np.asarray(cm, bool)
        rre[i], rsy[i] = rm, sm
    w = np.ascontiguousarray(weights.reshape(1, L, P).astype(np.complex64))
    REF.srs_ref_pdsch_modulate(_ptr(g), g.shape[0], g.shape[2], _ptr(packed), bits.size, rnti, bwp[0], bwp[1], qm,
                               _ptr(vrbs), start_symbol, nof_symbols, dmrs_symb_mask, int(dmrs_type2),
                               nof_cdm_groups_without_data, n_id, float(scaling), _ptr(rc), _ptr(rre), _ptr(rsy), nres,
                               L, P, _ptr(w), PRECODER[precoder])
    grid[...] = g
    return grid


def ref_dmrs_pdsch_map(grid, slot_index, reference_point_k_rb, dmrs_type2, scrambling_id, n_scid, amplitude,
                       symbols_mask, crbs, weights, prg_size=MAX_RB, numerology=1, precoder="avx2"):
    weights = np.ascontiguousarray(np.asarray(weights, np.complex64))
    nprg, L, P = weights.shape
    g = np.ascontiguousarray(grid)
    cm = np.zeros(MAX_RB, np.uint8)
    cm[np.asarray(crbs)] = 1
    REF.srs_ref_dmrs_pdsch_map(_ptr(g), g.shape[0], g.shape[2], numerology, slot_index, reference_point_k_rb,
                               int(dmrs_type2), scrambling_id, int(n_scid), float(amplitude), symbols_mask, _ptr(cm),
                               L, P, nprg, prg_size, _ptr(weights), PRECODER[precoder])
    grid[...] = g
    return grid

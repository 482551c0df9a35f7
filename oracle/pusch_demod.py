"""CPU oracle of the PUSCH demodulator -- TEST INFRASTRUCTURE ONLY.

Restatement: the data-RE selection of pusch_demodulator_impl.cpp:218-262
(rb_mask x 12 REs, DM-RS CDM groups without data removed on DM-RS symbols,
dmrs_mapping.h:76-91), the channel equalizer (oracle/equalizer.py), the soft
demapper (oracle.demodulate, srs_oracle_mod.c) called once per OFDM symbol as
pusch_demodulator_impl.cpp:336-400 does when the codeword buffer is the PUSCH
decoder's (pusch_decoder_impl.cpp:140-157 hands out the whole requested block),
and revert_scrambling (pusch_demodulator_impl.cpp:36-190: LLR negated where
c(n) = 1, c_init = rnti * 2^15 + n_id, one sequence over the codeword).

Pinned: `ref_pusch_demodulate` runs the reference's own pusch_demodulator_impl
(oracle/ref_wrapper_pusch.cpp) on the same inputs; tests/test_oracle_vs_ref.py
checks the restatement against it and tests/test_pusch_demod_gpu.py checks the
GPU demodulator against both.
"""
import ctypes as _c

import numpy as np

from . import REF, _ptr, demodulate, prbs
from .equalizer import equalize, equalize_mimo
from .pdsch_mod import dmrs_prb_mask


def data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2, nof_cdm_groups_without_data):
    base = np.zeros(nsubc, bool)
    for c in crbs:
        base[c * 12:(c + 1) * 12] = True
    dm = dmrs_prb_mask(dmrs_type2, nof_cdm_groups_without_data)
    excl = np.array([(dm >> (k % 12)) & 1 for k in range(nsubc)], bool)
    out = np.zeros((14, nsubc), bool)
    for l in range(start_symbol, start_symbol + nof_symbols):
        out[l] = base & ~excl if (dmrs_symb_mask >> l) & 1 else base
    return out


def pusch_demodulate(grid, estimates, noise_vars, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask,
                     dmrs_type2, nof_cdm_groups_without_data, nof_layers, mmse=False):
    """grid uint32 [P][14][nsubc]; estimates uint32 [P][L][14][nsubc]; noise_vars [P].
    Returns int8 LLRs (codeword order, descrambled)."""
    P, _, nsubc = grid.shape
    mask = data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                        nof_cdm_groups_without_data)
    ls, ks = np.nonzero(mask)
    sym = np.ascontiguousarray(grid[:, ls, ks]).view(np.uint16)                       # [P][2*nre]
    est = np.ascontiguousarray(np.transpose(estimates[:, :, ls, ks], (1, 0, 2))).view(np.uint16)  # [L][P][2*nre]
    if nof_layers >= 3 or (mmse and nof_layers == 2):
        # the L-layer solves the open reference does not implement (parity unpinned, fp64)
        eq, nv, _ = equalize_mimo(sym, est, noise_vars, 1.0, nof_layers, "mmse" if mmse else "zf")
    else:
        eq, nv = equalize(sym, est, noise_vars, 1.0, nof_layers)  # MMSE with one layer is ZF (channel_equalizer_generic_impl.cpp:348)
    eq = eq.reshape(-1).astype(np.complex64)
    nv = nv.reshape(-1).astype(np.float32)
    # one demapper call per OFDM symbol (its SIMD blocks end at the symbol's last RE)
    counts = mask.sum(axis=1) * nof_layers
    parts, s0 = [], 0
    for l in range(14):
        n = int(counts[l])
        if n:
            parts.append(demodulate(eq[s0:s0 + n], nv[s0:s0 + n], qm))
            s0 += n
    llr = np.concatenate(parts) if parts else np.zeros(0, np.int8)
    c = prbs(rnti * (1 << 15) + n_id, llr.size)
    return np.where(c == 1, -llr.astype(np.int16), llr.astype(np.int16)).astype(np.int8)


if REF is not None and hasattr(REF, "srs_ref_pusch_demodulate"):
    REF.srs_ref_pusch_demodulate.restype = _c.c_int
    REF.srs_ref_pusch_demodulate.argtypes = ([_c.c_void_p, _c.c_uint, _c.c_uint, _c.c_void_p, _c.c_uint, _c.c_void_p,
                                              _c.c_uint, _c.c_uint, _c.c_int, _c.c_void_p, _c.c_uint, _c.c_uint,
                                              _c.c_uint, _c.c_int, _c.c_uint, _c.c_int, _c.c_int, _c.c_int,
                                              _c.c_void_p, _c.c_uint, _c.c_void_p])


def ref_pusch_demodulate(grid, estimates, noise_vars, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask,
                         dmrs_type2, nof_cdm_groups_without_data, nof_layers, mmse=False, transform_precoding=False,
                         post_eq_sinr=False, with_stats=False):
    """The reference's pusch_demodulator_impl::demodulate on the same inputs. Returns int8 LLRs
    (and, with_stats, (llrs, nof_blocks, per-symbol SINR dB [14], final SINR dB))."""
    if REF is None:
        raise RuntimeError("oracle/_ref not built")
    P, _, nsubc = grid.shape
    L = nof_layers
    mask = data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                        nof_cdm_groups_without_data)
    nllr = int(mask.sum()) * L * max(1, qm)
    g = np.ascontiguousarray(grid, np.uint32)
    e = np.ascontiguousarray(estimates, np.uint32)
    nv = np.ascontiguousarray(noise_vars, np.float32)
    cr = np.zeros(nsubc // 12, np.uint8)
    cr[list(crbs)] = 1
    out = np.zeros(nllr, np.int8)
    sinr = np.zeros(15, np.float32)
    r = REF.srs_ref_pusch_demodulate(_ptr(g), P, nsubc, _ptr(e), L, _ptr(nv), rnti, n_id, qm, _ptr(cr), start_symbol,
                                     nof_symbols, dmrs_symb_mask, int(dmrs_type2), nof_cdm_groups_without_data,
                                     int(mmse), int(transform_precoding), int(post_eq_sinr), _ptr(out), nllr,
                                     _ptr(sinr))
    if r < 0:
        raise RuntimeError("reference PUSCH demodulator failed")
    if with_stats:
        return out, r, sinr[:14].copy(), float(sinr[14])
    return out


def ref_equalize_per_symbol(grid, estimates, noise_vars, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                            nof_cdm_groups_without_data, nof_layers, mmse=False):
    """The reference channel equalizer called once per OFDM symbol on that symbol's data REs, as
    pusch_demodulator_impl.cpp:318-333 calls it. Returns (complex64 [nre * L], float32 [nre * L])
    in codeword order -- the exact equalized symbols the reference demodulator demaps."""
    from . import ref_equalize

    P, _, nsubc = grid.shape
    mask = data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                        nof_cdm_groups_without_data)
    eqs, nvs = [], []
    for l in range(14):
        ks = np.nonzero(mask[l])[0]
        if ks.size == 0:
            continue
        sym = np.ascontiguousarray(grid[:, l, ks]).view(np.uint16)
        est = np.ascontiguousarray(np.transpose(estimates[:, :, l, ks], (1, 0, 2))).view(np.uint16)
        eq, nv = ref_equalize(sym, est, noise_vars, 1.0, nof_layers, mmse=mmse)
        eqs.append(eq.reshape(-1))
        nvs.append(nv.reshape(-1))
    return np.concatenate(eqs).astype(np.complex64), np.concatenate(nvs).astype(np.float32)


def demap_descramble_per_symbol(eq, nv, counts, qm, c_init, demod=None):
    """Restated tail of the demodulator on given equalized symbols: one demapper call per OFDM symbol
    (counts = demapper symbols per symbol), then revert_scrambling over the whole codeword.
    demod: the demapper (default the restated oracle.demodulate; oracle.ref_demodulate for the
    reference's demodulation_mapper_impl)."""
    demod = demod or demodulate
    parts, s0 = [], 0
    for n in counts:
        n = int(n)
        if n:
            parts.append(demod(eq[s0:s0 + n], nv[s0:s0 + n], qm))
            s0 += n
    llr = np.concatenate(parts)
    c = prbs(c_init, llr.size)
    return np.where(c == 1, -llr.astype(np.int16), llr.astype(np.int16)).astype(np.int8)

"""CPU oracle of the PUSCH demodulator -- TEST INFRASTRUCTURE ONLY.

Composition of restatements that are each pinned to the reference
(tests/test_oracle_vs_ref.py): data-RE selection of pusch_demodulator_impl.cpp:218-262
(rb_mask x 12 REs, DM-RS CDM groups without data removed on DM-RS symbols,
dmrs_mapping.h:76-91), channel equalizer (oracle/equalizer.py), soft demapper
(oracle.demodulate, srs_oracle_mod.c) and revert_scrambling
(pusch_demodulator_impl.cpp:36-190: LLR negated where c(n) = 1, c_init =
rnti * 2^15 + n_id).  The reference pusch_demodulator_impl class itself is not
wrapped (it needs the pusch_codeword_buffer / notifier / EVM-calculator
collaborators): its glue is restated, its numerics come from the pinned parts.
"""
import numpy as np

from . import demodulate, prbs
from .equalizer import equalize
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
                     dmrs_type2, nof_cdm_groups_without_data, nof_layers):
    """grid uint32 [P][14][nsubc]; estimates uint32 [P][L][14][nsubc]; noise_vars [P].
    Returns int8 LLRs (codeword order, descrambled)."""
    P, _, nsubc = grid.shape
    mask = data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                        nof_cdm_groups_without_data)
    ls, ks = np.nonzero(mask)
    sym = np.ascontiguousarray(grid[:, ls, ks]).view(np.uint16)                       # [P][2*nre]
    est = np.ascontiguousarray(np.transpose(estimates[:, :, ls, ks], (1, 0, 2))).view(np.uint16)  # [L][P][2*nre]
    eq, nv = equalize(sym, est, noise_vars, 1.0, nof_layers)
    llr = demodulate(eq.reshape(-1).astype(np.complex64), nv.reshape(-1).astype(np.float32), qm)
    c = prbs(rnti * (1 << 15) + n_id, llr.size)
    return np.where(c == 1, -llr.astype(np.int16), llr.astype(np.int16)).astype(np.int8)

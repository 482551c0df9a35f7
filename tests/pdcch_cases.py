"""PDCCH PDUs of the parity tests (tests/test_pdcch_gpu.py, tests/test_oracle_vs_ref.py): every CCE-to-REG mapping
(CORESET0, non-interleaved, interleaved with each REG bundle size), every aggregation level, 1-4 ports with complex
weights, power offsets (including one whose amplitude is subnormal, which the modulator does not apply), DCI sizes
from 12 to 128 bits (the maximum DCI payload) and CORESETs from symbol 0 to symbol 11."""
import numpy as np

from srsran_project_amd.pdcch import CceToRegMapping as M, make_pdu


def _payload(rng, n):
    return rng.integers(0, 2, n).astype(np.uint8)


def cases():
    rng = np.random.default_rng(7)
    c = []
    c.append(("nonil_al1_1port", dict(payload=_payload(rng, 39), bwp_size_rb=52, duration=1, aggregation_level=1,
                                      cce_index=3, rnti=0x4601, n_rnti=0x4601, n_id_pdcch_data=17,
                                      n_id_pdcch_dmrs=23)))
    c.append(("nonil_al4_2ports_power", dict(payload=_payload(rng, 57), bwp_size_rb=106, bwp_start_rb=4,
                                             frequency_resources=[0, 2, 3, 7, 9, 12, 16], duration=2,
                                             aggregation_level=4, cce_index=4, data_power_offset_dB=-3.0,
                                             dmrs_power_offset_dB=3.0, weights=(0.5 + 0.5j, -0.5 + 0.25j),
                                             slot_index=5, numerology=1, start_symbol_index=2)))
    c.append(("il_L6_R2_al8", dict(payload=_payload(rng, 44), bwp_size_rb=51, frequency_resources=range(8),
                                   duration=1, cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=6,
                                   interleaver_size=2, shift_index=7, aggregation_level=8, cce_index=0)))
    c.append(("il_L2_R3_dur2", dict(payload=_payload(rng, 33), bwp_size_rb=60, bwp_start_rb=12,
                                    frequency_resources=[1, 2, 3, 4, 5, 6], duration=2,
                                    cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=2, interleaver_size=3,
                                    shift_index=101, aggregation_level=8, cce_index=4, start_symbol_index=1)))
    c.append(("il_L3_R6_dur3_al16", dict(payload=_payload(rng, 100), bwp_size_rb=100, frequency_resources=range(12),
                                         duration=3, cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=3,
                                         interleaver_size=6, shift_index=275, aggregation_level=16, cce_index=16,
                                         weights=(1.0, 1j, -1.0, -1j), slot_index=9)))
    c.append(("coreset0_al4", dict(payload=_payload(rng, 41), bwp_size_rb=48, bwp_start_rb=10,
                                   frequency_resources=range(8), duration=2, cce_to_reg_mapping=M.CORESET0,
                                   shift_index=500, aggregation_level=4, cce_index=4, rnti=0xFFFF, n_rnti=0,
                                   n_id_pdcch_data=500, n_id_pdcch_dmrs=500)))
    c.append(("nonil_al16_k152_4ports", dict(payload=_payload(rng, 128), bwp_size_rb=273, duration=3,
                                             aggregation_level=16, cce_index=112, numerology=1, slot_index=17,
                                             weights=(0.5, 0.5j, -0.5, 0.3 - 0.4j), start_symbol_index=11,
                                             n_id_pdcch_data=65535, n_id_pdcch_dmrs=65535, n_rnti=65535,
                                             rnti=0x1234)))
    c.append(("nonil_al2_k36_subnormal_amp", dict(payload=_payload(rng, 12), bwp_size_rb=24, duration=1,
                                                  aggregation_level=2, cce_index=2, data_power_offset_dB=-800.0,
                                                  dmrs_power_offset_dB=-6.0)))
    c.append(("nonil_al16_dur1_96rb", dict(payload=_payload(rng, 70), bwp_size_rb=120, bwp_start_rb=3, duration=1,
                                           aggregation_level=16, cce_index=0, weights=(0.25 - 0.5j, 0.75j),
                                           start_symbol_index=13)))
    c.append(("coreset0_dur1_al4", dict(payload=_payload(rng, 39), bwp_size_rb=24, bwp_start_rb=0,
                                        frequency_resources=range(4), duration=1, cce_to_reg_mapping=M.CORESET0,
                                        shift_index=1, aggregation_level=4, cce_index=0, numerology=1,
                                        slot_index=3)))
    return [(name, make_pdu(**kw)) for name, kw in c]


def slot_pdus(nof_grids=3, nsubc=12 * 106):
    """Several DCIs per grid (non-overlapping CCEs of two CORESETs) over nof_grids grids."""
    rng = np.random.default_rng(11)
    out = []
    for g in range(nof_grids):
        for k, (al, cce) in enumerate([(1, 0), (2, 2), (4, 4), (8, 8)]):
            out.append(make_pdu(payload=_payload(rng, 39 + 4 * k + g), bwp_size_rb=nsubc // 12, duration=2,
                                aggregation_level=al, cce_index=cce, rnti=0x4601 + k, n_rnti=0x4601 + k,
                                n_id_pdcch_data=g, n_id_pdcch_dmrs=g + 1, slot_index=4 + g, numerology=1,
                                weights=(1.0, 0.5j), grid=g))
        out.append(make_pdu(payload=_payload(rng, 60), bwp_size_rb=nsubc // 12, frequency_resources=range(8),
                            start_symbol_index=2, duration=1, cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=6,
                            interleaver_size=2, shift_index=g, aggregation_level=4, cce_index=4, slot_index=4 + g,
                            numerology=1, weights=(0.7, -0.7), grid=g))
    return out


INVALID = [
    ("aggregation_level_3", dict(aggregation_level=3), "Invalid aggregation level"),
    ("cce_overflow", dict(aggregation_level=8, cce_index=2, frequency_resources=[0]), "exceeds CORESET capacity"),
    ("duration_4", dict(duration=4), "out of the range"),
    ("symbol_overflow", dict(duration=3, start_symbol_index=12), "exceeds the slot"),
    ("bad_bundle", dict(cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=3, duration=2), "Invalid REG bundle size"),
    ("bad_interleaver", dict(cce_to_reg_mapping=M.INTERLEAVED, reg_bundle_size=6, interleaver_size=4),
     "Invalid interleaver size"),
]

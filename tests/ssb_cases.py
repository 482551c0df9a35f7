"""SS/PBCH block PDUs for the SSB tests: every pattern case (A-E), L_max 4 / 8 / 64, both half frames, SFN bit
combinations, k_SSB with and without its 5th bit, PCIs over every DM-RS shift v = PCI mod 4, PSS power offsets, 1-4
ports.  TEST INFRASTRUCTURE ONLY."""
import numpy as np

import srsran_project_amd as amd

NPRB = 273
NSUBC = 12 * NPRB

# (name, kwargs of make_pdu)
CASES = [
    ("A_L4_idx0", dict(numerology=0, sfn=5, slot_index=0, phys_cell_id=1, ssb_idx=0, L_max=4, common_scs=0,
                       subcarrier_offset=0, offset_to_pointA=2, pattern_case=0, ports=(0,))),
    ("A_L4_idx1_hrf_pss3dB", dict(numerology=0, sfn=1023, slot_index=5, phys_cell_id=502, ssb_idx=1, L_max=4,
                                  common_scs=0, subcarrier_offset=7, offset_to_pointA=10, pattern_case=0,
                                  beta_pss_dB=3.0, ports=(0, 1))),
    ("A_L8_idx3_kssb23", dict(numerology=0, sfn=6, slot_index=6, phys_cell_id=1007, ssb_idx=3, L_max=8, common_scs=1,
                              subcarrier_offset=23, offset_to_pointA=0, pattern_case=0, ports=(1,))),
    ("B_L8_idx2_4ports", dict(numerology=1, sfn=2, slot_index=1, phys_cell_id=17, ssb_idx=2, L_max=8, common_scs=1,
                              subcarrier_offset=4, offset_to_pointA=6, pattern_case=1, beta_pss_dB=-3.0,
                              ports=(0, 1, 2, 3))),
    ("C_L8_idx5_hrf", dict(numerology=1, sfn=3, slot_index=12, phys_cell_id=300, ssb_idx=5, L_max=8, common_scs=0,
                           subcarrier_offset=2, offset_to_pointA=20, pattern_case=2, ports=(2, 3))),
    ("D_L64_idx37", dict(numerology=3, sfn=700, slot_index=22, phys_cell_id=888, ssb_idx=37, L_max=64, common_scs=3,
                         subcarrier_offset=5, offset_to_pointA=4, pattern_case=3, ports=(0,))),
    ("E_L64_idx60_hrf", dict(numerology=4, sfn=13, slot_index=114, phys_cell_id=0, ssb_idx=60, L_max=64, common_scs=2,
                             subcarrier_offset=8, offset_to_pointA=10, pattern_case=4, beta_pss_dB=1.5,
                             ports=(0, 1))),
    ("A_L4_idx0_pci3", dict(numerology=0, sfn=4, slot_index=0, phys_cell_id=3, ssb_idx=0, L_max=4, common_scs=0,
                            subcarrier_offset=16, offset_to_pointA=100, pattern_case=0, ports=(3,))),
]

# the reference asserts (aborts) on these; the C-ABI rejects them with the reason
INVALID = [
    ("wrong_slot", dict(numerology=0, sfn=0, slot_index=1, ssb_idx=0, pattern_case=0)),
    ("non_integer_subcarrier", dict(numerology=1, sfn=0, slot_index=0, ssb_idx=0, pattern_case=1, common_scs=1,
                                    subcarrier_offset=1, offset_to_pointA=0)),
    ("fr2_common_scs_15", dict(numerology=3, sfn=0, slot_index=0, ssb_idx=0, L_max=64, pattern_case=3, common_scs=0)),
    ("kssb_over_fr2_max", dict(numerology=3, sfn=0, slot_index=0, ssb_idx=0, L_max=64, pattern_case=3, common_scs=3,
                               subcarrier_offset=12)),
    ("index_out_of_range", dict(numerology=3, sfn=0, slot_index=0, ssb_idx=64, L_max=64, pattern_case=3,
                                common_scs=3)),
]


def pdu(case, seed=0, grid=0):
    rng = np.random.default_rng(seed)
    return amd.ssb.make_pdu(rng.integers(0, 2, 24), grid=grid, **case[1])


def grid0(seed=1, ports=4):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 1 << 32, (ports, 14, NSUBC), dtype=np.uint64).astype(np.uint32)

"""Shared PDSCH modulator / DM-RS test cases (oracle vs reference on the CPU,
MI355X vs oracle on the GPU). The reference's own modulator sweep
(tests/unittests/phy/upper/channel_processors/pdsch/pdsch_modulator_test_data.h:
QPSK..256QAM, 1/2/4 layers, identity precoding, <= 52 PRB, type-1 DM-RS) is
extended to 273 PRB, non-identity precoding, reserved REs, sparse CRB sets and
type-2 DM-RS; its .dat vectors are not in the reference tree."""
import numpy as np

from oracle import pdsch_mod as pm

# (name, nof_prb, qm, layers, ports, crbs, start, nof_symbols, dmrs_mask, dmrs_type2, cdm_no_data, reserved, scaling)
MOD_CASES = [
    ("qpsk_1x1_25prb", 25, 2, 1, 1, (0, 25), 1, 13, (1 << 2) | (1 << 11), False, 2, [], 1.0),
    ("16qam_2x2_52prb_reserved", 52, 4, 2, 2, (3, 50), 2, 12, (1 << 2) | (1 << 7) | (1 << 11), False, 1,
     [((5, 9), 0b111100001111, (1 << 5) | (1 << 6))], 0.7),
    ("64qam_3x4_106prb_type2", 106, 6, 3, 4, (0, 106), 0, 14, (1 << 2) | (1 << 3), True, 2,
     [((0, 106, 4), 0b000100010001, 1 << 9)], 1.0),
    ("256qam_4x4_273prb", 273, 8, 4, 4, (0, 273), 0, 14, (1 << 2) | (1 << 11), False, 2, [], 1.0),
    ("256qam_2x4_sparse", 100, 8, 2, 4, "sparse", 1, 10, 1 << 2, True, 3, [], 2.0),
    ("bpsk_pi2_1x2", 24, 0, 1, 2, (2, 20), 3, 9, 1 << 3, False, 1, [], 1.0),
]


def _crbs(spec, nof_prb, rng):
    if spec == "sparse":
        return np.sort(rng.choice(nof_prb, nof_prb // 2, replace=False))
    return np.arange(spec[0], spec[1])


def _reserved(res, nof_prb):
    out = []
    for r in res:
        (rng_spec, re_mask, symbols) = r
        cm = np.zeros(pm.MAX_RB, bool)
        if len(rng_spec) == 3:
            cm[rng_spec[0]:rng_spec[1]:rng_spec[2]] = True
        else:
            cm[rng_spec[0]:rng_spec[1]] = True
        out.append((cm, re_mask, symbols))
    return out


def mod_case(case, seed=0):
    """Returns dict: grid0 (uint16 [P][14][nsubc][2]), bits (one per byte), oracle kwargs."""
    name, nof_prb, qm, L, P, crbs, start, ns, dmrs, t2, ncdm, res, scaling = case
    rng = np.random.default_rng(seed)
    crbs = _crbs(crbs, nof_prb, rng)
    reserved = _reserved(res, nof_prb)
    nsubc = 12 * nof_prb
    bwp = np.zeros(pm.MAX_RB, bool)
    bwp[:nof_prb] = True
    mask = pm.data_re_mask(nsubc, crbs, start, ns, reserved + [(bwp, pm.dmrs_prb_mask(t2, ncdm), dmrs)])
    nre = int(mask.sum())
    bits = rng.integers(0, 2, nre * L * (qm if qm > 1 else 1)).astype(np.uint8)
    if L == 1 and P == 1:
        W = np.ones((1, 1), np.complex64)
    else:
        W = ((rng.normal(size=(L, P)) + 1j * rng.normal(size=(L, P))) / np.sqrt(2 * P)).astype(np.complex64)
    grid0 = rng.integers(0, 1 << 16, (P, 14, nsubc, 2)).astype(np.uint16)
    kw = dict(rnti=int(rng.integers(1, 65520)), n_id=int(rng.integers(0, 1024)), qm=qm, crbs=crbs,
              start_symbol=start, nof_symbols=ns, dmrs_symb_mask=dmrs, dmrs_type2=t2,
              nof_cdm_groups_without_data=ncdm, reserved=reserved, weights=W, scaling=scaling, bwp=(0, nof_prb))
    return grid0, bits, kw


# (name, nof_prb, type2, layers, ports, crbs, symbols_mask, ref_k_rb)
DMRS_CASES = [
    ("t1_1x1", 25, False, 1, 1, (0, 25), (1 << 2) | (1 << 11), 0),
    ("t1_2x2_ref", 52, False, 2, 2, (4, 40), (1 << 2) | (1 << 3), 2),
    ("t1_4x4_273", 273, False, 4, 4, (0, 273), (1 << 2) | (1 << 7) | (1 << 11), 0),
    ("t2_3x4", 106, True, 3, 4, "sparse", (1 << 2) | (1 << 3) | (1 << 9), 0),
    ("t2_4x4", 51, True, 4, 4, (0, 51), 1 << 2, 0),
]


def dmrs_case(case, seed=0):
    name, nof_prb, t2, L, P, crbs, symbols, ref = case
    rng = np.random.default_rng(seed + 100)
    crbs = _crbs(crbs, nof_prb, rng)
    crbs = crbs[crbs >= ref]
    W = ((rng.normal(size=(1, L, P)) + 1j * rng.normal(size=(1, L, P))) / np.sqrt(2 * P)).astype(np.complex64)
    if L == 1 and P == 1:
        W = np.ones((1, 1, 1), np.complex64)
    grid0 = rng.integers(0, 1 << 16, (P, 14, 12 * nof_prb, 2)).astype(np.uint16)
    kw = dict(slot_index=int(rng.integers(0, 20)), reference_point_k_rb=ref, dmrs_type2=t2,
              scrambling_id=int(rng.integers(0, 65536)), n_scid=int(rng.integers(0, 2)),
              amplitude=float(rng.uniform(0.5, 2.0)), symbols_mask=symbols, crbs=crbs, weights=W)
    return grid0, kw

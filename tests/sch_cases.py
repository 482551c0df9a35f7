"""Transport-block test cases shared by the oracle-vs-reference and GPU tests."""
import numpy as np

# (tbs, base graph, Qm, layers, channel symbols, rv, Nref)
SCH_CASES = [
    (8 * 3, 2, 2, 1, 96, 0, 0),            # tiny TB, CRC16, BG2 Z small
    (8 * 100, 2, 2, 1, 600, 0, 0),         # CRC16, C = 1
    (8 * 478, 2, 4, 2, 1400, 1, 0),        # CRC16 boundary (TBS 3824), two layers
    (8 * 500, 1, 4, 1, 1800, 0, 0),        # CRC24A, C = 1, BG1
    (8 * 1056, 1, 6, 1, 2000, 2, 0),       # C = 2 (BG1 segmentation)
    (8 * 3000, 2, 6, 2, 12000, 3, 0),      # BG2 C = 7
    (8 * 4000, 1, 8, 4, 8400, 0, 25344),   # limited buffer rate matching
    (8 * 12000, 1, 2, 2, 96000, 0, 0),     # low rate, C = 12
]


def tb_bytes(tbs, seed):
    return np.random.default_rng(seed).integers(0, 256, tbs // 8).astype(np.uint8)


def noisy_llrs(cw_bits, amp, sigma, seed):
    rng = np.random.default_rng(seed)
    x = (1 - 2 * cw_bits.astype(np.float64)) * amp + rng.normal(0, sigma, cw_bits.size)
    return np.clip(np.round(x), -120, 120).astype(np.int8)

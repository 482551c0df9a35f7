"""Shared input generators for the LDPC parity tests (seeded, deterministic)."""
import numpy as np

import oracle


def noisy_codeblocks(bg, Z, n, length=None, snr_amp=10, noise=8.0, seed=0, crc_poly=None):
    """Encodes n random messages (optionally with a CRC appended to the message)
    and returns (messages [n, K] bits, llrs [n, length] int8)."""
    rng = np.random.default_rng(seed)
    K = oracle.BG_K[bg] * Z
    N = oracle.BG_N_SHORT[bg] * Z
    L = N if length is None else length
    msgs = np.zeros((n, K), np.uint8)
    llrs = np.zeros((n, L), np.int8)
    for i in range(n):
        m = rng.integers(0, 2, K).astype(np.uint8)
        if crc_poly is not None:
            L_crc = 24 if crc_poly in (0, 1, 2) else 16
            c = oracle.crc_bits(crc_poly, m[:K - L_crc])
            m[K - L_crc:] = [(c >> (L_crc - 1 - b)) & 1 for b in range(L_crc)]
        cw = oracle.ldpc_encode(m, bg, Z)[:L]
        x = (1 - 2 * cw.astype(np.float64)) * snr_amp + rng.normal(0, noise, L)
        llrs[i] = np.clip(np.round(x), -120, 120).astype(np.int8)
        msgs[i] = m
    return msgs, llrs

"""Shared PUSCH demodulator test cases (CPU oracle pin and GPU parity).

Channels: "random" (frequency selective) and "identity" (unit estimates,
equal power-of-two noise variances). The reference's ZF equalizer multiplies by
an approximate reciprocal (AVX2 rcp), so even the identity channel does not give
exact equalized symbols: LLR parity of the whole demodulator is |dLLR| <= 1.
The demapper block structure (one demapper call per OFDM symbol,
pusch_demodulator_impl.cpp:363-400) is pinned bit-exactly instead by feeding
the reference's own per-symbol equalizer output (ref_equalize_per_symbol) and
dyadic symbols that sit on the SIMD/scalar rounding ties (dyadic_equalized).
Cases include the configs[0] shape (51 PRB SISO), the headline 273-PRB 4x2
256QAM and allocations whose data REs per OFDM symbol x layers are not a
multiple of the demapper's SIMD block (16 symbols QPSK/64QAM, 8 16QAM, 4 256QAM).
"""
import numpy as np

from tests.chest_cases import bf16_grid

# (name, ports, layers, nof_prb, (crb lo, hi), qm, start, nsym, dmrs mask, cdm groups without data)
CASES = [
    ("1x1_qpsk", 1, 1, 52, (0, 52), 2, 0, 14, (1 << 2) | (1 << 11), 2),
    ("2x1_16qam_cdm1", 2, 1, 52, (4, 40), 4, 1, 13, (1 << 2), 1),
    ("4x1_64qam", 4, 1, 106, (0, 106), 6, 0, 14, (1 << 2) | (1 << 7) | (1 << 11), 2),
    ("2x2_256qam_273", 2, 2, 273, (0, 273), 8, 0, 14, (1 << 2) | (1 << 11), 2),
    ("4x2_64qam", 4, 2, 51, (0, 51), 6, 0, 14, (1 << 2), 1),
    # configs[0]: 20 MHz at 30 kHz = 51 PRB, SISO, MCS 9 (QPSK): 612 REs / data symbol (tail 4 of 16)
    ("cfg0_1x1_qpsk_51", 1, 1, 51, (0, 51), 2, 0, 14, (1 << 2) | (1 << 11), 2),
    # headline PUSCH: 273 PRB, 4 rx x 2 layers, 256QAM
    ("4x2_256qam_273", 4, 2, 273, (0, 273), 8, 0, 14, (1 << 2) | (1 << 11), 2),
    # tails: 5 PRB 16QAM cdm1 -> 30 REs on the DM-RS symbol (30 % 8 = 6), 60 elsewhere (60 % 8 = 4)
    ("1x1_16qam_5prb_tail", 1, 1, 20, (3, 8), 4, 0, 14, (1 << 2), 1),
    # 256QAM 1 layer 7 PRB: 84 REs (84 % 4 = 0) and DM-RS cdm1 42 (42 % 4 = 2)
    ("2x1_256qam_7prb_tail", 2, 1, 25, (9, 16), 8, 2, 11, (1 << 2) | (1 << 8), 1),
    # 64QAM 2 layers 3 PRB: 36 x 2 = 72 (72 % 16 = 8)
    ("2x2_64qam_3prb_tail", 2, 2, 24, (0, 3), 6, 0, 14, (1 << 3), 2),
]


# L-layer topologies the open reference's equalizer asserts for (parity unpinned): (name, ports, layers, nof_prb,
# crbs, qm, start, nsym, dmrs mask, cdm groups without data, algorithm)
MIMO_CASES = [
    ("4x4_256qam_273_mmse", 4, 4, 273, (0, 273), 8, 0, 14, (1 << 2) | (1 << 11), 2, "mmse"),
    ("4x4_64qam_51_zf", 4, 4, 51, (0, 51), 6, 0, 14, (1 << 2), 2, "zf"),
    ("4x3_16qam_52_mmse", 4, 3, 52, (4, 40), 4, 1, 13, (1 << 3) | (1 << 10), 2, "mmse"),
    ("4x3_qpsk_25_zf", 4, 3, 25, (0, 25), 2, 0, 14, (1 << 2), 2, "zf"),
    ("4x2_256qam_106_mmse", 4, 2, 106, (0, 106), 8, 0, 14, (1 << 2) | (1 << 11), 1, "mmse"),
    ("2x2_64qam_24_mmse", 2, 2, 24, (0, 24), 6, 0, 14, (1 << 3), 2, "mmse"),
]


def make_case(case, seed, kind="random"):
    """Returns (grid uint32 [P][14][nsubc], estimates uint32 [P][L][14][nsubc], noise vars [P], crbs)."""
    name, P, L, nprb, (lo, hi), qm, start, nsym, dmrs, ncdm = case[:10]
    rng = np.random.default_rng(seed)
    nsubc = 12 * nprb
    k = np.arange(nsubc)
    h = np.zeros((P, L, 14, nsubc), np.complex64)
    if kind == "mimo":
        # full-rank frequency-selective channel: random complex gains, one delay per (port, layer)
        g = (rng.normal(size=(P, L)) + 1j * rng.normal(size=(P, L))) * 0.6 + 0.8 * np.eye(P, L)
        tau = rng.integers(0, 24, (P, L))
        for p in range(P):
            for v in range(L):
                h[p, v] = (g[p, v] * np.exp(-2j * np.pi * k * tau[p, v] / 4096))[None, :]
        x = ((rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1) + 1j * (rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1)) * 0.7
        y = np.einsum("pvls,vls->pls", h, x) + 0.03 * (rng.normal(size=(P, 14, nsubc))
                                                       + 1j * rng.normal(size=(P, 14, nsubc)))
        nv = (0.0018 * (1 + 0.1 * np.arange(P))).astype(np.float32)
        return bf16_grid(y), bf16_grid(h), nv, list(range(lo, hi))
    if kind == "identity":
        for p in range(P):
            h[p, p % L] = 1.0
        amp = 2.0 ** -int(rng.integers(0, 3))
        x = ((rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1) + 1j * (rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1))
        x = x * amp * (0.25 + 0.75 * rng.random((L, 14, nsubc)))
        y = np.einsum("pvls,vls->pls", h, x)
        nv = np.full(P, 2.0 ** -6, np.float32)
    else:
        for p in range(P):
            for v in range(L):
                h[p, v] = ((0.7 + 0.2 * p - 0.3j * v) * np.exp(-2j * np.pi * k * (2 + p + 3 * v) / 4096))[None, :]
        x = ((rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1) + 1j * (rng.integers(0, 2, (L, 14, nsubc)) * 2 - 1)) * 0.7
        y = np.einsum("pvls,vls->pls", h, x) + 0.05 * (rng.normal(size=(P, 14, nsubc))
                                                       + 1j * rng.normal(size=(P, 14, nsubc)))
        nv = (0.005 * (1 + 0.1 * np.arange(P))).astype(np.float32)
    return bf16_grid(y), bf16_grid(h), nv, list(range(lo, hi))


def demod_args(case):
    name, P, L, nprb, _, qm, start, nsym, dmrs, ncdm = case[:10]
    d = dict(qm=qm, start_symbol=start, nof_symbols=nsym, dmrs_symb_mask=dmrs, dmrs_type2=False,
             nof_cdm_groups_without_data=ncdm, nof_layers=L)
    if len(case) > 10:
        d["mmse"] = case[10] == "mmse"
    return d


def assert_llrs_close(got, want, what, min_equal=0.99):
    """Float equalizer inside: |dLLR| <= 1 and at least min_equal of them identical."""
    assert got.shape == want.shape, what
    d = np.abs(got.astype(np.int16) - want.astype(np.int16))
    assert d.max() <= 1, "%s: max |dLLR| %d" % (what, d.max())
    assert (d == 0).mean() >= min_equal, "%s: only %.4f equal" % (what, (d == 0).mean())


SIMD_BLOCK = {2: 16, 4: 8, 6: 16, 8: 4}  # demapper symbols per AVX2 block (demodulation_mapper_*.cpp)


def dyadic_equalized(qm, n, seed, demod):
    """n equalized symbols / noise variances on a dyadic grid, half of them drawn from values where the
    demapper `demod`'s SIMD and scalar-tail arithmetic give different LLRs (rounding ties), so a demapper
    block boundary in the wrong place shows up."""
    rng = np.random.default_rng(seed)
    m = 4096
    s = (rng.integers(-64, 65, m) / 32.0 + 1j * rng.integers(-64, 65, m) / 32.0).astype(np.complex64)
    v = (2.0 ** -rng.integers(0, 5, m)).astype(np.float32)
    blk = SIMD_BLOCK[qm]
    m -= m % blk
    simd = demod(s[:m], v[:m], qm).reshape(m, -1)
    tail = blk - 1  # calls shorter than a block run the scalar code only
    scal = np.concatenate([demod(s[i:i + tail], v[i:i + tail], qm) for i in range(0, m - tail + 1, tail)])
    k = scal.size // simd.shape[1]
    diff = np.nonzero((simd[:k] != scal.reshape(k, -1)).any(axis=1))[0]
    pick = rng.integers(0, m, n)
    if diff.size:
        sens = rng.random(n) < 0.5
        pick[sens] = diff[rng.integers(0, diff.size, int(sens.sum()))]
    return s[pick], v[pick]

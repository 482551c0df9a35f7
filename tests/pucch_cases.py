"""PUCCH Format 0 PDUs with transmitted cyclic shifts (or noise only): 1-2 symbols, frequency hopping, 0-2 HARQ-ACK
bits with and without an SR opportunity, 1-4 ports, slots across numerologies, SNRs from well above to below the
detection threshold.  TEST INFRASTRUCTURE ONLY."""
import numpy as np

import srsran_project_amd as amd

NSUBC = 12 * 52


def cases(n=24, seed=0):
    """[(pdu, grid uint32 [4][14][NSUBC], transmitted table index or None)]"""
    from oracle import pucch as op

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        nh = int(rng.integers(0, 3))
        sr = bool(rng.integers(0, 2)) or nh == 0
        nsym = int(rng.integers(1, 3))
        hop = int(rng.integers(0, 52)) if (nsym == 2 and rng.integers(0, 2)) else None
        nports = int(rng.integers(1, 5))
        mu = int(rng.integers(0, 3))
        pdu = amd.pucch.make_f0_pdu(numerology=mu, slot_index=int(rng.integers(0, 10 << mu)),
                                    starting_prb=int(rng.integers(0, 52)), second_hop_prb=hop,
                                    start_symbol_index=int(rng.integers(0, 15 - nsym)), nof_symbols=nsym,
                                    initial_cyclic_shift=int(rng.integers(0, 12)), n_id=int(rng.integers(0, 1024)),
                                    nof_harq_ack=nh, sr_opportunity=sr,
                                    ports=tuple(int(x) for x in rng.permutation(4)[:nports]))
        table = op.TABLES[(nh, sr)]
        sent = None if i % 6 == 5 else int(rng.integers(0, len(table)))
        grid = rng.integers(0, 1 << 32, (4, 14, NSUBC), dtype=np.uint64).astype(np.uint32)
        gains = (rng.normal(size=nports) + 1j * rng.normal(size=nports)) / np.sqrt(2)
        noise = [0.01, 0.1, 1.0, 3.0][i % 4]
        op.transmit(grid, pdu, None if sent is None else table[sent][0], gains, noise, rng)
        out.append((pdu, grid, sent))
    return out


def f1_cases(n=16, seed=0):
    """[(batch, grid uint32 [4][14][NSUBC], {(shift, occ): transmitted bits})]: 4-14 symbols from symbols 0-10, with
    and without frequency hopping, 1 / 2 / 4 ports, 1-6 multiplexed PUCCHs of 0-2 HARQ-ACK bits of which some are
    silent (DTX), noise variance 0.01-3 against unit-power channel taps."""
    from oracle import pucch as op

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        hop = bool(rng.integers(0, 2))
        nports = [1, 2, 4][int(rng.integers(0, 3))]
        start = int(rng.integers(0, 11))
        nsym = int(rng.integers(4, 15 - start))
        mu = int(rng.integers(0, 3))
        nocc = nsym // (4 if hop else 2)
        k = int(rng.integers(1, 7))
        coords = set()
        while len(coords) < k:
            coords.add((int(rng.integers(0, 12)), int(rng.integers(0, nocc))))
        entries = [(ics, o, int(rng.integers(0, 3))) for ics, o in sorted(coords, key=lambda c: rng.random())]
        b = amd.pucch.make_f1_batch(entries, numerology=mu, slot_index=int(rng.integers(0, 10 << mu)),
                                    starting_prb=int(rng.integers(0, 52)),
                                    second_hop_prb=int(rng.integers(0, 52)) if hop else None,
                                    start_symbol_index=start, nof_symbols=nsym, n_id=int(rng.integers(0, 1024)),
                                    ports=tuple(int(x) for x in rng.permutation(4)[:nports]))
        sent = {}
        pucchs = []
        for ics, o, nh in entries:
            if rng.random() < 0.2:
                continue  # DTX
            bits = [int(x) for x in rng.integers(0, 2, nh)]
            sent[(ics, o)] = bits
            gains = (rng.normal(size=nports) + 1j * rng.normal(size=nports)) / np.sqrt(2)
            pucchs.append((ics, o, bits, gains))
        grid = rng.integers(0, 1 << 32, (4, 14, NSUBC), dtype=np.uint64).astype(np.uint32)
        op.transmit_f1(grid, b, pucchs, [0.01, 0.1, 1.0, 3.0][i % 4], rng)
        out.append((b, grid, sent))
    return out


def f2_cases(n=16, seed=0):
    """[(pdu, grid uint32 [4][14][NSUBC], payload bits)]: 1-16 PRBs, 1-2 symbols, hopping, 1-4 ports (0 .. n-1: the
    reference's demodulator reads grid ports 0 .. n-1), 3-11 bit (Reed-Muller) and 12+ bit (polar) payloads within the
    0.8 code rate, SNRs from clean to failing."""
    from oracle import pucch as op

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        nprb = int(rng.integers(1, 17))
        nsym = int(rng.integers(1, 3))
        hop = nsym == 2 and i % 3 == 0
        nports = int(rng.integers(1, 5))
        mu = int(rng.integers(0, 3))
        E = 16 * nprb * nsym
        kmax = max(3, min(int(0.8 * E) - 11, 300))
        K = int(rng.integers(3, 12)) if (i % 2 == 0 or kmax < 12) else int(rng.integers(12, kmax + 1))
        while K > 11 and (K + (6 if K < 20 else 11)) > 0.8 * E:
            K -= 1
        if K > 11 and K + (6 if K < 20 else 11) > 0.8 * E or (K <= 11 and K > 0.8 * E):
            K = 3
        nh = int(rng.integers(0, K + 1))
        nsr = int(rng.integers(0, min(4, K - nh) + 1))
        pdu = amd.pucch.make_f2_pdu(numerology=mu, slot_index=int(rng.integers(0, 10 << mu)), bwp_start_rb=2,
                                    bwp_size_rb=48, starting_prb=int(rng.integers(0, 48 - nprb + 1)),
                                    second_hop_prb=int(rng.integers(0, 48 - nprb + 1)) if hop else None,
                                    nof_prb=nprb, start_symbol_index=int(rng.integers(0, 15 - nsym)),
                                    nof_symbols=nsym, rnti=int(rng.integers(1, 65536)), n_id=int(rng.integers(0, 1024)),
                                    n_id_0=int(rng.integers(0, 65536)), nof_harq_ack=nh, nof_sr=nsr,
                                    nof_csi_part1=K - nh - nsr, ports=tuple(range(nports)))
        payload = rng.integers(0, 2, K).astype(np.uint8)
        grid = rng.integers(0, 1 << 32, (4, 14, NSUBC), dtype=np.uint64).astype(np.uint32)
        gains = (rng.normal(size=nports) + 1j * rng.normal(size=nports)) / np.sqrt(2)
        op.transmit_f2(grid, pdu, payload, gains, [0.001, 0.03, 0.3, 3.0][i % 4], rng)
        out.append((pdu, grid, payload))
    return out


F3_PRBS = [1, 2, 3, 4, 5, 6, 8, 9, 10, 12, 15, 16]


def f34_cases(n=16, seed=0, fmt=None):
    """[(pdu, grid uint32 [4][14][NSUBC], payload bits)]: Formats 3 (1-16 PRBs of the transform-precoding sizes) and 4
    (OCC 2 / 4), 4-14 symbols, hopping, additional DM-RS, QPSK and pi/2-BPSK, 1-4 ports in any order, Reed-Muller and
    polar payloads within the 0.8 code rate, SNRs from clean to failing."""
    from oracle import pucch as op

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        f = fmt if fmt is not None else (3 if i % 3 else 4)
        nprb = F3_PRBS[int(rng.integers(0, len(F3_PRBS)))] if f == 3 else 1
        nsym = int(rng.integers(4, 15))
        hop = bool(rng.integers(0, 2))
        add = bool(rng.integers(0, 2))
        pi2 = bool(rng.integers(0, 2))
        occ = [2, 4][int(rng.integers(0, 2))]
        nports = int(rng.integers(1, 5))
        mu = int(rng.integers(0, 3))
        kw = dict(format=f, numerology=mu, slot_index=int(rng.integers(0, 10 << mu)), bwp_start_rb=1, bwp_size_rb=50,
                  starting_prb=int(rng.integers(0, 50 - nprb + 1)),
                  second_hop_prb=int(rng.integers(0, 50 - nprb + 1)) if hop else None, nof_prb=nprb,
                  start_symbol_index=int(rng.integers(0, 15 - nsym)), nof_symbols=nsym,
                  rnti=int(rng.integers(1, 65536)), n_id_hopping=int(rng.integers(0, 1024)),
                  n_id_scrambling=int(rng.integers(0, 1024)), additional_dmrs=add, pi2_bpsk=pi2,
                  occ_index=int(rng.integers(0, occ)), occ_length=occ,
                  ports=tuple(int(x) for x in rng.permutation(4)[:nports]))
        probe = amd.pucch.make_f34_pdu(nof_harq_ack=3, **kw)
        E = amd.pucch.f34_nof_llrs(probe)
        chan = E  # the codeword E (the validator's Format 4 rate counts 12 REs per symbol whatever the OCC)
        K = int(rng.integers(3, 12)) if i % 2 == 0 else int(rng.integers(12, max(13, min(int(0.8 * chan) - 11, 200))))
        while K > 3 and (K + (0 if K <= 11 else (6 if K < 20 else 11))) > 0.8 * chan:
            K -= 1
        nh = int(rng.integers(0, K + 1))
        nsr = int(rng.integers(0, min(4, K - nh) + 1))
        pdu = amd.pucch.make_f34_pdu(nof_harq_ack=nh, nof_sr=nsr, nof_csi_part1=K - nh - nsr, **kw)
        payload = rng.integers(0, 2, K).astype(np.uint8)
        grid = rng.integers(0, 1 << 32, (4, 14, NSUBC), dtype=np.uint64).astype(np.uint32)
        gains = (rng.normal(size=nports) + 1j * rng.normal(size=nports)) / np.sqrt(2)
        op.transmit_f34(grid, pdu, payload, gains, [0.001, 0.03, 0.3, 3.0][i % 4], rng)
        out.append((pdu, grid, payload))
    return out

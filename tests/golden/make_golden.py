#!/usr/bin/env python3
"""Generates tests/golden/ldpc_golden.npz from the REFERENCE decoders/encoder
compiled from /root/reference (oracle/_ref/libsrsran_ref.so).

The reference's own LDPC test vectors (ldpc_encoder_test_input*.dat, MATLAB
generated, tests/unittests/phy/upper/channel_coding/ldpc/ldpc_encoder_test_data.h)
are not shipped in /root/reference, so the golden vectors here are produced by
running the reference code itself on seeded inputs that follow the same recipe
(random messages, encoded, LLR amplitude 10, plus AWGN-like noise).
Run once in the build container: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

assert oracle.REF is not None, "build oracle/_ref first (make -C oracle)"

CASES = []  # (impl, bg, Z, L_nodes or None, iters, crc_poly, filler, noise)
for bg in (1, 2):
    for Z in (2, 7, 15, 36, 104):
        CASES.append(("avx2", bg, Z, None, 6, -1, 0, 8.0))
        CASES.append(("generic", bg, Z, None, 6, -1, 0, 8.0))
CASES += [("avx2", 1, 384, None, 8, -1, 0, 9.0), ("avx2", 1, 384, None, 8, 1, 0, 9.0),
          ("generic", 2, 384, None, 8, -1, 0, 9.0), ("avx2", 1, 64, 38, 5, 0, 64, 7.0),
          ("avx2", 2, 26, 20, 4, 3, 0, 6.0), ("avx2", 1, 13, 24, 1, -1, 0, 0.0)]
# round 4: BG2 and Z < 384 through every class of the packed runtime-Z kernel (1, 2, 3 waves per codeblock),
# shortened, with CRC early stop and filler bits
CASES += [("avx2", 2, 52, None, 6, 3, 0, 7.5), ("generic", 2, 144, 30, 6, 1, 40, 7.0),
          ("avx2", 2, 256, 20, 5, 0, 0, 6.5), ("avx2", 1, 120, None, 6, 1, 0, 8.0),
          ("generic", 1, 224, 40, 6, 0, 96, 8.0), ("avx2", 1, 320, 30, 8, 1, 0, 7.0),
          ("avx2", 1, 352, 26, 6, 1, 64, 6.0), ("generic", 2, 320, 14, 4, 3, 0, 5.0)]


def main():
    rng = np.random.default_rng(20251128)
    out = {}
    for n, (impl, bg, Z, Ln, iters, crc, filler, noise) in enumerate(CASES):
        K = oracle.BG_K[bg] * Z
        N = oracle.BG_N_SHORT[bg] * Z
        L = N if Ln is None else Ln * Z
        m = rng.integers(0, 2, K).astype(np.uint8)
        if filler:
            m[K - filler:] = 0
        if crc >= 0:
            Lc = 24 if crc in (0, 1, 2) else 16
            c = oracle.REF.srs_ref_crc_bits(crc, m[: K - filler - Lc].ctypes.data_as(oracle.P), K - filler - Lc)
            m[K - filler - Lc: K - filler] = [(c >> (Lc - 1 - b)) & 1 for b in range(Lc)]
        cw = oracle.ref_ldpc_encode(m, bg, Z, N)
        x = (1 - 2 * cw[:L].astype(np.float64)) * 10 + rng.normal(0, noise, L) if noise else (1 - 2 * cw[:L]) * 10.0
        llr = np.clip(np.round(x), -120, 120).astype(np.int8)
        r, bits = oracle.ref_ldpc_decode(impl, llr, bg, Z, iters, crc_poly=None if crc < 0 else crc,
                                         nof_filler_bits=filler, nof_crc_bits=24 if crc in (0, 1, 2) else 16)
        key = "c%02d" % n
        out[key + "_cfg"] = np.array([bg, Z, iters, crc, filler, 0 if impl != "generic" else 1], np.int32)
        out[key + "_msg"] = np.packbits(m)
        out[key + "_cw"] = np.packbits(cw)
        out[key + "_llr"] = llr
        out[key + "_out"] = bits
        out[key + "_iters"] = np.array([-1 if r is None else r], np.int32)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ldpc_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(CASES), "cases", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

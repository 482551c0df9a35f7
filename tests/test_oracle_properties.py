"""Oracle self-checks that need neither the GPU nor the reference build."""
import numpy as np

import oracle


def test_encoder_output_satisfies_parity_checks():
    rng = np.random.default_rng(7)
    for bg in (1, 2):
        for Z in (2, 3, 10, 36, 384):
            K = oracle.BG_K[bg] * Z
            m = rng.integers(0, 2, K).astype(np.uint8)
            cw = oracle.ldpc_encode(m, bg, Z)
            full = np.concatenate([m[: 2 * Z], cw])
            assert oracle.ORACLE.srs_oracle_ldpc_syndrome(bg, Z, full.ctypes.data_as(oracle.P)) == 0
            np.testing.assert_array_equal(cw[: K - 2 * Z], m[2 * Z:])  # systematic


def test_crc_of_message_with_crc_is_zero():
    rng = np.random.default_rng(1)
    for poly, L in ((0, 24), (1, 24), (2, 24), (3, 16), (4, 11), (5, 6)):
        m = rng.integers(0, 2, 500).astype(np.uint8)
        c = oracle.crc_bits(poly, m)
        tail = np.array([(c >> (L - 1 - b)) & 1 for b in range(L)], np.uint8)
        assert oracle.crc_bits(poly, np.concatenate([m, tail])) == 0


def test_lifting_index_table():
    # TS 38.212 Table 5.3.2-1
    sets = {0: [2, 4, 8, 16, 32, 64, 128, 256], 1: [3, 6, 12, 24, 48, 96, 192, 384], 2: [5, 10, 20, 40, 80, 160, 320],
            3: [7, 14, 28, 56, 112, 224], 4: [9, 18, 36, 72, 144, 288], 5: [11, 22, 44, 88, 176, 352],
            6: [13, 26, 52, 104, 208], 7: [15, 30, 60, 120, 240]}
    for ils, zs in sets.items():
        for z in zs:
            assert oracle.ORACLE.srs_oracle_lifting_index(z) == ils
    assert oracle.ORACLE.srs_oracle_lifting_index(17) == -1


def test_zero_llrs_give_all_ones():
    for bg in (1, 2):
        Z = 8
        llrs = np.zeros(oracle.BG_N_SHORT[bg] * Z, np.int8)
        r, out, _ = oracle.ldpc_decode(llrs, bg, Z, 1)
        assert r is None
        assert (oracle.unpack_bits(out, oracle.BG_K[bg] * Z) == 1).all()


def test_mimo_equalizer_oracle_reduces_to_pinned_zf():
    """oracle.equalizer.equalize_mimo (fp64, parity unpinned for L >= 3 / MMSE L >= 2) agrees with the pinned
    reference restatement where the topologies overlap: ZF with one and two layers, MMSE with one layer (which
    the reference evaluates with its ZF equalizer)."""
    from oracle import equalizer as E

    rng = np.random.default_rng(4)
    for ports, layers in ((1, 1), (2, 1), (4, 1), (2, 2), (4, 2)):
        s, h, nv, _ = E.random_channel(rng, 500, ports, layers, 12.0)
        want, wantn = E.equalize(s, h, nv, 0.7, layers)
        for algo in (("zf", "mmse") if layers == 1 else ("zf",)):
            got, gotn, _ = E.equalize_mimo(s, h, nv, 0.7, layers, algo)
            if layers == 1:  # the 1-layer reference weights ports by their own noise variances; equal here
                assert np.allclose(got, want, rtol=1e-9, atol=1e-12)
                assert np.allclose(gotn, wantn, rtol=1e-9)
            else:
                assert np.allclose(got, want, rtol=1e-9, atol=1e-12)
                assert np.allclose(gotn, wantn, rtol=1e-9)


def test_mimo_equalizer_oracle_mmse_is_unbiased():
    """Unbiased MMSE: with noise-free observations the estimate equals the transmitted symbols scaled back, and
    the MMSE variance never exceeds the ZF one."""
    from oracle import equalizer as E

    rng = np.random.default_rng(8)
    s, h, nv, x = E.random_channel(rng, 300, 4, 4, 60.0)
    zf, zfn, _ = E.equalize_mimo(s, h, nv, 1.0, 4, "zf")
    mm, mmn, _ = E.equalize_mimo(s, h, nv, 1.0, 4, "mmse")
    assert np.all(mmn <= zfn * (1 + 1e-9))
    assert np.median(np.abs(mm - x)) < 0.02

"""Pins the CPU oracle (oracle/srs_oracle.c) to the reference itself.

oracle/_ref/libsrsran_ref.so is compiled from /root/reference's own LDPC/CRC
sources (oracle/Makefile); the reference's .dat test vectors are not shipped,
so this is the pin: the oracle must reproduce the reference decoders
(generic, AVX2, AVX512) bit-for-bit, the reference encoder and CRCs.
"""
import numpy as np
import pytest

import oracle
from tests.ldpc_cases import noisy_codeblocks

pytestmark = pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref/libsrsran_ref.so not built")

IMPLS = [("generic", "generic"), ("avx2", "simd"), ("avx512", "simd")]


def _impls():
    return [(i, a) for i, a in IMPLS if oracle.REF.srs_ref_has_impl(i.encode())]


@pytest.mark.parametrize("bg", [1, 2])
def test_encoder_matches_reference(bg):
    rng = np.random.default_rng(bg)
    for Z in (2, 3, 5, 6, 7, 9, 11, 13, 15, 22, 36, 60, 104, 176, 208, 240, 352, 384):
        K = oracle.BG_K[bg] * Z
        m = rng.integers(0, 2, K).astype(np.uint8)
        np.testing.assert_array_equal(oracle.ldpc_encode(m, bg, Z), oracle.ref_ldpc_encode(m, bg, Z),
                                      err_msg="bg%d Z%d" % (bg, Z))


@pytest.mark.parametrize("bg", [1, 2])
def test_decoder_matches_reference(bg):
    for impl, arith in _impls():
        for Z in (2, 5, 14, 40, 112, 384):
            for noise in (4.0, 10.0):
                msgs, llrs = noisy_codeblocks(bg, Z, 2, noise=noise, seed=Z + int(noise))
                for i in range(2):
                    for iters in (1, 5):
                        r1, o1 = oracle.ref_ldpc_decode(impl, llrs[i], bg, Z, iters)
                        r2, o2, _ = oracle.ldpc_decode(llrs[i], bg, Z, iters, arith)
                        assert r1 == r2
                        np.testing.assert_array_equal(o1, o2, err_msg="%s bg%d Z%d" % (impl, bg, Z))


def test_decoder_crc_early_stop_matches_reference():
    for impl, arith in _impls():
        for bg, Z, poly in ((1, 384, 1), (1, 52, 0), (2, 16, 3)):
            msgs, llrs = noisy_codeblocks(bg, Z, 3, noise=10.0, seed=Z, crc_poly=poly)
            nb = 24 if poly in (0, 1) else 16
            for i in range(3):
                r1, o1 = oracle.ref_ldpc_decode(impl, llrs[i], bg, Z, 10, crc_poly=poly, nof_crc_bits=nb)
                r2, o2, _ = oracle.ldpc_decode(llrs[i], bg, Z, 10, arith, crc_poly=poly, nof_crc_bits=nb)
                assert r1 == r2, (impl, bg, Z, i)
                np.testing.assert_array_equal(o1, o2)


def test_decoder_shortened_filler_and_force():
    for impl, arith in _impls():
        bg, Z = 1, 64
        msgs, llrs = noisy_codeblocks(bg, Z, 1, noise=6.0, seed=3)
        for L in (24 * Z, 38 * Z, 52 * Z, 66 * Z, 30 * Z + 7):
            r1, o1 = oracle.ref_ldpc_decode(impl, llrs[0, :L], bg, Z, 4, crc_poly=0, nof_filler_bits=40,
                                            nof_crc_bits=24)
            r2, o2, _ = oracle.ldpc_decode(llrs[0, :L], bg, Z, 4, arith, crc_poly=0, nof_filler_bits=40,
                                           nof_crc_bits=24)
            assert r1 == r2
            np.testing.assert_array_equal(o1, o2)
        short = np.zeros(66 * Z, np.int8)
        short[:100] = 9
        r1, o1 = oracle.ref_ldpc_decode(impl, short, bg, Z, 2, force_decoding=True)
        r2, o2, _ = oracle.ldpc_decode(short, bg, Z, 2, arith, force_decoding=True)
        assert r1 == r2 is None
        np.testing.assert_array_equal(o1, o2)


def test_crc_matches_reference():
    rng = np.random.default_rng(0)
    for poly in range(6):
        for n in (0, 1, 7, 8, 100, 3823, 8424):
            bits = rng.integers(0, 2, n).astype(np.uint8)
            ref = oracle.REF.srs_ref_crc_bits(poly, bits.ctypes.data_as(oracle.P), n)
            assert oracle.crc_bits(poly, bits) == ref, (poly, n)


def _rm_cases(rng):
    """(bg, Z, F, rv, Qm, Nref, E) covering filler, LBRM, every rv/Qm, E < / > Ncb."""
    for bg in (1, 2):
        for Z in (2, 7, 52, 384):
            N = oracle.BG_N_SHORT[bg] * Z
            for F in (0, 5, Z):
                for rv in range(4):
                    for Qm in (1, 2, 4, 6, 8):
                        for Nref in (0, (N * 2) // 3):
                            for E in (Qm * 3, Qm * ((N // Qm) // 2), Qm * ((5 * N // 2) // Qm)):
                                yield bg, Z, F, rv, Qm, Nref, E


def test_rate_matcher_matches_reference():
    rng = np.random.default_rng(11)
    for bg, Z, F, rv, Qm, Nref, E in _rm_cases(rng):
        K = oracle.BG_K[bg] * Z
        m = rng.integers(0, 2, K).astype(np.uint8)
        m[K - F:K] = 0
        cw = oracle.ldpc_encode(m, bg, Z)
        np.testing.assert_array_equal(oracle.rate_match(cw, bg, Z, rv, Qm, E, Nref, F),
                                      oracle.ref_encode_rate_match(m, bg, Z, rv, Qm, E, Nref, F),
                                      err_msg=str((bg, Z, F, rv, Qm, Nref, E)))


@pytest.mark.parametrize("impl", ["generic", "avx2", "avx512"])
def test_rate_dematcher_matches_reference(impl):
    rng = np.random.default_rng(12)
    probe = np.zeros(66 * 2, np.int8)
    try:
        oracle.ref_rate_dematch(np.zeros(2, np.int8), 1, 2, 0, 2, probe, impl=impl)
    except ValueError:
        pytest.skip("%s dematcher not supported on this host" % impl)
    # The SIMD dematchers combine with a clamped saturating byte add
    # (ldpc_rate_dematcher_avx2_impl.cpp:49), the generic one with the LLR sum's
    # infinity rules (log_likelihood_ratio.cpp:38); they agree on finite LLRs,
    # which is all a PUSCH soft buffer ever combines (demodulator output is
    # within +-LLR_MAX and the +inf filler positions are never combined).
    # The oracle follows generic, so infinities are exercised against it only.
    lim = 127 if impl == "generic" else 120
    corners = np.array([-127, -121, -120, -119, -1, 0, 1, 60, 119, 120, 121, 127], np.int8)
    corners = corners[np.abs(corners.astype(int)) <= lim]
    for bg, Z, F, rv, Qm, Nref, E in _rm_cases(rng):
        N = oracle.BG_N_SHORT[bg] * Z
        llr = rng.choice(corners, E)
        llr[::3] = rng.integers(-120, 121, len(llr[::3]))
        for new_data in (True, False):
            init = rng.integers(-lim, lim + 1, N).astype(np.int8)
            a, b = init.copy(), init.copy()
            oracle.rate_dematch(llr, bg, Z, rv, Qm, a, new_data, Nref, F)
            oracle.ref_rate_dematch(llr, bg, Z, rv, Qm, b, new_data, Nref, F, impl=impl)
            np.testing.assert_array_equal(a, b, err_msg=str((impl, bg, Z, F, rv, Qm, Nref, E, new_data)))


# --- OFDM (oracle/ofdm.py vs the reference modulator / demodulator / generic DFT) ---

# ofdm_modulator_test_data.h / ofdm_demodulator_test_data.h configurations
# {numerology, bw_rb, dft_size, cp, scale, center_freq_Hz}, port, slot (the .dat
# vectors themselves are not shipped; grids are synthetic).
OFDM_CASES = [
    (0, 12, 256, False, 0.81158, 2740100000, 0), (0, 96, 2048, False, 0.93184, 97900000, 0),
    (0, 192, 4096, False, 0.87523, 1424700000, 0), (1, 24, 512, False, -0.47474, 293200000, 0),
    (1, 48, 1024, False, 0.27046, 1607000000, 1), (1, 192, 4096, False, -0.54681, 619800000, 1),
    (2, 12, 256, True, 0.73538, 837900000, 2), (2, 48, 1024, False, -0.14768, 2527000000, 3),
    (2, 96, 2048, True, -0.93258, 2059300000, 3), (3, 192, 4096, False, 0.73052, 2633100000, 6),
    (1, 273, 4096, False, 1.0, 3500000000, 0), (1, 106, 1536, False, 0.5, 1800000000, 1),
]


def test_dft_matches_reference():
    """Float tolerance: max |ref - exact| <= 1e-5 * rms (the reference's float32 DFT)."""
    rng = np.random.default_rng(21)
    for N in (12, 128, 256, 512, 1024, 1536, 2048, 3072, 4096):
        x = (rng.normal(size=N) + 1j * rng.normal(size=N)).astype(np.complex64)
        for inv in (False, True):
            r = oracle.ref_dft(x, inv)
            e = np.fft.ifft(x.astype(complex)) * N if inv else np.fft.fft(x.astype(complex))
            assert np.max(np.abs(r - e)) <= 1e-5 * np.sqrt(np.mean(np.abs(e) ** 2)), (N, inv)


@pytest.mark.parametrize("case", OFDM_CASES)
def test_ofdm_matches_reference(case):
    from oracle import ofdm

    mu, bw, N, ext, scale, fc, slot = case
    rng = np.random.default_rng(N + bw)
    g = ofdm.random_grid(rng, 12 if ext else 14, bw * 12)
    r = oracle.ref_ofdm_modulate_slot(g, slot, mu, bw, N, scale, fc, ext)
    o = ofdm.modulate_slot(g, slot, mu, bw, N, scale, fc, ext)
    assert r.size == o.size == ofdm.slot_size(slot, mu, N, ext)
    # modulator: float tolerance 1e-5 x RMS of the symbol stream
    assert np.max(np.abs(r - o)) <= 1e-5 * np.sqrt(np.mean(np.abs(o) ** 2))
    # received signal: the modulated slot plus noise (a pure round trip of a bf16
    # grid can land exactly on bf16 rounding ties)
    rx = (r + (rng.normal(0, 0.05, r.size) + 1j * rng.normal(0, 0.05, r.size)) * np.sqrt(np.mean(np.abs(r) ** 2)))
    rx = rx.astype(np.complex64)
    for off in (0, 5):
        rg = oracle.ref_ofdm_demodulate_slot(rx, slot, mu, bw, N, scale, fc, off, ext)
        og = ofdm.demodulate_slot(rx, slot, mu, bw, N, scale, fc, off, ext)
        # demodulator: bf16 grid; equal except values straddling a bf16 rounding
        # boundary, which may differ by one bf16 ulp
        diff = np.abs(rg.astype(np.int32) - og.astype(np.int32))
        assert diff.max() <= 1 and np.mean(diff != 0) < 1e-3, (off, diff.max(), np.mean(diff != 0))


# --- channel equalizer (oracle/equalizer.py vs channel_equalizer_generic_impl) ---

@pytest.mark.parametrize("ports,layers", [(1, 1), (2, 1), (4, 1), (2, 2), (4, 2)])
def test_equalizer_matches_reference(ports, layers):
    """The reference's AVX2 path uses an approximate reciprocal (_mm256_rcp_ps,
    relative error <= 1.5 * 2^-12): tolerance 1e-3 relative on symbols, 2e-3 on
    variances (squared reciprocal)."""
    from oracle import equalizer as E

    rng = np.random.default_rng(ports * 10 + layers)
    for nre, tx in ((1, 1.0), (37, 0.5), (3276, 1.0)):
        s, h, nv, _ = E.random_channel(rng, nre, ports, layers)
        for mmse in (False, True):
            if not E.is_supported("mmse" if mmse else "zf", ports, layers):
                continue
            a, an = oracle.ref_equalize(s, h, nv, tx, layers, mmse)
            b, bn = E.equalize(s, h, nv, tx, layers)
            assert np.all(np.abs(a - b) <= 1e-3 * np.abs(b) + 1e-6), (ports, layers, nre)
            assert np.all(np.abs(an - bn) <= 2e-3 * bn), (ports, layers, nre)


def test_equalizer_invalid_noise_matches_reference():
    from oracle import equalizer as E

    rng = np.random.default_rng(5)
    s, h, nv, _ = E.random_channel(rng, 100, 4, 1)
    for bad in ([0.0, 0.01, 0.01, 0.01], [np.inf, 0.01, -1.0, 0.02], [0.0, 0.0, 0.0, 0.0]):
        nvb = np.array(bad, np.float32)
        a, an = oracle.ref_equalize(s, h, nvb, 1.0, 1)
        b, bn = E.equalize(s, h, nvb, 1.0, 1)
        assert np.all(np.abs(a - b) <= 1e-3 * np.abs(b) + 1e-6)
        assert np.all((np.isinf(an) & np.isinf(bn)) | (np.abs(an - bn) <= 2e-3 * bn))


# --- polar codes (oracle/srs_oracle_polar.c vs the reference's polar classes) ---

def polar_cases():
    """(K, E, nMax): DCI sizes (nMax 9, PDCCH aggregation levels 1-16 -> E = 108 * L)
    and UCI sizes (nMax 10, with and without parity-check bits), covering
    repetition (E >= N), puncturing and shortening."""
    cases = []
    for K in (36, 41, 57, 80, 100, 140, 164):
        for L in (1, 2, 4, 8, 16):
            if 108 * L > K:
                cases.append((K, 108 * L, 9))
    for K in (18, 19, 22, 25, 31, 40, 64, 130, 300, 500, 1000):
        for E in (K + 7, int(K * 1.7), 2 * K + 60, K + 220, 1200, 3000, 8192):
            if K + (3 if K <= 25 else 0) < E <= 8192:
                cases.append((K, E, 10))
    return sorted(set(cases))


def test_polar_code_construction_matches_reference():
    for K, E, nMax in polar_cases():
        try:
            want = oracle.ref_polar_code(K, E, nMax)
        except Exception:
            continue
        got = oracle.polar_code(K, E, nMax)
        assert got[0] == want[0] and np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2]), (K, E)


def test_polar_chains_match_reference():
    rng = np.random.default_rng(33)
    for K, E, nMax in polar_cases():
        for ibil in (False, True):
            m = rng.integers(0, 2, K).astype(np.uint8)
            cw = oracle.polar_encode_chain(m, E, nMax, ibil)
            np.testing.assert_array_equal(cw, oracle.ref_polar_encode_chain(m, E, nMax, ibil), err_msg=str((K, E)))
            llr = np.clip(np.round((1 - 2.0 * cw) * 5 + rng.normal(0, 7, E)), -120, 120).astype(np.int8)
            llr[rng.random(E) < 0.03] = 127
            llr[rng.random(E) < 0.03] = -127
            np.testing.assert_array_equal(oracle.polar_decode_chain(llr, K, nMax, ibil),
                                          oracle.ref_polar_decode_chain(llr, K, nMax, ibil), err_msg=str((K, E)))


def test_polar_interleaver_matches_reference():
    rng = np.random.default_rng(2)
    for K in (1, 12, 40, 100, 164):
        b = rng.integers(0, 2, K).astype(np.uint8)
        for d in (0, 1):
            np.testing.assert_array_equal(oracle.polar_interleave(b, d), oracle.polar_interleave(b, d, lib=oracle.REF))


# --- modulation mapper, soft demodulation mapper, Gold sequence ---

@pytest.mark.parametrize("qm", [0, 1, 2, 4, 6, 8])
def test_modulation_and_demodulation_match_reference(qm):
    """Modulation: bit-exact symbols.  Soft demodulation: bit-exact int8 LLRs
    against an x86-64-v3 build of the reference (AVX2 blocks + scalar tail),
    including zero / NaN-free invalid noise variances."""
    rng = np.random.default_rng(qm + 100)
    bps = 1 if qm < 2 else qm
    for nsym in (1, 3, 4, 7, 8, 15, 16, 17, 100, 3276):
        bits = rng.integers(0, 256, (nsym * bps + 7) // 8).astype(np.uint8)
        a = oracle.modulate(bits, nsym, qm)
        np.testing.assert_array_equal(a.view(np.uint32), oracle.ref_modulate(bits, nsym, qm).view(np.uint32))
        sym = (a + (rng.normal(size=nsym) + 1j * rng.normal(size=nsym)) * 0.4).astype(np.complex64)
        sym[rng.random(nsym) < 0.02] = 0
        nv = rng.uniform(0.005, 2.0, nsym).astype(np.float32)
        nv[rng.random(nsym) < 0.03] = 0.0
        nv[rng.random(nsym) < 0.02] = -1.0
        np.testing.assert_array_equal(oracle.demodulate(sym, nv, qm), oracle.ref_demodulate(sym, nv, qm),
                                      err_msg="qm %d nsym %d" % (qm, nsym))


def test_gold_sequence_matches_reference():
    for ci in (0, 1, 0x1234567, 2 ** 31 - 1):
        for n in (1, 31, 32, 1000, 100003):
            np.testing.assert_array_equal(oracle.prbs(ci, n), oracle.ref_prbs(ci, n))


# --- PDSCH encoder / PUSCH decoder (transport-block chain) ---

def test_sch_pdsch_encode_matches_reference():
    """oracle.sch.pdsch_encode == pdsch_encoder_impl (segmenter + AVX2 LDPC encoder + rate matcher), bit-exact."""
    import oracle.sch as sch
    from tests.sch_cases import SCH_CASES, tb_bytes

    for i, (tbs, bg, qm, lay, nre, rv, nref) in enumerate(SCH_CASES):
        p = sch.plan(tbs, bg, rv, qm, nref, lay, nre)
        tb = tb_bytes(tbs, i)
        np.testing.assert_array_equal(sch.pdsch_encode(tb, p), oracle.ref_pdsch_encode(tb, p), err_msg=str(p))


@pytest.mark.parametrize("arith", ["simd", "generic"])
def test_sch_pusch_decode_matches_reference(arith):
    """oracle.sch.pusch_decode == pusch_decoder_impl: TB bytes, TB CRC status and LDPC
    statistics, with and without early stop, and a two-transmission HARQ sequence
    (rv 0 too noisy to decode, rv 2 combined in the soft buffer)."""
    import oracle.sch as sch
    from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes

    for i, (tbs, bg, qm, lay, nre, rv, nref) in enumerate(SCH_CASES[:6]):
        p = sch.plan(tbs, bg, rv, qm, nref, lay, nre)
        tb = tb_bytes(tbs, i)
        cw = sch.pdsch_encode(tb, p)
        for early in (True, False):
            llr = noisy_llrs(cw, 10, 9, seed=i)
            h = sch.HarqBuffer(p)
            out = np.zeros(tbs // 8, np.uint8)
            ok, _, stats = sch.pusch_decode(llr, p, h, out, 6, arith, use_early_stop=early)
            rb = oracle.RefRxBuffer(p["nof_segments"])
            out2 = np.zeros(tbs // 8, np.uint8)
            r = oracle.ref_pusch_decode(llr, p, rb, out2, 6, arith == "generic", use_early_stop=early)
            assert r[0] == ok and r[1] == p["nof_segments"], (p, r, ok)
            assert (r[3], r[4], r[5]) == (sum(stats), min(stats), max(stats)), (r, stats)
            np.testing.assert_array_equal(out, out2)
    # HARQ: first transmission undecodable, the second (rv 2) combined.
    tbs, bg, qm, lay, nre = 8 * 1056, 1, 2, 1, 6000
    p0 = sch.plan(tbs, bg, 0, qm, 0, lay, nre)
    p2 = sch.plan(tbs, bg, 2, qm, 0, lay, nre)
    tb = tb_bytes(tbs, 99)
    h = sch.HarqBuffer(p0)
    rb = oracle.RefRxBuffer(p0["nof_segments"])
    out, out2 = np.zeros(tbs // 8, np.uint8), np.zeros(tbs // 8, np.uint8)
    for p, new, sigma in ((p0, True, 9), (p2, False, 5)):
        llr = noisy_llrs(sch.pdsch_encode(tb, p), 8, sigma, seed=p["rv"])
        ok, _, _ = sch.pusch_decode(llr, p, h, out, 6, arith, new_data=new)
        r = oracle.ref_pusch_decode(llr, p, rb, out2, 6, arith == "generic", new_data=new)
        assert r[0] == ok
        np.testing.assert_array_equal(out, out2)
    assert ok, "HARQ combining should recover the TB"


# ---- PDSCH modulator / DM-RS (oracle/pdsch_mod.py vs the reference's classes) ----
from tests.pdsch_cases import DMRS_CASES, MOD_CASES, dmrs_case, mod_case  # noqa: E402


@pytest.mark.parametrize("case", MOD_CASES, ids=[c[0] for c in MOD_CASES])
@pytest.mark.parametrize("precoder", ["generic", "avx2", "avx512"])
def test_pdsch_modulator_matches_reference(case, precoder):
    from oracle import pdsch_mod as pm

    grid0, bits, kw = mod_case(case)
    want = pm.ref_pdsch_modulate(grid0.copy(), bits, precoder=precoder, **kw)
    got = pm.pdsch_modulate(grid0.copy(), bits, **kw)
    np.testing.assert_array_equal(got, want)
    assert (want != grid0).any()


@pytest.mark.parametrize("case", DMRS_CASES, ids=[c[0] for c in DMRS_CASES])
@pytest.mark.parametrize("precoder", ["generic", "avx2", "avx512"])
def test_dmrs_pdsch_matches_reference(case, precoder):
    from oracle import pdsch_mod as pm

    grid0, kw = dmrs_case(case)
    want = pm.ref_dmrs_pdsch_map(grid0.copy(), precoder=precoder, **kw)
    got = pm.dmrs_pdsch_map(grid0.copy(), **kw)
    np.testing.assert_array_equal(got, want)


# ---- PUSCH DM-RS channel estimator (oracle/chest.py vs the reference's classes) ----
from tests import chest_cases  # noqa: E402


@pytest.mark.parametrize("case", chest_cases.CASES, ids=[c[0] for c in chest_cases.CASES])
def test_pusch_chest_matches_reference(case):
    from oracle import chest

    grid, kw = chest_cases.case_args(case, seed=1)
    est0 = chest_cases.stale_estimates(grid.shape, kw["nof_layers"])
    want, ws = chest.ref_pusch_chest(grid, estimates=est0, **kw)
    got, gs = chest.pusch_chest(grid, estimates=est0, **kw)
    chest_cases.assert_estimates_close(got, want, case[0])
    chest_cases.assert_stats_close(gs, ws, case[0])


@pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("case_idx", range(10))
def test_pusch_demodulator_matches_reference(case_idx):
    """The restated PUSCH demodulator tail (one demapper call per OFDM symbol, descrambling) on the
    reference equalizer's per-symbol output reproduces pusch_demodulator_impl bit-exactly; the
    float64-equalizer restatement is within one LLR step."""
    from oracle import pusch_demod as od
    from tests.pusch_demod_cases import CASES, assert_llrs_close, demod_args, dyadic_equalized, make_case

    case = CASES[case_idx]
    name, P, L, nprb, _, qm, start, nsym, dmrs, ncdm = case
    grid, est, nv, crbs = make_case(case, 7, "random")
    want = od.ref_pusch_demodulate(grid, est, nv, 0x4601, 17, crbs=crbs, **demod_args(case))
    a = dict(demod_args(case))
    a.pop("qm")
    eq, env = od.ref_equalize_per_symbol(grid, est, nv, crbs, **a)
    counts = od.data_re_mask(12 * nprb, crbs, start, nsym, dmrs, False, ncdm).sum(axis=1) * L
    got = od.demap_descramble_per_symbol(eq, env, counts, qm, 0x4601 * (1 << 15) + 17)
    assert np.array_equal(got, want), name
    assert_llrs_close(od.pusch_demodulate(grid, est, nv, 0x4601, 17, crbs=crbs, **demod_args(case)), want, name,
                      0.97)
    # demapper ties: restated per-symbol demapping == the reference demapper per symbol
    if qm >= 4:
        deq, dnv = dyadic_equalized(qm, int(counts.sum()), 3, oracle.ref_demodulate)
        ref = od.demap_descramble_per_symbol(deq, dnv, counts, qm, 99, demod=oracle.ref_demodulate)
        assert np.array_equal(od.demap_descramble_per_symbol(deq, dnv, counts, qm, 99), ref), name


def _pdcch_cases():
    from tests import pdcch_cases

    return pdcch_cases.cases()


@pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("idx", range(10))
def test_pdcch_matches_reference(idx):
    """The restated PDCCH processor (oracle/pdcch.py) writes the same grid as the compiled pdcch_processor_impl, and
    its CRB lists equal cce_to_prb_mapping's (order included); the C-ABI's host-only rb_mask (the validator and the
    CCE-to-PRB mapping of pdcch_api.cpp) gives the same CRB set."""
    from oracle import pdcch as op
    from srsran_project_amd.pdcch import rb_mask

    name, pdu = _pdcch_cases()[idx]
    assert op.crbs(pdu) == op.ref_crbs(pdu), name
    assert list(rb_mask(pdu)) == sorted(set(op.ref_crbs(pdu))), name
    c = pdu.coreset
    nsubc = 12 * (c.bwp_start_rb + c.bwp_size_rb)
    g0 = np.random.default_rng(idx).integers(0, 2**32, (pdu.dci.nof_ports, 14, nsubc), dtype=np.uint64)
    g0 = g0.astype(np.uint32)
    want = op.ref_process(g0.copy(), [pdu])
    assert (want != g0).sum() == 12 * len(op.ref_crbs(pdu)) * c.duration * pdu.dci.nof_ports, name
    assert np.array_equal(op.process(g0.copy(), pdu), want), name


@pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")
def test_pdcch_invalid_pdus_rejected_like_reference():
    """The C-ABI validator rejects what pdcch_processor_validator_impl rejects, with the same message."""
    from oracle import pdcch as op
    from srsran_project_amd.pdcch import make_pdu, rb_mask
    from tests.pdcch_cases import INVALID

    for name, kw, text in INVALID:
        pdu = make_pdu(np.ones(20, np.uint8), **kw)
        with pytest.raises(ValueError, match=text):
            op.ref_process(np.zeros((1, 14, 12 * 52), np.uint32), [pdu])
        with pytest.raises(ValueError, match=text):
            rb_mask(pdu)


@pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")
def test_reference_pdsch_multi_prg_precoding_is_out_of_bounds():
    """Why the PDSCH plug-in rejects precoding that differs between PRGs (integration/pdsch_processor_hip.h): the
    reference's pdsch_processor_impl, run on such a PDU, dies in its DM-RS processor (dmrs_pdsch_processor_impl.cpp:
    150-160 writes the weights of PRG >= 1 into a one-PRG precoding_configuration), while the same PDU with one PRG
    runs.  Each run in its own process (CPU only: the harness's PDSCH path does not touch the GPU)."""
    import os
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent("""
        import sys
        sys.path[:0] = [%r, %r]
        from pdsch_slot_cases import MULTI_PRG_PDU, slot
        from oracle import phy as ophy
        case = MULTI_PRG_PDU if sys.argv[1] == "multi" else MULTI_PRG_PDU[:12] + (None,)
        (pdu, tb), = slot(seed=3, pdus=[case])[0]
        ophy.ref_pdsch_process(ophy.WriterGrid(slot(seed=3, pdus=[case])[1]), pdu, tb)
        print("done")
    """ % (root, os.path.join(root, "tests")))
    one = subprocess.run([sys.executable, "-c", code, "one"], capture_output=True, text=True, timeout=300)
    assert one.returncode == 0 and "done" in one.stdout, one.stderr[-2000:]
    multi = subprocess.run([sys.executable, "-c", code, "multi"], capture_output=True, text=True, timeout=300)
    assert multi.returncode != 0 and "done" not in multi.stdout, (multi.returncode, multi.stdout)


# ---- SS/PBCH block -------------------------------------------------------------------------------------------------
from tests import ssb_cases  # noqa: E402


@pytest.mark.parametrize("case", ssb_cases.CASES, ids=[c[0] for c in ssb_cases.CASES])
def test_ssb_restatement_matches_reference(case):
    """oracle/ssb.py (numpy) equals the compiled ssb_processor_impl bit for bit, and the C-ABI's block position equals
    ssb_get_l_first / ssb_get_k_first."""
    import srsran_project_amd as amd
    from oracle import ssb as oss

    p = ssb_cases.pdu(case, seed=3)
    g0 = ssb_cases.grid0(seed=4)
    want = oss.ref_process(g0.copy(), [p])
    got = oss.process(g0.copy(), p)
    assert np.array_equal(got, want), "%d REs differ" % int((got != want).sum())
    assert amd.ssb.position(p) == oss.ref_position(p)


def test_ssb_invalid_pdus_rejected():
    """PDUs the reference asserts on (wrong slot, non-integer subcarrier, FR2 SCS / k_SSB limits, SSB index beyond
    the pattern) are rejected by the C-ABI's host checks (no GPU call)."""
    import srsran_project_amd as amd

    for c in ssb_cases.INVALID:
        with pytest.raises(ValueError):
            amd.ssb.position(ssb_cases.pdu(c))


# ---- PUCCH Format 0 ------------------------------------------------------------------------------------------------
def test_pucch_f0_restatement_matches_reference():
    """oracle/pucch.py gives the compiled pucch_detector_format0's message bits and status on every case, and its
    metric / CSI within float tolerance (the restated cyclic shift is a double-precision exponential, the reference's
    a float table: 1e-3 relative / 0.01 dB)."""
    from oracle import pucch as op
    from tests.pucch_cases import cases

    for i, (pdu, grid, sent) in enumerate(cases()):
        st, sr, harq, metric, sinr, rsrp, epre = op.detect(grid, pdu)
        r = op.ref_detect(grid, pdu)
        assert r.status == st, (i, r.status, st, metric)
        assert list(r.harq_ack)[:r.nof_harq_ack] == list(harq), i
        assert ([r.sr] if r.nof_sr else []) == list(sr), i
        np.testing.assert_allclose(r.detection_metric, metric, rtol=1e-3, err_msg=str(i))
        for a, b in ((r.sinr_dB, sinr), (r.rsrp_dB, rsrp), (r.epre_dB, epre)):
            assert abs(a - b) <= 0.01, (i, a, b)


def test_pucch_f1_restatement_matches_reference():
    """oracle/pucch.py detect_f1 gives the compiled pucch_detector_format1's status and HARQ-ACK bits for every
    multiplexed PUCCH of every batch, and its normalised metric / CSI within 1e-3 relative / 0.01 dB."""
    from oracle import pucch as op
    from tests.pucch_cases import f1_cases

    for i, (b, grid, sent) in enumerate(f1_cases()):
        ref = op.ref_detect_f1(grid, b)
        mine = op.detect_f1(grid, b, [(e.initial_cyclic_shift, e.time_domain_occ, e.nof_harq_ack)
                                      for e in b._entries[:b.nof_entries]])
        for j, (r, (st, bits, metric, sinr, rsrp, epre)) in enumerate(zip(ref, mine)):
            assert r.status == st, (i, j, r.status, st, metric)
            assert list(r.harq_ack)[:r.nof_harq_ack] == bits, (i, j)
            np.testing.assert_allclose(r.detection_metric, metric, rtol=1e-3, err_msg=str((i, j)))
            for a, c in ((r.sinr_dB, sinr), (r.rsrp_dB, rsrp), (r.epre_dB, epre)):
                assert abs(a - c) <= 0.01, (i, j, a, c)


def test_pucch_f2_transmitter_decoded_by_reference():
    """tests/pucch_cases.py's Format 2 transmitter (UCI encoding, scrambling, DM-RS) is the reference receiver's
    convention: at the highest SNR of the cases the compiled pucch_processor_impl returns the payload, valid."""
    from oracle import pucch as op
    from tests.pucch_cases import f2_cases

    n = 0
    for i, (pdu, grid, payload) in enumerate(f2_cases(n=12, seed=5)):
        if i % 4 != 0:
            continue
        r, pay = op.ref_process_f2(grid, pdu)
        assert r.status == 1 and np.array_equal(pay, payload), i
        n += 1
    assert n == 3


def test_pucch_f34_transmitter_decoded_by_reference():
    """tests/pucch_cases.py's Format 3 / 4 transmitter (UCI encoding, scrambling, pi/2-BPSK / QPSK, OCC spreading,
    transform precoding, low-PAPR DM-RS) is the reference receiver's convention: at the highest SNR of the cases the
    compiled pucch_processor_impl returns the payload, valid."""
    from oracle import pucch as op
    from tests.pucch_cases import f34_cases

    n = 0
    for i, (pdu, grid, payload) in enumerate(f34_cases(n=24, seed=5)):
        if i % 4 != 0:
            continue
        r, pay = op.ref_process_f34(grid, pdu)
        assert r.status == 1 and np.array_equal(pay, payload), (i, pdu.format, pdu.nof_prb, pdu.pi2_bpsk, r.status)
        n += 1
    assert n == 6


def test_pucch_f2_restatement_llrs_match_reference():
    """oracle/pucch.py demodulate_f2 (estimator + demodulator restated in numpy) against the compiled
    dmrs_pucch_estimator_format2 + pucch_demodulator_format2: every LLR within one quantisation step, >= 98 % equal
    (the restatement accumulates in float64 where the reference sums in float)."""
    from oracle import pucch as op
    from tests.pucch_cases import f2_cases

    for i, (pdu, grid, _) in enumerate(f2_cases(n=12, seed=1)):
        want = op.ref_demodulate_f2(grid, pdu).astype(np.int32)
        got = op.demodulate_f2(grid, pdu).astype(np.int32)
        diff = np.abs(got - want)
        assert diff.max() <= 1, (i, int(diff.max()), int(np.argmax(diff)))
        assert np.mean(diff == 0) >= 0.98, (i, float(np.mean(diff == 0)))


def test_pucch_f34_restatement_llrs_match_reference():
    """oracle/pucch.py demodulate_f34 against the compiled dmrs_pucch_estimator_formats3_4 +
    pucch_demodulator_format3 / 4: every LLR within one quantisation step, >= 98 % equal."""
    from oracle import pucch as op
    from tests.pucch_cases import f34_cases

    for i, (pdu, grid, _) in enumerate(f34_cases(n=12, seed=1)):
        want = op.ref_demodulate_f34(grid, pdu).astype(np.int32)
        got = op.demodulate_f34(grid, pdu).astype(np.int32)
        diff = np.abs(got - want)
        assert diff.max() <= 1, (i, pdu.format, pdu.pi2_bpsk, int(diff.max()), int(np.argmax(diff)))
        assert np.mean(diff == 0) >= 0.98, (i, float(np.mean(diff == 0)))

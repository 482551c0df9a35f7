"""The reference-side boundary, compiled against the reference's own headers (integration/Makefile) and
exercised through the reference's own code (oracle/hw_harness.cpp, oracle/adapter_harness.cpp):

  * the REFERENCE's hardware-accelerated PUSCH decoder, pusch_decoder_hw_impl
    (lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp), driving the MI355X plug-in
    hal::hw_accelerator_pusch_dec (integration/hip_accelerator_pusch_dec.cpp: external HARQ in HBM, one
    rate-dematch + LDPC batch per transport block), must give the same transport block, TB CRC verdict and
    LDPC statistics as the reference's software pusch_decoder_impl (oracle ref_wrapper_sch.cpp) on the same
    LLRs -- new data, HARQ combining across redundancy versions, single- and multi-codeblock TBs (CRC16 /
    CRC24A / CRC24B), BG1 / BG2, limited-buffer rate matching; two accelerator instances of one factory on two
    threads; a HARQ process abandoned without a CRC pass;
  * the reference's pdsch_encoder_hw_impl driving hal::hw_accelerator_pdsch_enc (TB and CB mode) must equal
    pdsch_encoder_impl bit-exactly;
  * the reference's OFDM slot modulator / demodulator built with the dft_processor adapter, its
    pusch_demodulator_impl with the channel_equalizer adapter, and its pusch_decoder_impl with the ldpc_decoder
    adapter must match the generic builds within the float tolerances stated per test (bit-exact for the decoder).
"""
import numpy as np
import pytest

import oracle
import oracle.sch as osch
from tests.pusch_demod_cases import CASES as DEMOD_CASES
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hw():
    import torch

    torch.cuda.init()  # torch's HIP runtime first, whatever test file ran before
    from oracle import hw as ohw

    return ohw, ohw.HwPuschDecoder(0)


def _plan(case, rv=None):
    tbs, bg, qm, lay, nre, rv0, nref = case
    return osch.plan(tbs, bg, rv0 if rv is None else rv, qm, nref, lay, nre)


@pytest.mark.parametrize("ci", range(len(SCH_CASES)))
def test_hw_plugin_matches_pusch_decoder_impl(hw, ci):
    ohw, dec = hw
    case = SCH_CASES[ci]
    p = _plan(case)
    tb = tb_bytes(p["tbs"], 100 + ci)
    cw = osch.pdsch_encode(tb, p)
    for k, sigma in enumerate((2.0, 6.0, 9.0)):
        llr = noisy_llrs(cw, 8, sigma, seed=ci * 10 + k)
        got_tb = np.zeros(p["tbs"] // 8, np.uint8)
        want_tb = np.zeros(p["tbs"] // 8, np.uint8)
        got = ohw.hw_pusch_decode(dec, llr, p, ohw.HwRxBuffer(p["nof_segments"], 1000 * ci + 100 * k), got_tb)
        want = oracle.ref_pusch_decode(llr, p, oracle.RefRxBuffer(p["nof_segments"]), want_tb)
        assert got == want, (case, sigma, got, want)
        np.testing.assert_array_equal(got_tb, want_tb, err_msg="case %d sigma %g" % (ci, sigma))
        if k == 0 and p["rv"] == 0:  # clean first transmission (rv > 0 alone may lack systematic bits)
            assert got[0] and np.array_equal(got_tb, tb)


def test_hw_plugin_harq_combining(hw):
    """rv 0 too noisy, then rv 2 and rv 3 combined in the accelerator's HBM HARQ rows (new_data = 0), then a new
    transport block on the same HARQ process (new_data = 1 resets)."""
    ohw, dec = hw
    case = (8 * 4000, 1, 4, 1, 12000, 0, 0)
    rx_hw = ohw.HwRxBuffer(_plan(case)["nof_segments"], 50000)
    rx_ref = oracle.RefRxBuffer(_plan(case)["nof_segments"])
    tb = tb_bytes(case[0], 5)
    got_tb = np.zeros(case[0] // 8, np.uint8)
    want_tb = np.zeros(case[0] // 8, np.uint8)
    oks = []
    for k, (rv, new, sigma) in enumerate(((0, True, 12.0), (2, False, 9.0), (3, False, 7.0))):
        p = _plan(case, rv)
        llr = noisy_llrs(osch.pdsch_encode(tb, p), 8, sigma, seed=77 + k)
        got = ohw.hw_pusch_decode(dec, llr, p, rx_hw, got_tb, new_data=new)
        want = oracle.ref_pusch_decode(llr, p, rx_ref, want_tb, new_data=new)
        assert got == want, (k, got, want)
        np.testing.assert_array_equal(got_tb, want_tb)
        oks.append(got[0])
    assert not oks[0] and oks[-1] and np.array_equal(got_tb, tb)
    tb2 = tb_bytes(case[0], 6)
    p = _plan(case, 0)
    llr = noisy_llrs(osch.pdsch_encode(tb2, p), 8, 3.0, seed=99)
    got = ohw.hw_pusch_decode(dec, llr, p, rx_hw, got_tb, new_data=True)
    want = oracle.ref_pusch_decode(llr, p, rx_ref, want_tb, new_data=True)
    assert got == want and got[0] and np.array_equal(got_tb, tb2)


def test_hw_plugin_no_early_stop(hw):
    ohw, dec = hw
    p = _plan(SCH_CASES[4])
    tb = tb_bytes(p["tbs"], 3)
    llr = noisy_llrs(osch.pdsch_encode(tb, p), 8, 5.0, seed=3)
    got_tb = np.zeros(p["tbs"] // 8, np.uint8)
    want_tb = np.zeros(p["tbs"] // 8, np.uint8)
    got = ohw.hw_pusch_decode(dec, llr, p, ohw.HwRxBuffer(p["nof_segments"], 90000), got_tb, use_early_stop=False)
    want = oracle.ref_pusch_decode(llr, p, oracle.RefRxBuffer(p["nof_segments"]), want_tb, use_early_stop=False)
    assert got == want
    np.testing.assert_array_equal(got_tb, want_tb)


def test_hw_plugin_concurrent_instances(hw):
    """Two accelerator instances of ONE factory (one shared HBM HARQ pool) decode transport blocks on two
    threads at once, as the reference's decoder pool does (pusch_decoder_hw_impl::hw_decoder_pool): rows are
    reserved per transport block under the pool's lock, so neither thread takes the other's rows."""
    import threading

    ohw, dec = hw
    dec2 = ohw.HwPuschDecoder(0, sibling_of=dec)
    case = (8 * 6000, 1, 6, 2, 9000, 0, 0)
    p = _plan(case)
    C = p["nof_segments"]
    assert C > 1
    jobs = []
    for k in range(12):
        tb = tb_bytes(case[0], 300 + k)
        llr = noisy_llrs(osch.pdsch_encode(tb, p), 8, 3.0 if k % 3 else 9.0, seed=500 + k)
        want_tb = np.zeros(case[0] // 8, np.uint8)
        want = oracle.ref_pusch_decode(llr, p, oracle.RefRxBuffer(C), want_tb)
        jobs.append((llr, want, want_tb))
    results = [None] * len(jobs)

    def worker(d, idx):
        for k in idx:
            got_tb = np.zeros(case[0] // 8, np.uint8)
            got = ohw.hw_pusch_decode(d, jobs[k][0], p, ohw.HwRxBuffer(C, 200000 + 64 * k), got_tb)
            results[k] = (got, got_tb)

    th = [threading.Thread(target=worker, args=(d, range(i, len(jobs), 2))) for i, d in enumerate((dec, dec2))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for k, (llr, want, want_tb) in enumerate(jobs):
        got, got_tb = results[k]
        assert got == want, (k, got, want)
        np.testing.assert_array_equal(got_tb, want_tb)
    dec2.close()


def test_hw_plugin_abandoned_harq_process(hw):
    """A HARQ process that never passed its CRC keeps its rows (the reference frees them only on a TB CRC pass);
    its absolute codeblock ids are then reused by a new transport block with MORE codeblocks (new data): the
    plug-in remaps the stale ids instead of failing, and still equals pusch_decoder_impl."""
    ohw, dec = hw
    small = (8 * 3000, 1, 4, 1, 8000, 0, 0)
    big = (8 * 9000, 1, 6, 2, 14000, 0, 0)
    ps, pb = _plan(small), _plan(big)
    assert pb["nof_segments"] > ps["nof_segments"] > 1
    tb = tb_bytes(small[0], 11)
    got_tb = np.zeros(small[0] // 8, np.uint8)
    got = ohw.hw_pusch_decode(dec, noisy_llrs(osch.pdsch_encode(tb, ps), 8, 14.0, seed=1), ps,
                              ohw.HwRxBuffer(ps["nof_segments"], 300001), got_tb)
    assert not got[0]  # abandoned: rows stay mapped
    tb = tb_bytes(big[0], 12)
    llr = noisy_llrs(osch.pdsch_encode(tb, pb), 8, 2.0, seed=2)
    got_tb = np.zeros(big[0] // 8, np.uint8)
    want_tb = np.zeros(big[0] // 8, np.uint8)
    got = ohw.hw_pusch_decode(dec, llr, pb, ohw.HwRxBuffer(pb["nof_segments"], 300000), got_tb)
    want = oracle.ref_pusch_decode(llr, pb, oracle.RefRxBuffer(pb["nof_segments"]), want_tb)
    assert got == want and got[0]
    np.testing.assert_array_equal(got_tb, tb)


# ---- the other reference-side adapters, each driven by the REFERENCE's own class (oracle/adapter_harness.cpp) ----

@pytest.mark.parametrize("cb_mode", [False, True], ids=["tb_mode", "cb_mode"])
@pytest.mark.parametrize("ci", range(len(SCH_CASES)))
def test_hw_pdsch_enc_plugin_matches_pdsch_encoder_impl(hw, ci, cb_mode):
    """pdsch_encoder_hw_impl (pdsch_encoder_hw_impl.cpp) with the MI355X hal::hw_accelerator_pdsch_enc: the same
    codeword bits as the reference's software pdsch_encoder_impl, bit-exact (TB mode: one GPU batch per transport
    block; CB mode: the reference segments, the GPU LDPC-encodes and rate-matches each codeblock)."""
    ohw, _ = hw
    p = _plan(SCH_CASES[ci])
    for seed in (0, 1):
        tb = tb_bytes(p["tbs"], 700 + 10 * ci + seed)
        got = ohw.hw_pdsch_encode(tb, p, cb_mode=cb_mode)
        want = oracle.ref_pdsch_encode(tb, p)
        assert np.array_equal(got, want), (SCH_CASES[ci], cb_mode, int((got != want).sum()))


def test_hw_pdsch_enc_plugin_failure_does_not_stall(hw):
    """a failed operation (TB-mode transport block one byte short of its configuration; CB-mode codeblock
    shorter than K - F) is logged and dequeues the configured codeword length as zeros on the first call, so the
    reference's driver loop (pdsch_encoder_hw_impl.cpp:150-160: dequeue until it returns true) moves on."""
    ohw, _ = hw
    assert ohw.lib().srs_ref_hw_pdsch_enc_forced_failure(0) == 0


DFT_OFDM_CASES = [(1, 273, 4096, 1.0, 3.5e9), (0, 52, 1024, 0.5, 1.8e9), (1, 106, 1536, 0.7, 2.6e9)]


@pytest.mark.parametrize("case", DFT_OFDM_CASES)
def test_dft_adapter_through_ofdm_modulator(hw, case):
    """ofdm_slot_modulator_impl / ofdm_slot_demodulator_impl (ofdm_modulator_impl.cpp / ofdm_demodulator_impl.cpp)
    built with the MI355X dft_processor instead of dft_processor_generic_impl: baseband samples within 4e-5 x RMS of
    the generic build (each float DFT sits within 2e-5 x RMS of the exact transform), resource grids within one bf16
    ulp (+ 3e-5 x RMS near zero) and >= 99 % identical."""
    from oracle import ofdm as oofdm

    ohw, _ = hw
    mu, bw, N, scale, fc = case
    rng = np.random.default_rng(N + bw)
    for slot in (0, (1 << mu) - 1):
        g = oofdm.random_grid(rng, 14, bw * 12)
        want = oracle.ref_ofdm_modulate_slot(g, slot, mu, bw, N, scale, fc)
        got = ohw.hip_ofdm_modulate_slot(g, slot, mu, bw, N, scale, fc, want.size)
        rms = float(np.sqrt(np.mean(np.abs(want) ** 2)))
        assert np.max(np.abs(got - want)) <= 4e-5 * rms, (case, slot, np.max(np.abs(got - want)) / rms)
        rx = (want + (rng.normal(0, 0.05, want.size) + 1j * rng.normal(0, 0.05, want.size)) * rms).astype(np.complex64)
        gw = oracle.ref_ofdm_demodulate_slot(rx, slot, mu, bw, N, scale, fc).view(np.uint32)
        gg = ohw.hip_ofdm_demodulate_slot(rx, slot, mu, bw, N, scale, fc).view(np.uint32)
        a = (gg.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
        b = (gw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
        tol = 2.0 ** -7 * np.maximum(np.abs(a), np.abs(b)) + 3e-5 * np.sqrt(np.mean(b ** 2))
        assert (np.abs(a - b) <= tol).all(), case
        assert (gg == gw).mean() >= 0.99, (case, (gg == gw).mean())


# (numerology, PRBs, DFT size, extended CP, window offset, scale, fc, fc after set_center_frequency)
OFDM_PLUGIN_CASES = [(1, 273, 4096, False, 0, 1.0, 3.5e9, 3.6e9), (0, 52, 1024, False, 36, 0.5, 1.8e9, 1.8e9),
                     (2, 66, 1024, True, 20, 0.8, 28e9, 27.5e9), (1, 106, 1536, False, 0, 0.7, 2.6e9, 2.6e9)]


def _assert_grids_close(gg, gw, case):
    a = (gg.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    b = (gw.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    tol = 2.0 ** -7 * np.maximum(np.abs(a), np.abs(b)) + 3e-5 * np.sqrt(np.mean(b ** 2))
    assert (np.abs(a - b) <= tol).all(), case
    assert (gg.view(np.uint32) == gw.view(np.uint32)).mean() >= 0.99, case


@pytest.mark.parametrize("case", OFDM_PLUGIN_CASES)
def test_ofdm_factory_plugins_vs_reference(hw, case):
    """The ofdm_modulator_factory / ofdm_demodulator_factory plug-ins (integration/ofdm_modulator_hip.h: whole-slot
    launches for ofdm_slot_*, one launch per symbol for ofdm_symbol_*, set_center_frequency on the symbol forms)
    against the reference's ofdm_slot_(de)modulator_impl over the generic DFT built for the same center frequency:
    samples within 2e-5 x RMS, grids within one bf16 ulp (+ 3e-5 x RMS near zero) and >= 99 % identical; an
    extended-CP (12 symbols) and a window-offset case included."""
    from oracle import ofdm as oofdm

    ohw, _ = hw
    mu, bw, N, ext, off, scale, fc, fc2 = case
    ns = 12 if ext else 14
    rng = np.random.default_rng(N + bw + off)
    for slot in (0, (1 << mu) - 1):
        g = oofdm.random_grid(rng, ns, bw * 12)
        for mode, f in (("slot_mod", fc), ("symbol_mod", fc2)):
            want = oracle.ref_ofdm_modulate_slot(g, slot, mu, bw, N, scale, f, extended_cp=ext)
            got = ohw.ofdm_plugin(mode, g, slot, mu, bw, N, scale, fc, fc2=fc2, extended_cp=ext, n=want.size)
            rms = float(np.sqrt(np.mean(np.abs(want) ** 2)))
            assert np.max(np.abs(got - want)) <= 2e-5 * rms, (case, slot, mode, np.max(np.abs(got - want)) / rms)
        rx = (want + (rng.normal(0, 0.05, want.size) + 1j * rng.normal(0, 0.05, want.size)) * rms).astype(np.complex64)
        for mode, f in (("slot_demod", fc), ("symbol_demod", fc2)):
            gw = oracle.ref_ofdm_demodulate_slot(rx, slot, mu, bw, N, scale, f, window_offset=off, extended_cp=ext)
            gg = ohw.ofdm_plugin(mode, rx, slot, mu, bw, N, scale, fc, fc2=fc2, extended_cp=ext, window_offset=off)
            _assert_grids_close(gg, gw, (case, slot, mode))


def test_ofdm_factory_plugin_throughput(hw):
    """Symbols/s of the slot plug-ins (synchronous per (port, slot) call, as the interface is) beside the reference's
    ofdm_slot_(de)modulator_impl over the generic DFT on one host core, 100 MHz / 4096-point slots; written to
    gpurun_out/ofdm_plugin_bench.json."""
    import json
    import os

    ohw, _ = hw
    out = {}
    for demod in (False, True):
        name = "demodulator" if demod else "modulator"
        ohw.ofdm_bench(True, demod, 1, 273, 4096, 20)  # warm-up
        t_gpu = ohw.ofdm_bench(True, demod, 1, 273, 4096, 400)
        t_cpu = ohw.ofdm_bench(False, demod, 1, 273, 4096, 20)
        assert t_gpu > 0 and t_cpu > 0
        out[name] = {"plugin_symbols_per_s": 400 * 14 / t_gpu, "reference_1core_symbols_per_s": 20 * 14 / t_cpu,
                     "plugin_us_per_slot": 1e6 * t_gpu / 400, "reference_us_per_slot": 1e6 * t_cpu / 20}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/ofdm_plugin_bench.json", "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)


@pytest.mark.parametrize("ci", range(len(DEMOD_CASES)))
def test_equalizer_adapter_through_pusch_demodulator(hw, ci):
    """pusch_demodulator_impl (pusch_demodulator_impl.cpp:203-445) built with the MI355X channel_equalizer instead of
    channel_equalizer_generic_impl: the LLRs of the whole demodulator within |dLLR| <= 1, >= 97 % identical (the
    reference's AVX2 ZF path multiplies by an approximate reciprocal, tests/pusch_demod_cases.py)."""
    from oracle import pusch_demod as od
    from tests.pusch_demod_cases import assert_llrs_close, demod_args, make_case

    ohw, _ = hw
    case = DEMOD_CASES[ci]
    grid, est, nv, crbs = make_case(case, seed=40 + ci)
    args = demod_args(case)
    want = od.ref_pusch_demodulate(grid, est, nv, 0x4601, 500, crbs=crbs, **args)
    got = ohw.hip_pusch_demodulate(grid, est, nv, 0x4601, 500, crbs=crbs, **args)
    assert_llrs_close(got, want, case[0], min_equal=0.97)


@pytest.mark.parametrize("generic", [False, True], ids=["hip", "hip-generic"])
@pytest.mark.parametrize("ci", range(len(SCH_CASES)))
def test_ldpc_decoder_adapter_through_pusch_decoder(hw, ci, generic):
    """pusch_decoder_impl + pusch_codeblock_decoder (pusch_codeblock_decoder.cpp:35-69) whose ldpc_decoder is the
    MI355X adapter (integration/ldpc_decoder_hip, the "hip" / "hip-generic" decoder types): transport block, TB CRC
    and LDPC statistics identical to the reference's AVX2 / generic decoders, new data and HARQ combining."""
    ohw, _ = hw
    p = _plan(SCH_CASES[ci])
    tb = tb_bytes(p["tbs"], 900 + ci)
    cw = osch.pdsch_encode(tb, p)
    rx_a, rx_b = oracle.RefRxBuffer(p["nof_segments"]), oracle.RefRxBuffer(p["nof_segments"])
    for k, (sigma, new) in enumerate(((9.0, True), (6.0, False), (3.0, True))):
        llr = noisy_llrs(cw, 8, sigma, seed=ci * 17 + k)
        got_tb = np.zeros(p["tbs"] // 8, np.uint8)
        want_tb = np.zeros(p["tbs"] // 8, np.uint8)
        got = ohw.hip_ldpc_pusch_decode(llr, p, rx_a, got_tb, generic=generic, new_data=new)
        want = oracle.ref_pusch_decode(llr, p, rx_b, want_tb, generic=generic, new_data=new)
        assert got == want, (SCH_CASES[ci], sigma, got, want)
        np.testing.assert_array_equal(got_tb, want_tb)

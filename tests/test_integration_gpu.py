"""The reference-side boundary, compiled against the reference's own headers (integration/Makefile) and
exercised through the reference's own code:

  * the REFERENCE's hardware-accelerated PUSCH decoder, pusch_decoder_hw_impl
    (lib/phy/upper/channel_processors/pusch/pusch_decoder_hw_impl.cpp), driving the MI355X plug-in
    hal::hw_accelerator_pusch_dec (integration/hip_accelerator_pusch_dec.cpp: external HARQ in HBM, one
    rate-dematch + LDPC batch per transport block), must give the same transport block, TB CRC verdict and
    LDPC statistics as the reference's software pusch_decoder_impl (oracle ref_wrapper_sch.cpp) on the same
    LLRs -- new data, HARQ combining across redundancy versions, single- and multi-codeblock TBs (CRC16 /
    CRC24A / CRC24B), BG1 / BG2, limited-buffer rate matching.
"""
import numpy as np
import pytest

import oracle
import oracle.sch as osch
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

"""PUCCH Format 0 detector on the MI355X vs the compiled reference pucch_detector_format0 (oracle/_ref) and the numpy
restatement, every case of tests/pucch_cases.py, host and slot forms.  Status, SR and HARQ-ACK bits are exact; the
detection metric within 1e-3 relative and SINR / RSRP / EPRE within 0.01 dB (the GPU sums the correlation in another
order and builds the cyclic shifts from a double-precision exponential, the reference from a float table)."""
import numpy as np
import pytest

from tests.pucch_cases import NSUBC, cases

pytestmark = pytest.mark.gpu
RTOL, DB_TOL = 1e-3, 0.01


@pytest.fixture(scope="module")
def proc():
    import srsran_project_amd as amd

    return amd.PucchProcessor(device=0)


def _check(i, got, want):
    assert got["status"] == want.status, (i, got["status"], want.status, want.detection_metric)
    assert got["nof_sr"] == want.nof_sr and got["nof_harq_ack"] == want.nof_harq_ack, i
    if want.nof_sr:
        assert got["sr"] == want.sr, i
    assert list(got["harq_ack"][:want.nof_harq_ack]) == list(want.harq_ack)[:want.nof_harq_ack], i
    np.testing.assert_allclose(got["detection_metric"], want.detection_metric, rtol=RTOL, err_msg=str(i))
    for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
        assert abs(float(got[k]) - getattr(want, k)) <= DB_TOL, (i, k, got[k], getattr(want, k))


def _rec(r):
    import srsran_project_amd as amd

    return np.frombuffer(bytes(r), amd.pucch.RESULT_DTYPE)[0]


def test_pucch_f0_host_form_vs_reference(proc):
    from oracle import pucch as op

    n_valid = 0
    for i, (pdu, grid, sent) in enumerate(cases()):
        want = op.ref_detect(grid, pdu)
        got = _rec(proc.detect_f0(grid, pdu))
        _check(i, got, want)
        n_valid += want.status == 1
    assert 0 < n_valid < len(cases())


def test_pucch_f0_slot_form_every_pdu_one_launch(proc):
    """All cases' PDUs over their own grids (d_grids[i]) in one call, plus two more PDUs sharing grid 0."""
    import torch

    import srsran_project_amd as amd
    from oracle import pucch as op

    cs = cases(n=30, seed=4)
    pdus = []
    for i, (pdu, _, _) in enumerate(cs):
        pdu.grid = i
        pdus.append(pdu)
    g = np.stack([c[1] for c in cs])
    d = torch.from_numpy(g.view(np.int32).copy()).to("cuda:0")
    raw = proc.detect_f0_slot(d, pdus)
    torch.cuda.synchronize()
    got = amd.pucch.parse_results(raw.cpu().numpy())
    for i, (pdu, grid, _) in enumerate(cs):
        _check(i, got[i], op.ref_detect(grid, pdu))


def test_pucch_f0_restatement_agrees(proc):
    from oracle import pucch as op

    for i, (pdu, grid, sent) in enumerate(cases(n=12, seed=9)):
        st, sr, harq, metric, *_ = op.detect(grid, pdu)
        got = _rec(proc.detect_f0(grid, pdu))
        assert got["status"] == st and list(got["harq_ack"][:len(harq)]) == list(harq), i


def test_pucch_f0_invalid_pdu_fails_loudly(proc):
    import srsran_project_amd as amd

    g = np.zeros((4, 14, NSUBC), np.uint32)
    bad = [dict(nof_symbols=3), dict(start_symbol_index=13, nof_symbols=2), dict(nof_symbols=1, second_hop_prb=3),
           dict(initial_cyclic_shift=12), dict(nof_harq_ack=3), dict(starting_prb=52), dict(ports=(4,)),
           dict(nof_harq_ack=0, sr_opportunity=False, n_id=1024)]
    for kw in bad:
        with pytest.raises(ValueError):
            proc.detect_f0(g, amd.pucch.make_f0_pdu(**kw))


# ---- Format 1 ------------------------------------------------------------------------------------------------------
def test_pucch_f1_host_form_vs_reference(proc):
    """Every multiplexed PUCCH of every batch: status and HARQ-ACK bits exact, metric / CSI within tolerance."""
    from oracle import pucch as op
    from tests.pucch_cases import f1_cases

    n_valid = n = 0
    for i, (b, grid, sent) in enumerate(f1_cases(n=24, seed=1)):
        want = op.ref_detect_f1(grid, b)
        got = proc.detect_f1(grid, b)
        for j, (g, w) in enumerate(zip(got, want)):
            _check((i, j), _rec(g), w)
            n_valid += w.status == 1
            n += 1
    assert 0 < n_valid < n


def test_pucch_f1_slot_form_every_batch_one_launch(proc):
    import torch

    import srsran_project_amd as amd
    from oracle import pucch as op
    from tests.pucch_cases import f1_cases

    cs = f1_cases(n=20, seed=2)
    for i, (b, _, _) in enumerate(cs):
        b.grid = i
    g = np.stack([c[1] for c in cs])
    d = torch.from_numpy(g.view(np.int32).copy()).to("cuda:0")
    raw = proc.detect_f1_slot(d, [c[0] for c in cs])
    torch.cuda.synchronize()
    got = amd.pucch.parse_results(raw.cpu().numpy())
    k = 0
    for i, (b, grid, _) in enumerate(cs):
        for j, w in enumerate(op.ref_detect_f1(grid, b)):
            _check((i, j), got[k], w)
            k += 1
    assert k == len(got)


def test_pucch_f1_all_84_pucchs_of_a_prb(proc):
    """A full batch: every (shift, OCC) of a 14-symbol allocation, one launch."""
    import srsran_project_amd as amd
    from oracle import pucch as op

    rng = np.random.default_rng(3)
    entries = [(ics, o, int(rng.integers(0, 3))) for o in range(7) for ics in range(12)]
    b = amd.pucch.make_f1_batch(entries, slot_index=3, starting_prb=10, nof_symbols=14, n_id=333, ports=(1, 0))
    grid = rng.integers(0, 1 << 32, (2, 14, NSUBC), dtype=np.uint64).astype(np.uint32)
    sel = [(ics, o, [int(x) for x in rng.integers(0, 2, nh)], (rng.normal(size=2) + 1j * rng.normal(size=2)) / 2)
           for ics, o, nh in entries if (ics + o) % 5 == 0]
    op.transmit_f1(grid, b, sel, 0.05, rng)
    want = op.ref_detect_f1(grid, b)
    for j, (g, w) in enumerate(zip(proc.detect_f1(grid, b), want)):
        _check(j, _rec(g), w)


def test_pucch_f1_invalid_batch_fails_loudly(proc):
    import srsran_project_amd as amd

    g = np.zeros((4, 14, NSUBC), np.uint32)
    ok = [(0, 0, 1)]
    bad = [(ok, dict(nof_symbols=3)), (ok, dict(start_symbol_index=11, nof_symbols=4)),
           (ok, dict(start_symbol_index=4, nof_symbols=11)), (ok, dict(ports=(0, 1, 2))),
           (ok, dict(n_id=1024)), (ok, dict(starting_prb=52)), ([(12, 0, 1)], {}), ([(0, 7, 1)], {}),
           ([(0, 2, 1)], dict(nof_symbols=4)), ([(0, 1, 1)], dict(nof_symbols=7, second_hop_prb=3)),
           ([(0, 0, 3)], {}), ([(1, 0, 1), (1, 0, 2)], {}), ([], {})]
    for entries, kw in bad:
        with pytest.raises(ValueError):
            proc.detect_f1(g, amd.pucch.make_f1_batch(entries, **kw))


# ---- Format 2 ------------------------------------------------------------------------------------------------------
F2_TA_TOL = 2.5 / (480e3 * 4096)  # two T_C units: the correlation peak's fractional refinement in float


def _check_uci(i, got, pay, want, want_pay):
    assert got["status"] == want.status, (i, got["status"], want.status, want.sinr_dB)
    for k in ("nof_harq_ack", "nof_sr", "nof_csi_part1", "nof_csi_part2"):
        assert got[k] == getattr(want, k), (i, k)
    assert np.array_equal(np.asarray(pay), np.asarray(want_pay)), i
    for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
        assert abs(float(got[k]) - getattr(want, k)) <= 0.02, (i, k, got[k], getattr(want, k))
    assert abs(float(got["time_alignment_s"]) - want.time_alignment_s) <= F2_TA_TOL, (i, got["time_alignment_s"],
                                                                                      want.time_alignment_s)
    if np.isnan(want.cfo_Hz):
        assert np.isnan(got["cfo_Hz"]), i
    else:
        assert abs(float(got["cfo_Hz"]) - want.cfo_Hz) <= 1e-3 * max(1.0, abs(want.cfo_Hz)), (i, got["cfo_Hz"],
                                                                                               want.cfo_Hz)


def _uci_rec(r):
    import srsran_project_amd as amd

    return np.frombuffer(bytes(r), amd.pucch.UCI_RESULT_DTYPE)[0]


def test_pucch_f2_llrs_vs_reference(proc):
    """The descrambled LLRs of the estimator + demodulator against the compiled dmrs_pucch_estimator_format2 +
    pucch_demodulator_format2: every LLR within one quantisation step, at least 99 % identical."""
    from oracle import pucch as op
    from tests.pucch_cases import f2_cases

    for i, (pdu, grid, payload) in enumerate(f2_cases(n=24, seed=1)):
        want = op.ref_demodulate_f2(grid, pdu).astype(np.int32)
        got = proc.demodulate_f2(grid, pdu).astype(np.int32)
        diff = np.abs(got - want)
        bad = np.nonzero(diff > 1)[0]
        assert bad.size == 0, (i, pdu.nof_prb, pdu.nof_symbols, pdu.second_hop_prb, bad[:8], got[bad[:8]],
                               want[bad[:8]], int(np.sum(np.sign(got) != np.sign(want))))
        assert np.mean(diff == 0) >= 0.99, (i, float(np.mean(diff == 0)))


def test_pucch_f2_host_form_vs_reference(proc):
    """Payload bits and status equal to the compiled pucch_processor_impl; CSI within 0.02 dB / two T_C / 1e-3."""
    from oracle import pucch as op
    from tests.pucch_cases import f2_cases

    n_valid = 0
    for i, (pdu, grid, payload) in enumerate(f2_cases(n=24, seed=1)):
        want, want_pay = op.ref_process_f2(grid, pdu)
        got, pay = proc.process_f2(grid, pdu)
        _check_uci(i, _uci_rec(got), pay, want, want_pay)
        n_valid += want.status == 1
    assert 0 < n_valid < 24


def test_pucch_f2_slot_form_one_call(proc):
    """Many PDUs of mixed payload / codeword sizes (several UCI decoder groups) over their own grids in one call."""
    import torch

    import srsran_project_amd as amd
    from oracle import pucch as op
    from tests.pucch_cases import f2_cases

    cs = f2_cases(n=20, seed=2)
    for i, (pdu, _, _) in enumerate(cs):
        pdu.grid = i
    g = np.stack([c[1] for c in cs])
    d = torch.from_numpy(g.view(np.int32).copy()).to("cuda:0")
    res, pay = proc.process_f2_slot(d, [c[0] for c in cs])
    torch.cuda.synchronize()
    got = amd.pucch.parse_uci_results(res.cpu().numpy())
    pay = pay.cpu().numpy()
    for i, (pdu, grid, _) in enumerate(cs):
        want, want_pay = op.ref_process_f2(grid, pdu)
        _check_uci(i, got[i], pay[i, :amd.pucch.payload_bits(pdu)], want, want_pay)


def test_pucch_f2_invalid_pdu_fails_loudly(proc):
    import srsran_project_amd as amd

    g = np.zeros((4, 14, 624), np.uint32)
    ok = dict(nof_prb=2, nof_harq_ack=4)
    bad = [dict(nof_prb=17, nof_harq_ack=4), dict(nof_prb=0, nof_harq_ack=4), dict(ok, nof_symbols=3),
           dict(ok, start_symbol_index=13), dict(ok, nof_symbols=1, second_hop_prb=5), dict(ok, nof_harq_ack=2),
           dict(ok, nof_csi_part2=4), dict(nof_prb=1, nof_symbols=1, nof_harq_ack=20), dict(ok, starting_prb=51),
           dict(ok, bwp_start_rb=10, bwp_size_rb=48), dict(ok, ports=(4,)), dict(ok, n_id=1024)]
    for kw in bad:
        with pytest.raises(ValueError):
            proc.process_f2(g, amd.pucch.make_f2_pdu(**kw))


# ---- Formats 3 / 4 -------------------------------------------------------------------------------------------------
def test_pucch_f34_llrs_vs_reference(proc):
    """The descrambled LLRs against the compiled dmrs_pucch_estimator_formats3_4 + pucch_demodulator_format3 / 4:
    every LLR within one quantisation step, at least 99 % identical (the IDFT of the transform deprecoding sums in
    another order than the reference's DFT)."""
    from oracle import pucch as op
    from tests.pucch_cases import f34_cases

    for i, (pdu, grid, payload) in enumerate(f34_cases(n=24, seed=1)):
        want = op.ref_demodulate_f34(grid, pdu).astype(np.int32)
        got = proc.demodulate_f34(grid, pdu).astype(np.int32)
        diff = np.abs(got - want)
        bad = np.nonzero(diff > 1)[0]
        assert bad.size == 0, (i, pdu.format, pdu.nof_prb, pdu.nof_symbols, pdu.second_hop_prb, pdu.pi2_bpsk,
                               bad[:8], got[bad[:8]], want[bad[:8]])
        assert np.mean(diff == 0) >= 0.99, (i, float(np.mean(diff == 0)))


def test_pucch_f34_host_form_vs_reference(proc):
    from oracle import pucch as op
    from tests.pucch_cases import f34_cases

    n_valid = 0
    for i, (pdu, grid, payload) in enumerate(f34_cases(n=24, seed=2)):
        want, want_pay = op.ref_process_f34(grid, pdu)
        got, pay = proc.process_f34(grid, pdu)
        _check_uci(i, _uci_rec(got), pay, want, want_pay)
        n_valid += want.status == 1
    assert 0 < n_valid < 24


def test_pucch_f34_slot_form_one_call(proc):
    import torch

    import srsran_project_amd as amd
    from oracle import pucch as op
    from tests.pucch_cases import f34_cases

    cs = f34_cases(n=20, seed=3)
    for i, (pdu, _, _) in enumerate(cs):
        pdu.grid = i
    g = np.stack([c[1] for c in cs])
    d = torch.from_numpy(g.view(np.int32).copy()).to("cuda:0")
    res, pay = proc.process_f34_slot(d, [c[0] for c in cs])
    torch.cuda.synchronize()
    got = amd.pucch.parse_uci_results(res.cpu().numpy())
    pay = pay.cpu().numpy()
    for i, (pdu, grid, _) in enumerate(cs):
        want, want_pay = op.ref_process_f34(grid, pdu)
        _check_uci(i, got[i], pay[i, :amd.pucch.payload_bits(pdu)], want, want_pay)


def test_pucch_f34_invalid_pdu_fails_loudly(proc):
    import srsran_project_amd as amd

    g = np.zeros((4, 14, 624), np.uint32)
    ok = dict(nof_prb=2, nof_harq_ack=4)
    bad = [dict(ok, nof_prb=7), dict(ok, nof_prb=17), dict(ok, nof_symbols=3), dict(ok, start_symbol_index=11),
           dict(ok, nof_csi_part2=2), dict(nof_prb=1, nof_symbols=4, nof_harq_ack=70), dict(ok, format=5),
           dict(format=4, occ_length=3, nof_harq_ack=4), dict(format=4, occ_length=2, occ_index=2, nof_harq_ack=4),
           dict(ok, starting_prb=51), dict(ok, ports=(4,)), dict(ok, n_id_hopping=1024)]
    for kw in bad:
        with pytest.raises(ValueError):
            proc.process_f34(g, amd.pucch.make_f34_pdu(**kw))


def test_pucch_every_format_sharing_one_grid(proc):
    """Several PDUs of every format on disjoint PRBs of ONE grid, each format's slot form called once on it: every
    result equals the compiled reference's for the same grid (the kernels read only their PDU's REs)."""
    import torch

    import srsran_project_amd as amd
    from oracle import pucch as op
    from tests import pucch_cases as pc

    rng = np.random.default_rng(31)
    grid = rng.integers(0, 1 << 32, (4, 14, pc.NSUBC), dtype=np.uint64).astype(np.uint32)
    f0 = [amd.pucch.make_f0_pdu(numerology=1, slot_index=5, starting_prb=k, start_symbol_index=12, nof_symbols=2,
                                initial_cyclic_shift=k, n_id=40 + k, nof_harq_ack=1 + k % 2, sr_opportunity=k % 3 == 0,
                                ports=(0, 1)) for k in range(3)]
    for k, p in enumerate(f0):
        op.transmit(grid, p, op.TABLES[(p.nof_harq_ack, bool(p.sr_opportunity))][k % 2][0], [0.8, -0.5j], 0.05, rng)
    f2 = [amd.pucch.make_f2_pdu(numerology=1, slot_index=5, bwp_size_rb=52, starting_prb=4 + 3 * k, nof_prb=3,
                                start_symbol_index=12, nof_symbols=2, rnti=100 + k, n_id=7 + k, n_id_0=9 + k,
                                nof_harq_ack=2, nof_csi_part1=10 + 8 * k, ports=(0, 1)) for k in range(3)]
    pay2 = [rng.integers(0, 2, amd.pucch.payload_bits(p)).astype(np.uint8) for p in f2]
    for p, y in zip(f2, pay2):
        op.transmit_f2(grid, p, y, [0.9, 0.4 + 0.3j], 0.02, rng)
    f34 = [amd.pucch.make_f34_pdu(format=3, numerology=1, slot_index=5, bwp_size_rb=52, starting_prb=20 + 4 * k,
                                  nof_prb=4, start_symbol_index=0, nof_symbols=12, rnti=200 + k, n_id_hopping=3 + k,
                                  n_id_scrambling=5 + k, nof_harq_ack=3, nof_csi_part1=20 * (k + 1), ports=(0, 1))
           for k in range(2)]
    f34.append(amd.pucch.make_f34_pdu(format=4, numerology=1, slot_index=5, bwp_size_rb=52, starting_prb=30,
                                      start_symbol_index=0, nof_symbols=12, rnti=300, n_id_hopping=8,
                                      n_id_scrambling=9, nof_harq_ack=4, occ_index=1, occ_length=2, ports=(0, 1)))
    pay34 = [rng.integers(0, 2, amd.pucch.payload_bits(p)).astype(np.uint8) for p in f34]
    for p, y in zip(f34, pay34):
        op.transmit_f34(grid, p, y, [0.7j, 0.6], 0.02, rng)
    d = torch.from_numpy(grid[None].view(np.int32).copy()).to("cuda:0")
    r0 = amd.pucch.parse_results(proc.detect_f0_slot(d, f0).cpu().numpy())
    res2, p2 = proc.process_f2_slot(d, f2)
    res34, p34 = proc.process_f34_slot(d, f34)
    torch.cuda.synchronize()
    r2, p2 = amd.pucch.parse_uci_results(res2.cpu().numpy()), p2.cpu().numpy()
    r34, p34 = amd.pucch.parse_uci_results(res34.cpu().numpy()), p34.cpu().numpy()
    for k, p in enumerate(f0):
        _check(k, r0[k], op.ref_detect(grid, p))
    for k, p in enumerate(f2):
        want, want_pay = op.ref_process_f2(grid, p)
        _check_uci(k, r2[k], p2[k, :amd.pucch.payload_bits(p)], want, want_pay)
        assert want.status == 1 and np.array_equal(want_pay, pay2[k]), k
    for k, p in enumerate(f34):
        want, want_pay = op.ref_process_f34(grid, p)
        _check_uci(k, r34[k], p34[k, :amd.pucch.payload_bits(p)], want, want_pay)
        assert want.status == 1 and np.array_equal(want_pay, pay34[k]), k

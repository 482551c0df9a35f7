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

"""SS/PBCH block processor on the MI355X vs the compiled reference ssb_processor_impl (oracle/_ref) and the numpy
restatement: grids bit-exact for every case of tests/ssb_cases.py, host and slot forms."""
import numpy as np
import pytest

from tests.ssb_cases import CASES, INVALID, NSUBC, grid0, pdu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def proc():
    import srsran_project_amd as amd

    return amd.SsbProcessor(device=0)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_ssb_process_host_grid(proc, case):
    from oracle import ssb as oss

    p = pdu(case, seed=7)
    g0 = grid0(seed=3)
    want = oss.ref_process(g0.copy(), [p])
    got = proc.process(g0.copy(), p)
    assert np.array_equal(got, want), "%d REs differ" % int((got != want).sum())
    assert (want != g0).sum() > 0


def test_ssb_process_slot_every_case_one_call(proc):
    import torch

    from oracle import ssb as oss

    pdus = [pdu(c, seed=11 + i, grid=i) for i, c in enumerate(CASES)]
    g0 = np.stack([grid0(seed=20 + i) for i in range(len(CASES))])
    d = torch.from_numpy(g0.view(np.int32).copy()).to("cuda:0")
    proc.process_slot(d, pdus)
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32)
    for i, p in enumerate(pdus):
        want = oss.ref_process(g0[i].copy(), [p])
        assert np.array_equal(got[i], want), CASES[i][0]


def test_ssb_two_blocks_one_grid(proc):
    """Case A blocks 0 and 1 (symbols 2 and 8) of one slot into the same grid, one call."""
    import torch

    import srsran_project_amd as amd
    from oracle import ssb as oss

    rng = np.random.default_rng(5)
    pdus = [amd.ssb.make_pdu(rng.integers(0, 2, 24), numerology=0, sfn=9, slot_index=0, phys_cell_id=77, ssb_idx=k,
                             L_max=4, offset_to_pointA=30, ports=(0, 1)) for k in (0, 1)]
    g0 = grid0(seed=9, ports=2)
    want = oss.ref_process(g0.copy(), pdus)
    d = torch.from_numpy(g0[None].view(np.int32).copy()).to("cuda:0")
    proc.process_slot(d, pdus)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint32)[0], want)


def test_ssb_invalid_pdu_fails_loudly(proc):
    g = np.zeros((4, 14, NSUBC), np.uint32)
    for c in INVALID:
        with pytest.raises(ValueError):
            proc.process(g, pdu(c))

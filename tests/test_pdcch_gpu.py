"""GPU parity: the MI355X PDCCH processor (pdcch_crc_kernel, the polar encoder, pdcch_map_kernel) through the C-ABI
vs the compiled reference pdcch_processor_impl (oracle/ref_wrapper_pdcch.cpp) and the CPU restatement
(oracle/pdcch.py, itself bit-exact with the reference: tests/test_oracle_vs_ref.py).  Bar: every cbf16 RE of the
grid bit-exact, every other RE untouched."""
import numpy as np
import pytest

from oracle import pdcch as op
from tests.pdcch_cases import INVALID, cases, slot_pdus

pytestmark = pytest.mark.gpu

CASES = cases()


@pytest.fixture(scope="module")
def proc():
    from srsran_project_amd.pdcch import PdcchProcessor

    return PdcchProcessor(device=0)


def _grid(seed, ports, nsubc):
    g = np.random.default_rng(seed).integers(0, 2**32, (ports, 14, nsubc), dtype=np.uint64)
    return g.astype(np.uint32)


@pytest.mark.parametrize("idx", range(len(CASES)), ids=[c[0] for c in CASES])
def test_pdcch_process_host_grid(proc, idx):
    """pdcch_processor::process of one PDU onto a host grid (with one more port than the PDU precodes onto)."""
    name, pdu = CASES[idx]
    c = pdu.coreset
    nsubc = 12 * min(c.bwp_start_rb + c.bwp_size_rb + 3, 275)
    g0 = _grid(idx, pdu.dci.nof_ports + 1, nsubc)
    want = op.ref_process(g0.copy(), [pdu])
    got = proc.process(g0.copy(), pdu)
    assert np.array_equal(got, want), (name, np.argwhere(got != want)[:5])
    assert np.array_equal(op.process(g0.copy(), pdu), want), name


def test_pdcch_process_slot_many_dci_many_grids(proc):
    """The slot form: 5 DCIs per grid (two CORESETs, every mapping kind but CORESET0, four polar codes) on 3 device
    grids in one call, against the reference processing each grid's PDUs in order."""
    import torch

    nsubc, ngrids = 12 * 106, 3
    pdus = slot_pdus(ngrids, nsubc)
    g0 = np.stack([_grid(40 + g, 2, nsubc) for g in range(ngrids)])
    d = torch.from_numpy(g0.view(np.int32).copy()).cuda()
    proc.process_slot(d, pdus)
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32)
    for g in range(ngrids):
        want = op.ref_process(g0[g].copy(), [p for p in pdus if p.grid == g])
        assert np.array_equal(got[g], want), (g, np.argwhere(got[g] != want)[:5])


def test_pdcch_process_slot_every_case_one_call(proc):
    """Every case PDU on its own grid, one slot call (mixed AL, K, E, port counts, mappings and slots)."""
    import torch

    nsubc = 12 * 275
    pdus = []
    for i, (_, p) in enumerate(CASES):
        p.grid = i
        pdus.append(p)
    g0 = np.stack([_grid(80 + i, 4, nsubc) for i in range(len(pdus))])
    d = torch.from_numpy(g0.view(np.int32).copy()).cuda()
    proc.process_slot(d, pdus)
    torch.cuda.synchronize()
    got = d.cpu().numpy().view(np.uint32)
    for i, p in enumerate(pdus):
        want = op.ref_process(g0[i].copy(), [p])
        assert np.array_equal(got[i], want), (CASES[i][0], np.argwhere(got[i] != want)[:5])
        p.grid = 0


def test_pdcch_process_slot_own_device_grid(proc):
    """A PDU carrying its own device grid pointer (d_grid) instead of an index."""
    import torch

    name, pdu = CASES[1]
    nsubc = 12 * (pdu.coreset.bwp_start_rb + pdu.coreset.bwp_size_rb)
    g0 = _grid(5, pdu.dci.nof_ports, nsubc)
    d = torch.from_numpy(g0.view(np.int32).copy()).cuda()
    pdu.d_grid = d.data_ptr()
    try:
        proc.process_slot(torch.zeros((1, 1, 14, nsubc), dtype=torch.int32, device="cuda"), [pdu])
    finally:
        pdu.d_grid = None
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().view(np.uint32), op.ref_process(g0.copy(), [pdu])), name


def test_pdcch_invalid_pdu_fails_loudly(proc):
    from srsran_project_amd.pdcch import make_pdu

    for name, kw, text in INVALID:
        with pytest.raises(ValueError, match=text):
            proc.process(np.zeros((1, 14, 12 * 52), np.uint32), make_pdu(np.ones(20, np.uint8), **kw))

"""GPU parity: MI355X PDSCH modulator (scrambling + modulation + layer mapping +
precoding + RE mapping in one kernel) and PDSCH DM-RS processor, through the
C-ABI, vs the CPU oracle oracle/pdsch_mod.py (itself bit-exact with the
reference's pdsch_modulator_impl / dmrs_pdsch_processor_impl on the generic,
AVX2 and AVX512 precoders, tests/test_oracle_vs_ref.py).  Bar: every bf16 RE of
the grid bit-exact, untouched REs preserved."""
import numpy as np
import pytest

from oracle import pdsch_mod as pm
from tests.pdsch_cases import DMRS_CASES, MOD_CASES, dmrs_case, mod_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mod():
    import srsran_project_amd as amd

    return amd.PdschModulator(device=0)


def _config(kw):
    import srsran_project_amd as amd

    res = [amd.ReservedPattern(list(np.nonzero(cm)[0]), rm, sm) for cm, rm, sm in kw["reserved"]]
    return amd.PdschModulatorConfig(rnti=kw["rnti"], bwp_start=kw["bwp"][0], bwp_size=kw["bwp"][1], modulation=kw["qm"],
                                    crbs=list(kw["crbs"]), start_symbol=kw["start_symbol"],
                                    nof_symbols=kw["nof_symbols"], dmrs_symb_pos=kw["dmrs_symb_mask"],
                                    dmrs_type=2 if kw["dmrs_type2"] else 1,
                                    nof_cdm_groups_without_data=kw["nof_cdm_groups_without_data"], n_id=kw["n_id"],
                                    scaling=kw["scaling"], reserved=res, precoding=kw["weights"])


def _as_u32(g16):
    return np.ascontiguousarray(g16).view(np.uint32).reshape(g16.shape[:3]).copy()


@pytest.mark.parametrize("case", MOD_CASES, ids=[c[0] for c in MOD_CASES])
def test_pdsch_modulate_host(mod, case):
    grid0, bits, kw = mod_case(case, seed=3)
    want = pm.pdsch_modulate(grid0.copy(), bits, **kw)
    got = mod.modulate(_as_u32(grid0), np.packbits(bits), _config(kw))
    np.testing.assert_array_equal(got, _as_u32(want))


def test_pdsch_modulate_batch(mod):
    import torch

    case = MOD_CASES[3]  # 273 PRB, 256QAM, 4 layers, 4 ports
    grid0, bits, kw = mod_case(case, seed=5)
    n = 3
    rng = np.random.default_rng(9)
    cws = [rng.integers(0, 2, bits.size).astype(np.uint8) for _ in range(n)]
    plan = mod.plan(_config(kw), grid0.shape[2])
    assert plan.nof_bits == bits.size
    stride = (bits.size // 8 + 64) // 64 * 64
    cw_dev = torch.zeros((n, stride), dtype=torch.uint8)
    for i in range(n):
        cw_dev[i, :bits.size // 8] = torch.from_numpy(np.packbits(cws[i]))
    g = np.stack([_as_u32(grid0)] * n)
    g_dev = torch.from_numpy(g.view(np.int32)).to("cuda:0")
    mod.modulate_batch(g_dev, cw_dev.to("cuda:0"), plan)
    torch.cuda.synchronize()
    got = g_dev.cpu().numpy().view(np.uint32)
    for i in range(n):
        want = pm.pdsch_modulate(grid0.copy(), cws[i], **kw)
        np.testing.assert_array_equal(got[i], _as_u32(want), err_msg="codeword %d" % i)


def test_pdsch_modulate_rejects_wrong_length(mod):
    grid0, bits, kw = mod_case(MOD_CASES[0], seed=1)
    plan = mod.plan(_config(kw), grid0.shape[2])
    g = _as_u32(grid0)
    cw = np.packbits(bits)
    # not a whole number of REs (QPSK, one layer: an odd bit count): rejected, as the reference's assertion
    rc = mod._lib.srs_amd_pdsch_modulate(mod._h, plan._h, g.ctypes.data, 1, cw.ctypes.data, plan.nof_bits - 1)
    assert rc == -1  # SRS_AMD_EINVAL
    # a whole number of REs shorter than the allocation: accepted, its first REs mapped (the reference's mapper)
    rc = mod._lib.srs_amd_pdsch_modulate(mod._h, plan._h, g.ctypes.data, 1, cw.ctypes.data, plan.nof_bits - 2)
    assert rc == 0


def _dmrs_config(kw):
    import srsran_project_amd as amd

    return amd.DmrsPdschConfig(slot_index=kw["slot_index"], reference_point_k_rb=kw["reference_point_k_rb"],
                               type=2 if kw["dmrs_type2"] else 1, scrambling_id=kw["scrambling_id"],
                               n_scid=kw["n_scid"], amplitude=kw["amplitude"], symbols_mask=kw["symbols_mask"],
                               crbs=list(kw["crbs"]), precoding=kw["weights"][0])


@pytest.mark.parametrize("case", DMRS_CASES, ids=[c[0] for c in DMRS_CASES])
def test_dmrs_pdsch_host(mod, case):
    grid0, kw = dmrs_case(case, seed=4)
    want = pm.dmrs_pdsch_map(grid0.copy(), **kw)
    got = mod.map_dmrs(_as_u32(grid0), _dmrs_config(kw))
    np.testing.assert_array_equal(got, _as_u32(want))


def test_dmrs_pdsch_batch(mod):
    import torch

    grid0, kw = dmrs_case(DMRS_CASES[2], seed=6)
    n = 2
    g_dev = torch.from_numpy(np.stack([_as_u32(grid0)] * n).view(np.int32)).to("cuda:0")
    mod.map_dmrs_batch(g_dev, _dmrs_config(kw))
    torch.cuda.synchronize()
    want = _as_u32(pm.dmrs_pdsch_map(grid0.copy(), **kw))
    got = g_dev.cpu().numpy().view(np.uint32)
    for i in range(n):
        np.testing.assert_array_equal(got[i], want)


# Four PDSCH PDUs of one 273-PRB, four-port slot on disjoint CRBs: (qm, layers, crbs, start, nof_symbols,
# dmrs mask, type 2, CDM groups without data, reserved, scaling)
SLOT_PDUS = [
    (2, 1, (0, 60), 0, 14, (1 << 2) | (1 << 11), False, 2, [], 1.0),
    (6, 2, (60, 140), 1, 13, (1 << 2) | (1 << 7) | (1 << 11), False, 1, [((70, 90), 0b000100010001, 1 << 9)], 0.7),
    (4, 3, (140, 200), 2, 12, (1 << 3) | (1 << 4), True, 2, [], 1.0),
    (8, 4, "sparse", 0, 14, 1 << 2, False, 2, [], 1.3),
]


def _slot_pdus(seed=11):
    from tests.pdsch_cases import _reserved

    rng = np.random.default_rng(seed)
    nprb, P = 273, 4
    bwp = np.zeros(pm.MAX_RB, bool)
    bwp[:nprb] = True
    out = []
    for i, (qm, L, crbs, start, ns, dmrs, t2, ncdm, res, scaling) in enumerate(SLOT_PDUS):
        crbs = (np.sort(rng.choice(np.arange(200, 273), 50, replace=False)) if crbs == "sparse"
                else np.arange(*crbs))
        reserved = _reserved(res, nprb)
        mask = pm.data_re_mask(12 * nprb, crbs, start, ns, reserved + [(bwp, pm.dmrs_prb_mask(t2, ncdm), dmrs)])
        bits = rng.integers(0, 2, int(mask.sum()) * L * qm).astype(np.uint8)
        W = ((rng.normal(size=(L, P)) + 1j * rng.normal(size=(L, P))) / np.sqrt(2 * P)).astype(np.complex64)
        kw = dict(rnti=int(rng.integers(1, 65520)), n_id=int(rng.integers(0, 1024)), qm=qm, crbs=crbs,
                  start_symbol=start, nof_symbols=ns, dmrs_symb_mask=dmrs, dmrs_type2=t2,
                  nof_cdm_groups_without_data=ncdm, reserved=reserved, weights=W, scaling=scaling, bwp=(0, nprb))
        dkw = dict(slot_index=7, reference_point_k_rb=0, dmrs_type2=t2, scrambling_id=int(rng.integers(0, 65536)),
                   n_scid=i % 2, amplitude=float(rng.uniform(0.5, 2.0)), symbols_mask=dmrs, crbs=crbs,
                   weights=W[None])
        out.append((bits, kw, dkw))
    grid0 = rng.integers(0, 1 << 16, (P, 14, 12 * nprb, 2)).astype(np.uint16)
    return grid0, out


def test_pdsch_modulate_slot_4pdu_vs_reference(mod):
    """four PDSCH PDUs (own CRBs, symbols, layers, Qm, precoding, reserved REs, DM-RS type /
    scrambling) of one grid in one slot call (two launches) against the reference pdsch_modulator_impl and
    dmrs_pdsch_processor_impl called once per PDU on the same grid: every RE bit-exact, untouched REs kept."""
    import torch

    grid0, pdus = _slot_pdus()
    want = grid0.copy()
    for bits, kw, dkw in pdus:
        pm.ref_pdsch_modulate(want, bits, **kw)
        pm.ref_dmrs_pdsch_map(want, **dkw)
    items = [(mod.plan(_config(kw), grid0.shape[2]), _dmrs_config(dkw), 0, np.packbits(bits))
             for bits, kw, dkw in pdus]
    g = torch.from_numpy(_as_u32(grid0)[None].view(np.int32)).to("cuda:0")
    mod.modulate_slot(g, items)
    got = g.cpu().numpy().view(np.uint32)[0]
    np.testing.assert_array_equal(got, _as_u32(want))


def test_pdsch_modulate_slot_several_grids(mod):
    """PDUs spread over two grids (grid index per PDU), data-only and DM-RS-only PDUs, against the batch forms."""
    import torch

    grid0, pdus = _slot_pdus(seed=12)
    base = np.stack([_as_u32(grid0)] * 2)
    items, want = [], base.copy()
    for i, (bits, kw, dkw) in enumerate(pdus):
        gi = i % 2
        plan = mod.plan(_config(kw), grid0.shape[2])
        dm = _dmrs_config(dkw) if i != 1 else None
        items.append((plan if i != 2 else None, dm, gi, np.packbits(bits)))
        w = torch.from_numpy(want[gi:gi + 1].view(np.int32)).to("cuda:0")
        if i != 2:
            cw = torch.from_numpy(np.packbits(bits)[None]).to("cuda:0")
            mod.modulate_batch(w, cw, plan)
        if dm is not None:
            mod.map_dmrs_batch(w, dm)
        torch.cuda.synchronize()
        want[gi] = w.cpu().numpy().view(np.uint32)[0]
    g = torch.from_numpy(base.view(np.int32)).to("cuda:0")
    mod.modulate_slot(g, items)
    np.testing.assert_array_equal(g.cpu().numpy().view(np.uint32), want)

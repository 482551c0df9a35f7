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
    rc = mod._lib.srs_amd_pdsch_modulate(mod._h, plan._h, g.ctypes.data, 1, cw.ctypes.data, plan.nof_bits - 2)
    assert rc == -1  # SRS_AMD_EINVAL, as the reference's assertion


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

"""GPU parity: MI355X PUSCH DM-RS channel estimator (through the C-ABI) vs the
CPU oracle oracle/chest.py, itself pinned to the reference's
dmrs_pusch_estimator_impl + port_channel_estimator_average_impl
(tests/test_oracle_vs_ref.py) -- and vs the compiled reference directly when
oracle/_ref is present.  Bar (float path, sums reassociated): every bf16
estimate within two bf16 roundings (2^-6 relative) of the oracle's, stale REs
bit-exact; noise variance, EPRE, RSRP, SNR, CFO within 2e-3 relative; time
alignment within 2e-3 relative + 2 ns."""
import numpy as np
import pytest

import oracle
from oracle import chest
from tests import chest_cases as cc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def est():
    import srsran_project_amd as amd

    return amd.DmrsPuschEstimator(device=0)


def _config(kw):
    import srsran_project_amd as amd

    return amd.DmrsPuschEstimatorConfig(slot_index=kw["slot_index"], numerology=kw["numerology"],
                                        nof_tx_layers=kw["nof_layers"], scrambling_id=kw["scrambling_id"],
                                        n_scid=kw["n_scid"], scaling=kw["scaling"], symbols_mask=kw["symbols_mask"],
                                        rb_start=kw["prb_lo"], rb_count=kw["prb_hi"] - kw["prb_lo"],
                                        first_symbol=kw["first_symbol"], nof_symbols=kw["nof_symbols"],
                                        fd_smoothing=kw["fd"], td_interpolation=kw["td"],
                                        compensate_cfo=kw["compensate_cfo"])


@pytest.mark.parametrize("case", cc.CASES, ids=[c[0] for c in cc.CASES])
def test_pusch_chest_host(est, case):
    grid, kw = cc.case_args(case, seed=5)
    est0 = cc.stale_estimates(grid.shape, kw["nof_layers"], seed=7)
    want, ws = chest.pusch_chest(grid, estimates=est0, **kw)
    got, gs = est.estimate(grid, _config(kw), estimates=est0)
    cc.assert_estimates_close(got, want, case[0])
    cc.assert_stats_close(gs, ws, case[0])
    if oracle.REF is not None:
        want_r, ws_r = chest.ref_pusch_chest(grid, estimates=est0, **kw)
        cc.assert_estimates_close(got, want_r, case[0] + " vs reference")
        cc.assert_stats_close(gs, ws_r, case[0] + " vs reference")


def test_pusch_chest_batch(est):
    import torch

    case = cc.CASES[2]  # 4 rx ports, 273 PRB, 4 layers
    n = 3
    grids, kws = zip(*[cc.case_args(case, seed=s) for s in range(n)])
    kw = dict(kws[0])
    g_dev = torch.from_numpy(np.stack(grids).view(np.int32)).to("cuda:0")
    e0 = np.stack([cc.stale_estimates(grids[0].shape, kw["nof_layers"], seed=11)] * n)
    e_dev = torch.from_numpy(e0.view(np.int32)).to("cuda:0")
    s_dev = torch.zeros((n, grids[0].shape[0], 6), dtype=torch.float32, device="cuda:0")
    est.estimate_batch(g_dev, _config(kw), e_dev, s_dev)
    torch.cuda.synchronize()
    got = e_dev.cpu().numpy().view(np.uint32)
    st = s_dev.cpu().numpy()
    keys = ["noise_var", "epre", "rsrp", "snr", "time_alignment_s", "cfo_hz"]
    for i in range(n):
        want, ws = chest.pusch_chest(grids[i], estimates=e0[i], **kw)
        cc.assert_estimates_close(got[i], want, "grid %d" % i)
        cc.assert_stats_close([dict(zip(keys, row)) for row in st[i]], ws, "grid %d" % i)


def test_pusch_chest_rejects_unsupported(est):
    import srsran_project_amd as amd

    grid, kw = cc.case_args(cc.CASES[0], seed=1)
    cfg = _config(kw)
    cfg.symbols_mask = 0
    with pytest.raises(ValueError):
        est.estimate(grid, cfg)
    cfg = _config(kw)
    cfg.nof_tx_layers = 5
    with pytest.raises(ValueError):
        est.estimate(grid, cfg)


# Transform precoding: the low-PAPR DM-RS sequence (one layer), against the compiled reference estimator
# configured with low_papr_sequence_configuration (dmrs_pusch_estimator_impl.cpp:86-92).
# (name, ports, nof_prb, rb_start, rb_count, dmrs mask, td, n_rs_id)
LP_CASES = [
    ("lp_1rb_M6", 1, 25, 3, 1, (1 << 2) | (1 << 11), 1, 5),
    ("lp_5rb_M30", 2, 52, 10, 5, (1 << 2) | (1 << 11), 1, 77),
    ("lp_25rb_M150_interp", 4, 52, 20, 25, (1 << 2) | (1 << 7) | (1 << 11), 0, 1007),
    ("lp_270rb_M1620", 2, 273, 2, 270, 1 << 2, 1, 301),
]


@pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("case", LP_CASES, ids=[c[0] for c in LP_CASES])
def test_pusch_chest_low_papr_vs_reference(est, case):
    name, P, nprb, lo, cnt, mask, td, n_rs_id = case
    grid = cc.make_grid(P, nprb, 0.05, seed=cnt)
    kw = dict(slot_index=4, type2=2, nof_layers=1, scrambling_id=n_rs_id, n_scid=0, scaling=1.41, symbols_mask=mask,
              prb_lo=lo, prb_hi=lo + cnt, first_symbol=0, nof_symbols=14, fd=2, td=td, compensate_cfo=True,
              numerology=1)
    est0 = cc.stale_estimates(grid.shape, 1, seed=3)
    want, ws = chest.ref_pusch_chest(grid, estimates=est0, **kw)
    cfg = _config(dict(kw, scrambling_id=0))
    cfg.low_papr, cfg.n_rs_id = True, n_rs_id
    got, gs = est.estimate(grid, cfg, estimates=est0)
    cc.assert_estimates_close(got, want, name)
    cc.assert_stats_close(gs, ws, name)


def test_pusch_chest_low_papr_rejects(est):
    grid = cc.make_grid(1, 52, 0.05, seed=0)
    kw = dict(slot_index=0, type2=False, nof_layers=2, scrambling_id=0, n_scid=0, scaling=1.41, symbols_mask=1 << 2,
              prb_lo=0, prb_hi=7, first_symbol=0, nof_symbols=14, fd=2, td=1, compensate_cfo=True, numerology=1)
    cfg = _config(kw)
    cfg.low_papr = True
    with pytest.raises(ValueError):  # two layers
        est.estimate(grid, cfg)
    cfg.nof_tx_layers = 1
    with pytest.raises(ValueError):  # 7 PRB: no low-PAPR sequence of length 42
        est.estimate(grid, cfg)

"""End-to-end parity of the MI355X slot pipeline (bench_pipeline.Pipeline: PDSCH
encode -> modulate -> DM-RS -> OFDM modulate; OFDM demodulate -> PUSCH
processor) against the REFERENCE's own CPU chain on the same inputs
(oracle/ref_chain.cpp: pdsch_encoder_impl, pdsch_modulator_impl,
dmrs_pdsch_processor_impl, ofdm_slot_modulator_impl, ofdm_slot_demodulator_impl,
pusch_processor_impl with the "auto" factory implementations), stage by stage:

  DL resource grid          bit-exact
  DL baseband               max |error| <= 3e-5 x RMS (two float DFTs, each ~1e-6..2e-5 x RMS of exact)
  UL resource grid          the reference ofdm_slot_demodulator on the same samples: bf16 within 1 ulp
                            (+ 3e-5 x RMS absolute, the two float DFTs' error near zero), >= 99 % identical
  UL channel estimates      the reference dmrs_pusch_estimator on the GPU's UL grid: the estimator
                            tolerances of tests/chest_cases.py (two bf16 roundings; stats 2e-3)
  UL codeword LLRs          the reference pusch_demodulator on the GPU's grid and estimates:
                            |dLLR| <= 1, >= 99 % identical (float equalizer)
  UL transport blocks       the reference chain's decoded TB bytes and TB CRC flag: identical, and equal
                            to what the UE sent
The 4-layer PUSCH of the default bench line (MMSE 4 x 4; the open reference's equalizer asserts for it) is
checked stage by stage against the pinned reference stages where they exist (OFDM demodulator, DM-RS
estimator with four layers) and against the restated demodulator with the fp64 4 x 4 solve (PARITY UNPINNED
equalizer), and its transport blocks must equal what the UE sent.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


# (name, Pipeline keyword arguments, cells, cells checked stage by stage): the headline's PDSCH 4 x 4 with the
# reference-runnable 2-layer PUSCH (the reference chain runs PUSCH with at most 2 layers), configs[3] as stated
# (PDSCH 2 layers x 2 ports, PUSCH 2 layers x 2 rx ports), and the bench batch of 64 cells (the headline's
# cross-cell indexing at its own size: every cell's DL grid and TB against the reference chain, three cells stage by
# stage) -- the pinned sibling line of bench.py runs exactly this 64-cell batch
CHAIN_CASES = [
    ("dl4x4_ul2x4", dict(ul_layers=2), 2, (0, 1)),
    ("2x2", dict(dl_layers=2, dl_ports=2, ul_layers=2, ul_ports=2), 2, (0, 1)),
    ("dl4x4_ul2x4_64cells", dict(ul_layers=2), 64, (0, 31, 63)),
]


def _bf16(u16):
    return (np.asarray(u16, np.uint32) << 16).view(np.float32)


@pytest.mark.parametrize("case", CHAIN_CASES, ids=[c[0] for c in CHAIN_CASES])
def test_pipeline_vs_reference_chain(case):
    import torch

    import bench_pipeline as bp
    import oracle
    from oracle import chain as oc
    from oracle import chest as och
    from oracle import pusch_demod as od
    from tests.chest_cases import assert_estimates_close, assert_stats_close
    from tests.pusch_demod_cases import assert_llrs_close

    _, kw, cells, staged = case
    dev = torch.device("cuda", 0)
    pl = bp.Pipeline(cells, dev, keep_estimates=True, **kw)
    stream = torch.cuda.current_stream(dev)
    pl.step(stream)
    torch.cuda.synchronize(dev)
    cfg = bp.chain_config(pl)
    n = oc.slot_size(cfg)
    res = pl.results()
    for c in range(pl.S):
        tb_dl = pl.tb_dl[c].cpu().numpy()
        samp_ul = pl.samp_ul[c, :, :n].cpu().numpy()
        grid_ref, samp_ref, tb_ref, ok_ref, it_ref = oc.run(cfg, tb_dl, samp_ul)
        # DL grid: bit-exact
        grid = pl.grid_dl[c].cpu().numpy().view(np.uint32)
        assert grid.shape == grid_ref.shape == (pl.dl_ports, 14, bp.NSUBC)
        assert np.array_equal(grid, grid_ref), "cell %d: DL grid differs in %d REs" % (c, int((grid != grid_ref).sum()))
        # UL transport block and CRC
        tb = pl.tb_rx[c].cpu().numpy()
        assert bool(res[c].data.tb_crc_ok) == ok_ref, c
        assert np.array_equal(tb, tb_ref), "cell %d: decoded TB differs from the reference chain" % c
        assert ok_ref and np.array_equal(tb, pl.tb_ul[c].cpu().numpy()), c
        assert res[c].data.ldpc_iterations_sum == it_ref, (c, res[c].data.ldpc_iterations_sum, it_ref)
        if c not in staged:
            continue
        # DL baseband
        samp = pl.samp_dl[c, :, :n].cpu().numpy()
        rms = np.sqrt(np.mean(np.abs(samp_ref) ** 2))
        err = np.max(np.abs(samp - samp_ref))
        assert err <= 3e-5 * rms, "cell %d: DL baseband max error %.3g x RMS" % (c, err / rms)
        # UL grid (OFDM demodulator)
        gul = pl.grid_ul[c].cpu().numpy().view(np.uint32)
        for p in range(pl.ul_ports):
            ref = oracle.ref_ofdm_demodulate_slot(samp_ul[p], bp.SLOT, bp.MU, bp.NPRB, bp.NFFT, 1.0, 3.5e9)
            ref = ref.view(np.uint32).reshape(14, bp.NSUBC)
            same = gul[p] == ref
            a, b = _bf16(gul[p].view(np.uint16)), _bf16(ref.view(np.uint16))
            rms = np.sqrt(np.mean(b ** 2))
            tol = 2.0 ** -7 * np.maximum(np.abs(a), np.abs(b)) + 3e-5 * rms  # 1 ulp: 2^(e-7) for |x| in [2^e, 2^(e+1))
            bad = ~(np.abs(a - b) <= tol)
            assert not bad.any(), "cell %d port %d: %d UL REs beyond 1 bf16 ulp, e.g. %s" % (
                c, p, int(bad.sum()), [(int(i), int(j), float(a[i, j]), float(b[i, j]))
                                       for i, j in zip(*np.nonzero(bad))][:6])
            assert same.mean() >= 0.99, "cell %d port %d: UL grid only %.5f identical" % (c, p, same.mean())
        # UL channel estimates on the GPU's grid
        est = pl.est_ul[c].cpu().numpy().view(np.uint32)
        est_ref, st_ref = och.ref_pusch_chest(gul, bp.SLOT, False, pl.ul_layers, bp.N_ID, 0, bp.DMRS_AMP, bp.DMRS_MASK,
                                              0, bp.NPRB, bp.UL_START, bp.UL_NSYM, fd=2, td=pl.ul_td, compensate_cfo=True,
                                              numerology=bp.MU)
        assert_estimates_close(est, est_ref, "cell %d estimates" % c)
        st = pl.stats_ul[c].cpu().numpy()
        got_st = [dict(zip(("noise_var", "epre", "rsrp", "snr", "time_alignment_s", "cfo_hz"), row)) for row in st]
        assert_stats_close(got_st, st_ref, "cell %d stats" % c)
        # UL LLRs on the GPU's grid and estimates
        G = pl.plan_ul.cw_length
        llr = pl.llr_ul[c, :G].cpu().numpy()
        want = od.ref_pusch_demodulate(gul, est, st[:, 0], bp.RNTI, bp.N_ID, bp.QM, list(range(bp.NPRB)),
                                       bp.UL_START, bp.UL_NSYM, bp.DMRS_MASK, False, bp.NCDM, pl.ul_layers)
        assert_llrs_close(llr, want, "cell %d LLRs" % c)


def test_pipeline_four_layer_pusch():
    import torch

    import bench_pipeline as bp
    import oracle
    from oracle import chest as och
    from oracle import pusch_demod as od
    from tests.chest_cases import assert_estimates_close, assert_stats_close
    from tests.pusch_demod_cases import assert_llrs_close

    dev = torch.device("cuda", 0)
    pl = bp.Pipeline(2, dev, ul_layers=4, keep_estimates=True)
    assert pl.ul_equalizer == "mmse"
    stream = torch.cuda.current_stream(dev)
    pl.step(stream)
    torch.cuda.synchronize(dev)
    res = pl.results()
    ok, its = pl.check()
    assert ok == 1.0, ok
    for c in range(pl.S):
        gul = pl.grid_ul[c].cpu().numpy().view(np.uint32)
        samp_ul = pl.samp_ul[c].cpu().numpy()
        for p in range(pl.ul_ports):
            ref = oracle.ref_ofdm_demodulate_slot(samp_ul[p], bp.SLOT, bp.MU, bp.NPRB, bp.NFFT, 1.0, 3.5e9)
            same = gul[p] == ref.view(np.uint32).reshape(14, bp.NSUBC)
            assert same.mean() >= 0.99, (c, p, same.mean())
        est = pl.est_ul[c].cpu().numpy().view(np.uint32)
        est_ref, st_ref = och.ref_pusch_chest(gul, bp.SLOT, False, 4, bp.N_ID, 0, bp.DMRS_AMP, bp.DMRS_MASK, 0,
                                              bp.NPRB, bp.UL_START, bp.UL_NSYM, fd=2, td=pl.ul_td, compensate_cfo=True,
                                              numerology=bp.MU)
        assert_estimates_close(est, est_ref, "cell %d estimates" % c)
        st = pl.stats_ul[c].cpu().numpy()
        got_st = [dict(zip(("noise_var", "epre", "rsrp", "snr", "time_alignment_s", "cfo_hz"), row)) for row in st]
        assert_stats_close(got_st, st_ref, "cell %d stats" % c)
        G = pl.plan_ul.cw_length
        llr = pl.llr_ul[c, :G].cpu().numpy()
        want = od.pusch_demodulate(gul, est, st[:, 0], bp.RNTI, bp.N_ID, bp.QM, list(range(bp.NPRB)), bp.UL_START,
                                   bp.UL_NSYM, bp.DMRS_MASK, False, bp.NCDM, 4, mmse=True)
        assert_llrs_close(llr, want, "cell %d LLRs (4 x 4 MMSE)" % c)
        assert res[c].data.tb_crc_ok == 1
        assert np.array_equal(pl.tb_rx[c].cpu().numpy(), pl.tb_ul[c].cpu().numpy()), c


@pytest.mark.parametrize("ul_layers", [2, 4])
def test_pipeline_fused_estimates_identical(ul_layers):
    """The estimator-fused equalizer (no estimate tensor: the bench path) rebuilds every RE's channel
    estimate with the expansion kernel's own operations, so its LLRs, transport blocks and results are
    bit-identical to the path that writes and re-reads the expanded estimates."""
    import torch

    import bench_pipeline as bp

    dev = torch.device("cuda", 0)
    out = []
    for keep in (True, False):
        pl = bp.Pipeline(2, dev, ul_layers=ul_layers, keep_estimates=keep)
        stream = torch.cuda.current_stream(dev)
        pl.step(stream)
        torch.cuda.synchronize(dev)
        G = pl.plan_ul.cw_length
        out.append((pl.llr_ul[:, :G].cpu().numpy(), pl.tb_rx.cpu().numpy(), pl.res_ul.cpu().numpy(),
                    pl.stats_ul.cpu().numpy()))
        del pl
    for a, b, what in zip(out[0], out[1], ("LLRs", "transport blocks", "results", "port stats")):
        assert np.array_equal(a, b), what

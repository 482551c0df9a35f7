"""GPU parity: the MI355X UL-SCH demultiplexer (include/srsran_amd/ulsch_demux.h) against the compiled reference
ulsch_demultiplex_impl on random descrambled codewords: the UL-SCH, HARQ-ACK and CSI part 1 streams bit-exact,
over HARQ-ACK payloads of 1 and 2 bits (reserved REs, placeholders x / y, zeroed UL-SCH copies) and of 3-40 bits,
CSI part 1 payloads of 1-2 bits (placeholders) and more, DM-RS types / CDM groups, 1-4 layers, every
modulation; geometry from srs_amd_ulsch_information as the reference processor derives it.  With CSI part 2 (1-2-bit
placeholders and longer, sharing reserved REs with 1/2-bit HARQ-ACK): the reference demultiplexer configured with
set_csi_part2 when its CSI part 1 stream ends, as its PUSCH processor does."""
import numpy as np
import pytest

import oracle
from oracle import pusch_proc as pp

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")]


def _cases(n, seed, csi2=False):
    import srsran_project_amd as amd

    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        qm = int(rng.choice([1, 2, 4, 6, 8]))
        layers = 1 if qm == 1 else int(rng.integers(1, 5))
        t2 = bool(rng.integers(2))
        start = int(rng.integers(0, 3))
        nsym = int(rng.integers(5, 15 - start))
        first = start + int(rng.integers(0, 2))
        mask = 1 << first
        if rng.integers(2) and first + 7 < start + nsym:
            mask |= 1 << (first + 7)
        nrb = int(rng.integers(1, 60))
        ack = int(rng.choice([0, 1, 2, 3, 6, 11, 17, 40]))
        csi1 = int(rng.choice([0, 1, 2, 9, 30]))
        part2 = int(rng.choice([1, 2, 5, 12, 40])) if csi2 else 0
        if (ack == 0 and csi1 == 0) or (csi2 and csi1 == 0):
            continue
        rate = 400.0
        tbs = amd.tbs_calculator_calculate(nsym, 6 * bin(mask).count("1"), 0, max(qm, 2), rate, layers, 0, nrb)
        cfg = amd.UlschConfig(tbs=tbs, modulation=qm, target_code_rate=rate, nof_harq_ack_bits=ack,
                              nof_csi_part1_bits=csi1, nof_csi_part2_bits=part2, alpha_scaling=1.0,
                              beta_offset_csi_part2=float(rng.choice([2.0, 5.0])),
                              beta_offset_harq_ack=float(rng.choice([2.0, 8.0])),
                              beta_offset_csi_part1=float(rng.choice([2.0, 5.0])), nof_rb=nrb, start_symbol_index=start,
                              nof_symbols=nsym, dmrs_type=2 if t2 else 1, dmrs_symbol_mask=mask,
                              nof_cdm_groups_without_data=int(rng.integers(1, 4 if t2 else 3)), nof_layers=layers)
        try:
            info = amd.ulsch_information(cfg)
        except Exception:
            continue  # the UCI does not fit this allocation
        out.append((cfg, info, int(rng.integers(0, 1 << 31))))
    return out


def test_ulsch_demultiplex_matches_reference():
    import srsran_project_amd as amd

    dm = amd.UlschDemux(device=0)
    rng = np.random.default_rng(4)
    for cfg, info, c_init in _cases(120, 7):
        dc = amd.UlschDemuxConfig(cfg.modulation, cfg.nof_layers, cfg.nof_rb, cfg.start_symbol_index, cfg.nof_symbols,
                                  info["nof_harq_ack_rvd"], cfg.dmrs_type, cfg.dmrs_symbol_mask,
                                  cfg.nof_cdm_groups_without_data, cfg.nof_harq_ack_bits, info["nof_harq_ack_bits"],
                                  cfg.nof_csi_part1_bits, info["nof_csi_part1_bits"], c_init)
        plan = dm.plan(dc)
        llrs = rng.integers(-127, 128, plan.nof_codeword_bits).astype(np.int8)
        got = dm.demultiplex(llrs, plan)
        want = pp.ref_ulsch_demultiplex(llrs, cfg.modulation, cfg.nof_layers, cfg.nof_rb, cfg.start_symbol_index,
                                        cfg.nof_symbols, info["nof_harq_ack_rvd"], cfg.dmrs_type == 2,
                                        cfg.dmrs_symbol_mask, cfg.nof_cdm_groups_without_data, cfg.nof_harq_ack_bits,
                                        info["nof_harq_ack_bits"], cfg.nof_csi_part1_bits, info["nof_csi_part1_bits"],
                                        c_init)
        assert plan.nof_sch_bits == info["nof_ul_sch_bits"], (cfg.as_dict(), info)
        for g, w, what in zip(got, want, ("sch", "ack", "csi1")):
            np.testing.assert_array_equal(g, w, err_msg="%s %s" % (what, cfg.as_dict()))


def test_ulsch_demultiplex_csi_part2_matches_reference():
    import srsran_project_amd as amd

    dm = amd.UlschDemux(device=0)
    rng = np.random.default_rng(5)
    for cfg, info, c_init in _cases(80, 11, csi2=True):
        dc = amd.UlschDemuxConfig(cfg.modulation, cfg.nof_layers, cfg.nof_rb, cfg.start_symbol_index, cfg.nof_symbols,
                                  info["nof_harq_ack_rvd"], cfg.dmrs_type, cfg.dmrs_symbol_mask,
                                  cfg.nof_cdm_groups_without_data, cfg.nof_harq_ack_bits, info["nof_harq_ack_bits"],
                                  cfg.nof_csi_part1_bits, info["nof_csi_part1_bits"], c_init, cfg.nof_csi_part2_bits,
                                  info["nof_csi_part2_bits"])
        plan = dm.plan(dc)
        llrs = rng.integers(-127, 128, plan.nof_codeword_bits).astype(np.int8)
        got = dm.demultiplex(llrs, plan)
        want = pp.ref_ulsch_demultiplex2(llrs, cfg.modulation, cfg.nof_layers, cfg.nof_rb, cfg.start_symbol_index,
                                         cfg.nof_symbols, info["nof_harq_ack_rvd"], cfg.dmrs_type == 2,
                                         cfg.dmrs_symbol_mask, cfg.nof_cdm_groups_without_data, cfg.nof_harq_ack_bits,
                                         info["nof_harq_ack_bits"], cfg.nof_csi_part1_bits, info["nof_csi_part1_bits"],
                                         cfg.nof_csi_part2_bits, info["nof_csi_part2_bits"], c_init)
        assert plan.nof_sch_bits == info["nof_ul_sch_bits"], (cfg.as_dict(), info)
        assert len(got) == 4
        for g, w, what in zip(got, want, ("sch", "ack", "csi1", "csi2")):
            np.testing.assert_array_equal(g, w, err_msg="%s %s" % (what, cfg.as_dict()))

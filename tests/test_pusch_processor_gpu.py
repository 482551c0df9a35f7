"""GPU parity: the MI355X PUSCH processor (DM-RS estimator -> demodulator ->
UL-SCH decoder, through the C-ABI include/srsran_amd/pusch_processor.h) against
the REFERENCE's own pusch_processor_impl (oracle/_ref, ref_wrapper_pusch.cpp)
on the same received grids, configured as the reference PUSCH processor
benchmark (ZF, filter FD smoothing, interpolate TD, CFO compensation, LDPC with
early stop, "auto" CRC / decoder / dematcher).

The UE transmissions are built with the reference's own transmit classes
(oracle/pusch_proc.ue_transmit). configs[0] (20 MHz = 51 PRB at 30 kHz, SISO,
MCS 9 = QPSK R 679/1024) is the first case.
Bars: transport block bytes and TB CRC flag identical; LDPC iteration
statistics identical (SNRs chosen away from the decoding threshold, where the
float estimator/equalizer differences cannot move a decision); CSI within the
estimator tolerances (SINR/EPRE/RSRP 0.05 dB, time alignment 2 ns).
"""
import numpy as np
import pytest

import srsran_project_amd as amd
from oracle import pusch_proc as pp

pytestmark = pytest.mark.gpu

BASE = dict(numerology=1, slot_index=0, rnti=1, bwp_start_rb=0, bwp_size_rb=51, modulation=2,
            target_code_rate=679.0, rv=0, base_graph=1, new_data=1, n_id=0, nof_tx_layers=1, nof_rx_ports=1,
            dmrs_symbol_mask=(1 << 2) | (1 << 11), dmrs_type=1, scrambling_id=0, n_scid=0,
            nof_cdm_groups_without_data=2, rb_start=0, rb_count=51, start_symbol_index=0, nof_symbols=14)

H42 = np.array([[1.0, 0.2j, 0.7 + 0.1j, 0.3], [0.1, 0.9, -0.2j, 0.8 - 0.2j]], np.complex64) * np.float32(0.8)

# (name, pdu overrides, grid PRBs, channel [L][P] or None, SNR dB, LDPC iterations)
CASES = [
    ("configs0_51prb_siso_mcs9", {}, 51, None, 20.0, 2),
    ("51prb_siso_mcs9_low_snr", {}, 51, None, 6.0, 6),
    ("bwp_part_2rx_16qam", dict(bwp_start_rb=10, bwp_size_rb=40, rb_start=5, rb_count=20, modulation=4,
                                target_code_rate=490.0, nof_rx_ports=2, n_id=77, rnti=0x4601, slot_index=7,
                                scrambling_id=33, nof_cdm_groups_without_data=1, dmrs_symbol_mask=(1 << 2)),
     52, np.array([[0.9, 0.4 - 0.3j]], np.complex64), 22.0, 6),
    ("273prb_4rx_2layer_256qam", dict(bwp_size_rb=273, rb_count=273, modulation=8, target_code_rate=948.0,
                                      nof_tx_layers=2, nof_rx_ports=4, n_id=500, rnti=0x4601),
     273, H42, 35.0, 6),
]


def _tbs(pdu):
    ndmrs = 6 * bin(pdu["dmrs_symbol_mask"]).count("1") * pdu["nof_cdm_groups_without_data"]
    return amd.tbs_calculator_calculate(pdu["nof_symbols"], ndmrs, 0, pdu["modulation"], pdu["target_code_rate"],
                                        pdu["nof_tx_layers"], 0, pdu["rb_count"])


def _check_csi(got, want, what):
    for k in ("sinr_db", "epre_db", "rsrp_db"):
        assert abs(getattr(got, k) - want[k]) <= 0.05, (what, k, getattr(got, k), want[k])
    assert abs(got.time_alignment_s - want["time_alignment_s"]) <= 2e-9, (what, "ta")


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_pusch_processor_vs_reference(case):
    name, over, nprb, ch, snr, iters = case
    pdu = dict(BASE, **over)
    tbs = _tbs(pdu)
    bg = 2 if (tbs <= 292 or (tbs <= 3824 and pdu["target_code_rate"] / 1024 <= 0.67)
               or pdu["target_code_rate"] / 1024 <= 0.25) else 1
    pdu["base_graph"] = bg
    rng = np.random.default_rng(hash(name) % 1000)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    grid, _ = pp.ue_transmit(tb, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=5)
    want_tb, want = pp.ref_pusch_process(grid, pdu, tbs // 8, iterations=iters)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    got_tb, got = proc.process(grid, plan)
    assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], name
    assert np.array_equal(got_tb, want_tb), name
    assert got.data.nof_codeblocks_total == want["nof_codeblocks_total"]
    assert got.data.ldpc_iterations_sum == want["iterations_sum"], (name, got.data.ldpc_iterations_sum, want)
    assert got.data.ldpc_iterations_max == want["iterations_max"]
    _check_csi(got, want, name)
    if snr >= 20:
        assert want["tb_crc_ok"] and np.array_equal(got_tb, tb), name


def test_pusch_processor_harq_combining():
    """rv 0 at an SNR where the TB fails, then rv 2 (new_data = false) with the HARQ soft buffer: the
    combined retransmission decodes, as the reference with its rx_buffer."""
    pdu = dict(BASE, modulation=4, target_code_rate=658.0)
    tbs = _tbs(pdu)
    tb = np.random.default_rng(9).integers(0, 256, tbs // 8, dtype=np.uint8)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    ref_buf = pp.RefRxBuffer(pp.nof_codeblocks(tbs, 1))
    soft = None
    results = []
    for rv, new in ((0, 1), (2, 0)):
        p = dict(pdu, rv=rv, new_data=new)
        grid, _ = pp.ue_transmit(tb, p, 12 * 51, snr_db=8.5, seed=rv + 1)
        want_tb, want = pp.ref_pusch_process(grid, p, tbs // 8, iterations=6, rx_buffer=ref_buf)
        plan = proc.plan(amd.make_pdu(**dict(p, tbs=tbs)), 12 * 51)
        if soft is None:
            soft = np.zeros(plan.soft_bytes, np.int8)
        got_tb, got = proc.process(grid, plan, soft_buffer=soft)
        assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], rv
        if want["tb_crc_ok"]:
            assert np.array_equal(got_tb, want_tb)
        results.append(want["tb_crc_ok"])
    assert results == [False, True], results


def test_pusch_processor_batch_matches_host():
    import torch

    case = CASES[3]
    name, over, nprb, ch, snr, iters = case
    pdu = dict(BASE, **over)
    tbs = _tbs(pdu)
    n = 3
    tbs_in = [np.random.default_rng(i).integers(0, 256, tbs // 8, dtype=np.uint8) for i in range(n)]
    grids = np.stack([pp.ue_transmit(t, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=i)[0]
                      for i, t in enumerate(tbs_in)])
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    g = torch.from_numpy(grids.view(np.int32)).to("cuda:0")
    out, res = proc.process_batch(g, plan)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    res = amd.pusch_processor.parse_results(res.cpu().numpy())
    for i in range(n):
        h_tb, h_res = proc.process(grids[i], plan)
        assert np.array_equal(out[i], h_tb) and np.array_equal(out[i], tbs_in[i])
        assert res[i].data.tb_crc_ok and res[i].data.ldpc_iterations_sum == h_res.data.ldpc_iterations_sum


@pytest.mark.parametrize("td,mask,eq", [(0, (1 << 2) | (1 << 11), 0), (1, (1 << 2) | (1 << 11), 0),
                                         (0, 1 << 2, 1), (0, (1 << 2) | (1 << 7) | (1 << 11), 0)],
                         ids=["interp_2dmrs_zf", "average_2dmrs_zf", "interp_1dmrs_mmse", "interp_3dmrs_zf"])
def test_pusch_processor_fused_equalizer_identical(td, mask, eq):
    """Without a caller estimate buffer the processor fuses the estimate expansion into the equalizer
    (each OFDM symbol reads the one or two LSE slices its time-domain strategy needs): LLRs, transport blocks
    and results are bit-identical to the run that writes the estimates."""
    import torch

    name, over, nprb, ch, snr, iters = CASES[3]
    pdu = dict(BASE, **over, dmrs_symbol_mask=mask)
    tbs = _tbs(pdu)
    tb = np.random.default_rng(3).integers(0, 256, tbs // 8, dtype=np.uint8)
    grids = np.stack([pp.ue_transmit(tb, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=i)[0] for i in range(2)])
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters, td_interpolation=td, equalizer=eq),
                              device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    g = torch.from_numpy(grids.view(np.int32)).to("cuda:0")
    P, L = pdu["nof_rx_ports"], pdu["nof_tx_layers"]
    G = plan.sch.cw_length
    got = []
    for keep in (True, False):
        est = torch.zeros((2, P, L, 14, 12 * nprb), dtype=torch.int32, device="cuda:0") if keep else None
        llrs = torch.zeros((2, (G + 63) // 64 * 64), dtype=torch.int8, device="cuda:0")
        out, res = proc.process_batch(g, plan, estimates=est, llrs=llrs)
        torch.cuda.synchronize()
        got.append((llrs[:, :G].cpu().numpy(), out.cpu().numpy(), res.cpu().numpy()))
    for a, b, what in zip(got[0], got[1], ("LLRs", "transport blocks", "results")):
        assert np.array_equal(a, b), what
    assert all(r.data.tb_crc_ok for r in amd.pusch_processor.parse_results(got[1][2]))
    assert np.array_equal(got[1][1][0], tb)


def _to_complex(g):
    f = np.stack([((g & 0xFFFF) << 16).view(np.float32), ((g >> 16) << 16).view(np.float32)], -1)
    return f[..., 0] + 1j * f[..., 1]


def _from_complex(z):
    from oracle.pdsch_mod import to_bf16
    return np.ascontiguousarray(to_bf16(z.real.astype(np.float32)).astype(np.uint32)
                                | (to_bf16(z.imag.astype(np.float32)).astype(np.uint32) << 16))


def _chan(L, P, seed):
    rng = np.random.default_rng(seed)
    h = np.eye(L, P) + 0.25 * (rng.normal(size=(L, P)) + 1j * rng.normal(size=(L, P)))
    return (0.8 * h).astype(np.complex64)


# Four UEs of one 273-PRB slot on four receive ports, disjoint PRBs, each with its own layers, modulation, code
# rate, DM-RS symbols / CDM groups / scrambling identity / n_SCID, time allocation, rnti and n_id.
SLOT_UES = [
    dict(rnti=0x4601, n_id=1, scrambling_id=11, rb_start=0, rb_count=60, modulation=2, target_code_rate=679.0,
         nof_tx_layers=1),
    dict(rnti=0x4602, n_id=2, scrambling_id=22, n_scid=1, rb_start=60, rb_count=80, modulation=6,
         target_code_rate=567.0, nof_tx_layers=2, dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11)),
    dict(rnti=0x4603, n_id=3, scrambling_id=33, rb_start=140, rb_count=60, modulation=4, target_code_rate=490.0,
         nof_tx_layers=1, nof_cdm_groups_without_data=1, dmrs_symbol_mask=1 << 3, start_symbol_index=1,
         nof_symbols=12),
    dict(rnti=0x4604, n_id=4, scrambling_id=44, rb_start=200, rb_count=73, modulation=4, target_code_rate=378.0,
         nof_tx_layers=2),
]


def _slot_case(slot_index=5, snr=28.0, seed=0, ue3_layers=2):
    pdus, txs = [], []
    z = 0
    for u, over in enumerate(SLOT_UES):
        pdu = dict(BASE, bwp_size_rb=273, nof_rx_ports=4, slot_index=slot_index, **over)
        if u == 3:
            pdu["nof_tx_layers"] = ue3_layers
        tbs = _tbs(pdu)
        pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and pdu["target_code_rate"] / 1024 <= 0.67)
                                  or pdu["target_code_rate"] / 1024 <= 0.25) else 1
        pdu["tbs"] = tbs
        tb = np.random.default_rng(seed * 10 + u).integers(0, 256, tbs // 8, dtype=np.uint8)
        g, _ = pp.ue_transmit(tb, pdu, 12 * 273, channel=_chan(pdu["nof_tx_layers"], 4, 40 + u))
        z = z + _to_complex(g)
        pdus.append(pdu)
        txs.append(tb)
    occ = np.abs(z) > 0
    sigma = np.sqrt(float(np.mean(np.abs(z[occ]) ** 2)) / 10 ** (snr / 10) / 2)
    rng = np.random.default_rng(100 + seed)
    grid = _from_complex(z + sigma * (rng.normal(size=z.shape) + 1j * rng.normal(size=z.shape)))
    return grid, pdus, txs


@pytest.mark.parametrize("eq", [0, 1], ids=["zf", "mmse"])
def test_pusch_slot_4ue_grid_vs_reference(eq):
    """four PUSCH PDUs of one grid through srs_amd_pusch_process_slot (one launch sequence)
    against the reference pusch_processor_impl called once per PDU on the same grid
    (uplink_processor_impl.cpp:270-326): transport blocks, CRC flags and LDPC iteration statistics identical,
    CSI within the estimator tolerances.  The MMSE run (no reference counterpart in the compiled processor)
    gives UE 3 four layers (the 4 x 4 solve) and is pinned to the single-PDU batch form."""
    import torch

    iters = 6
    grid, pdus, txs = _slot_case(ue3_layers=2 if eq == 0 else 4)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters, equalizer=eq), device=0)
    plans = [proc.plan(amd.make_pdu(**p), 12 * 273) for p in pdus]
    g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
    out, offs, res = proc.process_slot(g, [(pl, 0) for pl in plans])
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    res = amd.pusch_processor.parse_results(res.cpu().numpy())
    for u, (pdu, pl) in enumerate(zip(pdus, plans)):
        got_tb = out[offs[u]:offs[u] + pl.tb_bytes]
        if eq == 0:
            want_tb, want = pp.ref_pusch_process(grid, pdu, pl.tb_bytes, iterations=iters)
            assert bool(res[u].data.tb_crc_ok) == want["tb_crc_ok"], u
            assert np.array_equal(got_tb, want_tb), u
            assert res[u].data.nof_codeblocks_total == want["nof_codeblocks_total"], u
            assert res[u].data.ldpc_iterations_sum == want["iterations_sum"], (u, res[u].data.ldpc_iterations_sum,
                                                                                 want)
            assert res[u].data.ldpc_iterations_max == want["iterations_max"], u
            _check_csi(res[u], want, "ue%d" % u)
        assert res[u].data.tb_crc_ok and np.array_equal(got_tb, txs[u]), u
        # per PDU identical to the single-PDU batch form on the same grid
        b_tb, b_res = proc.process_batch(g, pl)
        torch.cuda.synchronize()
        b = amd.pusch_processor.parse_results(b_res.cpu().numpy())[0]
        assert np.array_equal(b_tb[0].cpu().numpy(), got_tb), u
        for k in ("sinr_db", "epre_db", "rsrp_db", "time_alignment_s"):
            assert getattr(b, k) == getattr(res[u], k), (u, k)
        assert b.data.ldpc_iterations_sum == res[u].data.ldpc_iterations_sum, u


def test_pusch_slot_mixed_pdus_vs_reference():
    """one slot call over every PDU kind of a slot -- HARQ-ACK + CSI part 1 on PUSCH, DFT-s-OFDM, a
    HARQ process kept in a device soft buffer (rv 0 new data, then rv 2 retransmission in the next slot) and two
    plain PDUs of the fused group -- on one four-port grid, against the compiled pusch_processor_impl called once
    per PDU on the same grid (the HARQ process with one reference rx_buffer across the two slots): TB bytes, CRC
    flags, LDPC statistics (from the per-codeblock iteration output), CSI, UCI payloads and statuses."""
    import torch

    import oracle
    from pusch_slot_cases import mixed_slot, NSUBC

    iters = 6
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters), device=0)
    ref_buf = soft = None
    for slot_index, rv in ((3, 0), (4, 2)):
        grid, pdus, sent = mixed_slot(slot_index, rv, seed=slot_index)
        plans = [proc.plan(amd.make_pdu(**p), NSUBC) for p in pdus]
        items = []
        for p, pl in zip(pdus, plans):
            if p["rnti"] == 0x5003:  # the HARQ process: its soft buffer lives across the slots
                if soft is None:
                    soft = torch.zeros(pl.soft_bytes, dtype=torch.int8, device="cuda:0")
                    ref_buf = oracle.RefRxBuffer(pl.nof_codeblocks)
                items.append((pl, 0, soft))
            else:
                items.append((pl, 0))
        slot = amd.PuschSlot(items)
        g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
        cbi = torch.full((slot.cb_total,), -7, dtype=torch.int32, device="cuda:0")
        uci = torch.zeros(max(slot.uci_total, 1), dtype=torch.uint8, device="cuda:0")
        out, offs, res = proc.process_slot(g, slot, cb_iterations=cbi, uci=uci)
        torch.cuda.synchronize()
        out, cbi, uci = out.cpu().numpy(), cbi.cpu().numpy(), uci.cpu().numpy()
        res = amd.pusch_processor.parse_results(res.cpu().numpy())
        for u, (pdu, pl) in enumerate(zip(pdus, plans)):
            tag = "slot %d rnti %#x" % (slot_index, pdu["rnti"])
            P = pdu["nof_rx_ports"]
            kw = dict(rx_buffer=ref_buf) if pdu["rnti"] == 0x5003 else {}
            want_tb, want = pp.ref_pusch_process(grid[:P], pdu, pl.tb_bytes, iterations=iters, **kw)
            got_tb = out[offs[u]:offs[u] + pl.tb_bytes]
            assert bool(res[u].data.tb_crc_ok) == want["tb_crc_ok"], tag
            assert np.array_equal(got_tb, want_tb), tag
            assert res[u].data.nof_codeblocks_total == want["nof_codeblocks_total"], tag
            assert res[u].data.ldpc_iterations_sum == want["iterations_sum"], (tag, res[u].data, want)
            c = cbi[slot.cb_offsets[u]:slot.cb_offsets[u] + pl.nof_codeblocks]
            assert (c != -7).all(), tag
            assert int(np.where(c >= 0, c, iters).sum()) == want["iterations_sum"], (tag, c)
            _check_csi(res[u], want, tag)
            if pdu.get("nof_harq_ack", 0):
                row = uci[slot.uci_offsets[u]:slot.uci_offsets[u] + pl.uci_bytes]
                n_ack, n_csi1 = pdu["nof_harq_ack"], pdu["nof_csi_part1"]
                assert res[u].harq_ack_status == want["harq_ack_status"] == 1, tag
                assert res[u].csi_part1_status == want["csi_part1_status"] == 1, tag
                assert np.array_equal(row[:n_ack], want["harq_ack"]) and np.array_equal(row[:n_ack], sent[u][1][0])
                assert np.array_equal(row[n_ack:n_ack + n_csi1], want["csi_part1"]), tag
            if pdu["rnti"] == 0x5003:
                assert want["tb_crc_ok"] == (rv == 2), tag  # rv 0 alone fails, the combined rv 2 decodes
            else:
                assert want["tb_crc_ok"] and np.array_equal(got_tb, sent[u][0]), tag


@pytest.mark.parametrize("slot_index", [3, 4, 6])
def test_pusch_slot_csi_part2_uci_only_fused_vs_reference(slot_index, monkeypatch):
    """PDUs with CSI part 2 (sized by their decoded CSI part 1) and UCI-only PDUs (no codeword,
    HARQ-ACK + CSI part 1) in the FUSED slot group -- CSI part 2 size selected on the device, the
    demultiplexer / UCI decoder / UL-SCH row geometry of the selected size, no host readback -- next to a HARQ-ACK +
    CSI part 1 PDU and two plain PDUs on one four-port grid, against the compiled pusch_processor_impl called once per
    PDU (pusch_processor_impl.cpp:56-103, :305-324): TB bytes, CRC flags, LDPC statistics, CSI, every UCI payload,
    status and CSI part 2 size; and every output identical to the per-PDU batch chains (SRSRAN_AMD_PUSCH_FUSED=0).
    The three slots' CSI part 1 payloads select different CSI part 2 sizes."""
    import torch

    from pusch_slot_cases import mixed_slot, kind_of, NSUBC

    iters = 6
    kinds = ["uci", "csi2", "ucionly", "plain", "plain2"]
    grid, pdus, sent = mixed_slot(slot_index, 0, seed=slot_index, kinds=kinds)
    assert sorted(kind_of(p) for p in pdus) == sorted(["uci", "csi2", "ucionly", "plain", "plain"])
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SRSRAN_AMD_PUSCH_FUSED", mode)
        proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=iters), device=0)
        plans = [proc.plan(amd.make_pdu(**p), NSUBC) for p in pdus]
        slot = amd.PuschSlot([(pl, 0) for pl in plans])
        g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
        cbi = torch.full((max(slot.cb_total, 1),), -7, dtype=torch.int32, device="cuda:0")
        uci = torch.zeros(max(slot.uci_total, 1), dtype=torch.uint8, device="cuda:0")
        out, offs, res = proc.process_slot(g, slot, cb_iterations=cbi, uci=uci)
        torch.cuda.synchronize()
        outs[mode] = (out.cpu().numpy(), offs, res.cpu().numpy(), cbi.cpu().numpy(), uci.cpu().numpy(), slot, plans)
    for a, b in zip(outs["1"][:5], outs["0"][:5]):
        if isinstance(a, np.ndarray):
            np.testing.assert_array_equal(a, b)
        else:
            assert list(a) == list(b)
    out, offs, res, cbi, uci, slot, plans = outs["1"]
    res = amd.pusch_processor.parse_results(res)
    seen_sizes = []
    for u, (pdu, pl) in enumerate(zip(pdus, plans)):
        kind = kind_of(pdu)
        tag = "slot %d %s" % (slot_index, kind)
        P = pdu["nof_rx_ports"]
        want_tb, want = pp.ref_pusch_process(grid[:P], pdu, pl.tb_bytes, iterations=iters)
        got = res[u]
        assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], tag
        assert got.data.nof_codeblocks_total == want["nof_codeblocks_total"], tag
        if kind != "ucionly":
            assert np.array_equal(out[offs[u]:offs[u] + pl.tb_bytes], want_tb), tag
            assert got.data.ldpc_iterations_sum == want["iterations_sum"], (tag, got.data, want)
            c = cbi[slot.cb_offsets[u]:slot.cb_offsets[u] + pl.nof_codeblocks]
            assert int(np.where(c >= 0, c, iters).sum()) == want["iterations_sum"], (tag, c)
            assert want["tb_crc_ok"] and np.array_equal(want_tb, sent[u][0]), tag
        _check_csi(got, want, tag)
        if kind in ("uci", "csi2", "ucionly"):
            row = uci[slot.uci_offsets[u]:slot.uci_offsets[u] + pl.uci_bytes]
            n_ack, n_csi1 = pdu["nof_harq_ack"], pdu["nof_csi_part1"]
            assert got.harq_ack_status == want["harq_ack_status"], tag
            assert got.csi_part1_status == want["csi_part1_status"], tag
            np.testing.assert_array_equal(row[:n_ack], want["harq_ack"], err_msg=tag)
            np.testing.assert_array_equal(row[n_ack:n_ack + n_csi1], want["csi_part1"], err_msg=tag)
            np.testing.assert_array_equal(want["harq_ack"], sent[u][1][0], err_msg=tag)
            np.testing.assert_array_equal(want["csi_part1"], sent[u][1][1], err_msg=tag)
            if kind == "csi2":
                n2 = len(want["csi_part2"])
                assert got.nof_csi_part2 == n2 == len(sent[u][1][2]), (tag, got.nof_csi_part2, n2)
                assert got.csi_part2_status == want["csi_part2_status"], tag
                np.testing.assert_array_equal(row[n_ack + n_csi1:n_ack + n_csi1 + n2], want["csi_part2"], err_msg=tag)
                np.testing.assert_array_equal(want["csi_part2"], sent[u][1][2], err_msg=tag)
                seen_sizes.append(n2)
    assert len(seen_sizes) == 1


def test_pusch_slot_rejects_unsupported():
    import torch

    proc = amd.PuschProcessor(amd.PuschProcessorConfig(), device=0)
    pdu = dict(BASE, tbs=_tbs(BASE))
    g = torch.zeros((1, 1, 14, 12 * 51), dtype=torch.int32, device="cuda:0")
    retx = proc.plan(amd.make_pdu(**dict(pdu, new_data=0)), 12 * 51)
    with pytest.raises(ValueError):
        proc.process_slot(g, [(retx, 0)])  # a retransmission without its soft buffer
    ok = proc.plan(amd.make_pdu(**pdu), 12 * 51)
    with pytest.raises(ValueError):
        proc.process_slot(g, [(ok, 1)])  # grid index out of range
    tbs, offs, res = proc.process_slot(g, [])
    assert offs == [] and res.shape[0] == 0


# Transform precoding (DFT-s-OFDM): low-PAPR DM-RS in the estimator, deprecoding in the demodulator, against the
# compiled pusch_processor_impl with dmrs_transform_precoding_configuration (pusch_processor_impl.cpp:172-196).
# (name, pdu overrides, grid PRBs, channel [rx ports], SNR dB)
TP_CASES = [
    ("tp_1rb_qpsk", dict(rb_start=3, rb_count=1, modulation=2, target_code_rate=308.0, n_rs_id=5), 52, None, 20.0),
    ("tp_5rb_16qam_2rx", dict(rb_start=10, rb_count=5, modulation=4, target_code_rate=434.0, nof_rx_ports=2,
                              n_rs_id=77, rnti=0x1234, n_id=33), 52, np.array([0.9, 0.4 - 0.3j]), 25.0),
    ("tp_25rb_64qam_4rx_3dmrs", dict(rb_start=20, rb_count=25, modulation=6, target_code_rate=567.0,
                                     nof_rx_ports=4, n_rs_id=1007, dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11)),
     52, np.array([0.8, 0.3j, -0.5, 0.6 + 0.2j]), 30.0),
    ("tp_270rb_16qam_2rx", dict(bwp_size_rb=273, rb_start=2, rb_count=270, modulation=4, target_code_rate=490.0,
                                nof_rx_ports=2, n_rs_id=301), 273, np.array([1.0, 0.5j]), 25.0),
]


@pytest.mark.parametrize("case", TP_CASES, ids=[c[0] for c in TP_CASES])
def test_pusch_processor_transform_precoding_vs_reference(case):
    """DFT-s-OFDM PUSCH through the processor (low-PAPR DM-RS estimate, equalizer, transform
    deprecoder, demapper, decoder) against the compiled pusch_processor_impl on the same grid."""
    name, over, nprb, ch, snr = case
    pdu = dict(BASE, **over, transform_precoding=1)
    nd = bin(pdu["dmrs_symbol_mask"]).count("1")
    tbs = amd.tbs_calculator_calculate(pdu["nof_symbols"], 12 * nd, 0, pdu["modulation"], pdu["target_code_rate"],
                                       1, 0, pdu["rb_count"])
    r = pdu["target_code_rate"] / 1024
    pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25) else 1
    tb = np.random.default_rng(len(name)).integers(0, 256, tbs // 8, dtype=np.uint8)
    grid, _ = pp.ue_transmit_tp(tb, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=3)
    want_tb, want = pp.ref_pusch_process(grid, pdu, tbs // 8, iterations=6)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    got_tb, got = proc.process(grid, plan)
    assert want["tb_crc_ok"] and np.array_equal(want_tb, tb), name  # the synthetic UE transmission is valid
    assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], name
    assert np.array_equal(got_tb, want_tb), name
    assert got.data.nof_codeblocks_total == want["nof_codeblocks_total"]
    assert got.data.ldpc_iterations_sum == want["iterations_sum"], (name, got.data.ldpc_iterations_sum, want)
    _check_csi(got, want, name)


def test_pusch_processor_transform_precoding_rejects():
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(), device=0)
    for over in (dict(nof_tx_layers=2, nof_rx_ports=2), dict(rb_count=7)):
        pdu = dict(BASE, **over, transform_precoding=1, tbs=1024)
        with pytest.raises(ValueError):
            proc.plan(amd.make_pdu(**pdu), 12 * 51)


# UCI on PUSCH: HARQ-ACK / CSI part 1 multiplexed with the UL-SCH by the UE (oracle ue_multiplex_uci: the
# reference's own UCI encoders and RE placement), against the compiled pusch_processor_impl with its
# ulsch_demultiplex_impl and uci_decoder_impl.  (name, pdu overrides, HARQ-ACK bits, CSI part 1 bits, SNR dB)
UCI_CASES = [
    ("ack1_16qam", dict(modulation=4, target_code_rate=490.0), 1, 0, 25.0),
    ("ack2_csi1_2", dict(modulation=4, target_code_rate=490.0, rnti=0x1234, n_id=11), 2, 2, 25.0),
    ("ack5_csi9_qpsk", dict(modulation=2, target_code_rate=679.0), 5, 9, 20.0),
    ("ack20_csi40_64qam_2rx", dict(modulation=6, target_code_rate=567.0, nof_rx_ports=2), 20, 40, 28.0),
    ("ack11_csi12_2layer", dict(modulation=4, target_code_rate=490.0, nof_tx_layers=2, nof_rx_ports=2,
                                dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11)), 11, 12, 28.0),
    ("ack2_csi400_256qam_4rx", dict(bwp_size_rb=106, rb_count=106, modulation=8, target_code_rate=797.0,
                                    nof_rx_ports=4), 2, 400, 35.0),
    ("ack3_lowsnr", dict(modulation=4, target_code_rate=658.0), 3, 20, 3.0),
]


@pytest.mark.parametrize("case", UCI_CASES, ids=[c[0] for c in UCI_CASES])
def test_pusch_processor_uci_vs_reference(case):
    """UCI bits on PUSCH -- demultiplexing, HARQ-ACK / CSI part 1 decoding and the UL-SCH around
    them -- identical to the compiled reference processor: TB, CRC, LDPC statistics, UCI payloads and statuses."""
    import torch

    name, over, n_ack, n_csi1, snr = case
    pdu = dict(BASE, **over, nof_harq_ack=n_ack, nof_csi_part1=n_csi1, beta_offset_harq_ack=8.0,
               beta_offset_csi_part1=6.25, alpha_scaling=1.0)
    nprb = pdu["bwp_size_rb"]
    tbs = _tbs(pdu)
    r = pdu["target_code_rate"] / 1024
    pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25) else 1
    rng = np.random.default_rng(len(name))
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    ack = rng.integers(0, 2, n_ack).astype(np.uint8)
    csi1 = rng.integers(0, 2, n_csi1).astype(np.uint8)
    L, P = pdu["nof_tx_layers"], pdu["nof_rx_ports"]
    ch = (np.eye(L, P) + 0.2j * np.ones((L, P))).astype(np.complex64)
    grid, _ = pp.ue_transmit(tb, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=2, uci=(ack, csi1))
    want_tb, want = pp.ref_pusch_process(grid, pdu, tbs // 8, iterations=6)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
    d_ack = torch.zeros((1, max(n_ack, 1)), dtype=torch.uint8, device="cuda:0")
    d_csi = torch.zeros((1, max(n_csi1, 1)), dtype=torch.uint8, device="cuda:0")
    out, res = proc.process_batch(g, plan, harq_ack=d_ack if n_ack else None, csi_part1=d_csi if n_csi1 else None)
    torch.cuda.synchronize()
    got = amd.pusch_processor.parse_results(res.cpu().numpy())[0]
    got_tb = out[0].cpu().numpy()
    assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], name
    assert np.array_equal(got_tb, want_tb), name
    assert got.data.ldpc_iterations_sum == want["iterations_sum"], (name, got.data.ldpc_iterations_sum, want)
    assert got.harq_ack_status == want["harq_ack_status"], (name, got.harq_ack_status, want["harq_ack_status"])
    assert got.csi_part1_status == want["csi_part1_status"], (name, got.csi_part1_status, want["csi_part1_status"])
    if n_ack:
        np.testing.assert_array_equal(d_ack[0, :n_ack].cpu().numpy(), want["harq_ack"], err_msg=name)
    if n_csi1:
        np.testing.assert_array_equal(d_csi[0, :n_csi1].cpu().numpy(), want["csi_part1"], err_msg=name)
    _check_csi(got, want, name)
    if snr >= 20:
        assert want["tb_crc_ok"] and want["harq_ack_status"] in (0, 1) and want["csi_part1_status"] in (0, 1), name
        assert np.array_equal(want["harq_ack"], ack) and np.array_equal(want["csi_part1"], csi1), name


# CSI part 2: its size comes from the decoded CSI part 1 through uci_part2_get_size; (name, pdu overrides,
# HARQ-ACK bits, CSI part 1 bits, CSI part 2 size description, SNR dB).  Each case runs a batch of grids whose CSI
# part 1 payloads select different CSI part 2 sizes (one of them 0: no CSI part 2 multiplexed).
CSI2_CASES = [
    ("csi2_qpsk", dict(modulation=2, target_code_rate=679.0), 4, 9, [([(0, 2)], [0, 5, 17, 40])], 20.0),
    ("csi2_ack2_16qam", dict(modulation=4, target_code_rate=490.0, rnti=0x321, n_id=5), 2, 12,
     [([(1, 1), (4, 2)], [3, 1, 2, 11, 30, 0, 64, 7])], 25.0),
    ("csi2_two_entries_2layer", dict(modulation=4, target_code_rate=490.0, nof_tx_layers=2, nof_rx_ports=2,
                                     dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11)), 6, 20,
     [([(0, 1)], [8, 0]), ([(2, 2)], [2, 0, 24, 100])], 28.0),
    ("csi2_large_64qam", dict(bwp_size_rb=106, rb_count=106, modulation=6, target_code_rate=567.0, nof_rx_ports=2),
     1, 40, [([(7, 1)], [150, 300])], 28.0),
]


@pytest.mark.parametrize("case", CSI2_CASES, ids=[c[0] for c in CSI2_CASES])
def test_pusch_processor_csi_part2_vs_reference(case):
    """CSI part 2 on PUSCH (pusch_processor_impl.cpp:73-103): the size each grid's decoded CSI part 1 selects, the
    demultiplexer's CSI part 2 placement from the symbol where CSI part 1 ends, the CSI part 2 decoding and the
    UL-SCH around it -- TB, CRC, LDPC statistics, every UCI payload and status identical to the compiled reference
    processor, per grid of one batch."""
    import torch

    name, over, n_ack, n_csi1, part2, snr = case
    pdu = dict(BASE, **over, nof_harq_ack=n_ack, nof_csi_part1=n_csi1, beta_offset_harq_ack=8.0,
               beta_offset_csi_part1=6.25, beta_offset_csi_part2=5.0, alpha_scaling=1.0, csi_part2_size=part2)
    nprb = pdu["bwp_size_rb"]
    tbs = _tbs(pdu)
    r = pdu["target_code_rate"] / 1024
    pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25) else 1
    rng = np.random.default_rng(len(name) + 100)
    L, P = pdu["nof_tx_layers"], pdu["nof_rx_ports"]
    ch = (np.eye(L, P) + 0.2j * np.ones((L, P))).astype(np.complex64)
    descr = amd.uci_part2_description(part2)
    grids, wants, sent = [], [], []
    for k in range(4):
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        ack = rng.integers(0, 2, n_ack).astype(np.uint8)
        csi1 = rng.integers(0, 2, n_csi1).astype(np.uint8)
        n2 = amd.uci_part2_get_size(csi1, descr)
        assert n2 == pp.ref_uci_part2_get_size(csi1, part2)
        csi2 = rng.integers(0, 2, n2).astype(np.uint8)
        grid, _ = pp.ue_transmit(tb, pdu, 12 * nprb, channel=ch, snr_db=snr, seed=3 + k, uci=(ack, csi1, csi2))
        grids.append(grid)
        wants.append(pp.ref_pusch_process(grid, pdu, tbs // 8, iterations=6))
        sent.append((tb, ack, csi1, csi2))
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * nprb)
    g = torch.from_numpy(np.stack(grids).view(np.int32)).to("cuda:0")
    n = len(grids)
    max2 = sum(max(sizes) for _, sizes in part2)
    d_ack = torch.zeros((n, max(n_ack, 1)), dtype=torch.uint8, device="cuda:0")
    d_csi1 = torch.zeros((n, max(n_csi1, 1)), dtype=torch.uint8, device="cuda:0")
    d_csi2 = torch.zeros((n, max(max2, 1)), dtype=torch.uint8, device="cuda:0")
    out, res = proc.process_batch(g, plan, harq_ack=d_ack if n_ack else None, csi_part1=d_csi1, csi_part2=d_csi2)
    torch.cuda.synchronize()
    results = amd.pusch_processor.parse_results(res.cpu().numpy())
    for k, ((want_tb, want), got) in enumerate(zip(wants, results)):
        tag = "%s grid %d" % (name, k)
        n2 = len(want["csi_part2"])
        assert got.nof_csi_part2 == n2, (tag, got.nof_csi_part2, n2)
        assert got.csi_part2_status == want["csi_part2_status"], (tag, got.csi_part2_status, want["csi_part2_status"])
        assert got.csi_part1_status == want["csi_part1_status"], tag
        assert got.harq_ack_status == want["harq_ack_status"], tag
        assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], tag
        assert np.array_equal(out[k].cpu().numpy(), want_tb), tag
        assert got.data.ldpc_iterations_sum == want["iterations_sum"], (tag, got.data.ldpc_iterations_sum, want)
        np.testing.assert_array_equal(d_csi1[k, :n_csi1].cpu().numpy(), want["csi_part1"], err_msg=tag)
        np.testing.assert_array_equal(d_csi2[k, :n2].cpu().numpy(), want["csi_part2"], err_msg=tag)
        if n_ack:
            np.testing.assert_array_equal(d_ack[k, :n_ack].cpu().numpy(), want["harq_ack"], err_msg=tag)
        tb, ack, csi1, csi2 = sent[k]
        # at these SNRs the reference recovers what the UE sent
        assert want["tb_crc_ok"] and np.array_equal(want["csi_part1"], csi1), tag
        assert np.array_equal(want["csi_part2"], csi2), tag


# DC subcarrier (pdu_t::dc_position): pusch_processor_impl.cpp:235-249 zeroes the DC subcarrier's channel estimate of
# a CP-OFDM PDU on every port, layer and OFDM symbol, so its REs equalize to zero symbols of infinite variance (zero
# LLRs); transform precoding leaves it.  DC at subcarrier 1638 = 12 x 273 / 2, where the reference's scheduler default
# (initial_ul_dc_offset = center) puts it.  (name, pdu overrides, SNR dB)
DC = 1638
DC_CASES = [
    ("dc_16qam_4rx", dict(bwp_size_rb=273, rb_start=100, rb_count=80, modulation=4, target_code_rate=490.0,
                          nof_rx_ports=4, rnti=0x4711, n_id=3), 25.0),
    ("dc_2layer_zf_64qam", dict(bwp_size_rb=273, rb_start=130, rb_count=12, modulation=6, target_code_rate=567.0,
                                nof_tx_layers=2, nof_rx_ports=2, dmrs_symbol_mask=(1 << 2) | (1 << 7) | (1 << 11)),
     30.0),
    ("dc_cdm1_bwp", dict(bwp_start_rb=100, bwp_size_rb=150, rb_start=30, rb_count=20, nof_cdm_groups_without_data=1,
                         dmrs_symbol_mask=1 << 3, start_symbol_index=1, nof_symbols=12, nof_rx_ports=2), 22.0),
    ("dc_outside_allocation", dict(bwp_size_rb=273, rb_start=0, rb_count=60, nof_rx_ports=2), 22.0),
]


def _dc_re_positions(pdu, nsubc):
    """Codeword RE indices (data-RE order) of the DC subcarrier."""
    from oracle.pusch_demod import data_re_mask

    crb0 = pdu["bwp_start_rb"] + pdu["rb_start"]
    mask = data_re_mask(nsubc, list(range(crb0, crb0 + pdu["rb_count"])), pdu["start_symbol_index"],
                        pdu["nof_symbols"], pdu["dmrs_symbol_mask"], False, pdu["nof_cdm_groups_without_data"])
    idx = np.cumsum(mask.reshape(-1)).reshape(mask.shape) - 1
    return [int(idx[l, DC]) for l in range(14) if mask[l, DC]]


@pytest.mark.parametrize("case", DC_CASES, ids=[c[0] for c in DC_CASES])
def test_pusch_processor_dc_position_vs_reference(case):
    """dc_position -- TB, CRC, LDPC statistics and CSI identical to the compiled pusch_processor_impl
    with the same dc_position, through the estimator-fused path and through the expanded-estimate path (whose caller
    estimates then hold zeros at the DC, as the reference's ch_estimate does); the DC REs' LLRs are zero and every
    other LLR equals the run without dc_position."""
    import torch

    name, over, snr = case
    pdu = dict(BASE, **over)
    nprb = 273
    nsubc = 12 * nprb
    tbs = _tbs(pdu)
    r = pdu["target_code_rate"] / 1024
    pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and r <= 0.67) or r <= 0.25) else 1
    rng = np.random.default_rng(len(name) + 7)
    tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
    L, P = pdu["nof_tx_layers"], pdu["nof_rx_ports"]
    ch = (np.eye(L, P) + 0.15j * np.ones((L, P))).astype(np.complex64)
    grid, splan = pp.ue_transmit(tb, pdu, nsubc, channel=ch, snr_db=snr, seed=4)
    want_tb, want = pp.ref_pusch_process(grid, dict(pdu, dc_position=DC), tbs // 8, iterations=6)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs, dc_position=DC)), nsubc)
    plan_nodc = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), nsubc)
    g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
    G = plan.sch.cw_length
    llrs = torch.zeros((1, (G + 63) // 64 * 64), dtype=torch.int8, device="cuda:0")
    llrs0 = torch.zeros_like(llrs)
    est = torch.zeros((1, P * L * 14 * nsubc), dtype=torch.int32, device="cuda:0")
    out_f, res_f = proc.process_batch(g, plan, llrs=llrs)
    out_e, res_e = proc.process_batch(g, plan, estimates=est)
    _, _ = proc.process_batch(g, plan_nodc, llrs=llrs0)
    torch.cuda.synchronize()
    for tag, out, res in (("fused", out_f, res_f), ("expanded", out_e, res_e)):
        got = amd.pusch_processor.parse_results(res.cpu().numpy())[0]
        assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"], (name, tag)
        assert np.array_equal(out[0].cpu().numpy(), want_tb), (name, tag)
        assert got.data.ldpc_iterations_sum == want["iterations_sum"], (name, tag, got.data.ldpc_iterations_sum, want)
        assert got.data.ldpc_iterations_max == want["iterations_max"], (name, tag)
        _check_csi(got, want, name + " " + tag)
    assert want["tb_crc_ok"] and np.array_equal(want_tb, tb), name
    # LLRs: zero at the DC REs (every layer and bit), equal elsewhere
    qm = pdu["modulation"]
    a, b = llrs[0, :G].cpu().numpy(), llrs0[0, :G].cpu().numpy()
    pos = _dc_re_positions(pdu, nsubc)
    dc_bits = np.zeros(G, bool)
    for j in pos:
        dc_bits[j * L * qm:(j + 1) * L * qm] = True
    assert (a[dc_bits] == 0).all(), name
    np.testing.assert_array_equal(a[~dc_bits], b[~dc_bits], err_msg=name)
    if pos:
        assert (b[dc_bits] != 0).any(), name  # the DC step changed something
    # the caller's estimates hold zeros at the DC subcarrier inside the allocation's symbols
    e = est[0].cpu().numpy().reshape(P * L, 14, nsubc)
    crb0 = pdu["bwp_start_rb"] + pdu["rb_start"]
    inside = crb0 * 12 <= DC < (crb0 + pdu["rb_count"]) * 12
    sy = slice(pdu["start_symbol_index"], pdu["start_symbol_index"] + pdu["nof_symbols"])
    if inside:
        assert (e[:, sy, DC] == 0).all() and (e[:, sy, DC + 1] != 0).all(), name
    else:
        assert not pos, name


def test_pusch_processor_dc_transform_precoding_untouched():
    """dc_position on a DFT-s-OFDM PDU changes nothing (pusch_processor_impl.cpp:235: only CP-OFDM), as the
    reference."""
    import torch

    pdu = dict(BASE, bwp_size_rb=273, rb_start=120, rb_count=25, modulation=4, target_code_rate=434.0,
               transform_precoding=1, n_rs_id=55, nof_rx_ports=2)
    tbs = pp_tbs_tp(pdu)
    pdu["base_graph"] = 2 if (tbs <= 292 or (tbs <= 3824 and 434.0 / 1024 <= 0.67)) else 1
    tb = np.random.default_rng(9).integers(0, 256, tbs // 8, dtype=np.uint8)
    grid, _ = pp.ue_transmit_tp(tb, pdu, 12 * 273, channel=np.array([0.8, 0.4j]), snr_db=25.0, seed=1)
    want_tb, want = pp.ref_pusch_process(grid, dict(pdu, dc_position=DC), tbs // 8, iterations=6)
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs, dc_position=DC)), 12 * 273)
    g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
    out, res = proc.process_batch(g, plan)
    torch.cuda.synchronize()
    got = amd.pusch_processor.parse_results(res.cpu().numpy())[0]
    assert bool(got.data.tb_crc_ok) == want["tb_crc_ok"] and want["tb_crc_ok"]
    assert np.array_equal(out[0].cpu().numpy(), want_tb)
    assert got.data.ldpc_iterations_sum == want["iterations_sum"]


def pp_tbs_tp(pdu):
    nd = bin(pdu["dmrs_symbol_mask"]).count("1")
    return amd.tbs_calculator_calculate(pdu["nof_symbols"], 12 * nd, 0, pdu["modulation"], pdu["target_code_rate"],
                                        1, 0, pdu["rb_count"])


# UCI-only PUSCH (no codeword): pusch_processor_impl.cpp:305-324 -- estimator, demodulator, demultiplexer into the
# UCI decoders, no UL-SCH.  (name, pdu overrides, HARQ-ACK bits, CSI part 1 bits, SNR dB)
# (without UL-SCH, CSI part 1 takes every RE the HARQ-ACK leaves, TS 38.212 6.3.2.4.1.2: allocations small enough for
# one polar codeword of E <= 8192 bits, as a scheduler grants them)
UCI_ONLY_CASES = [
    ("uci_only_ack5_csi12_16qam", dict(modulation=4, target_code_rate=490.0, nof_rx_ports=2, rb_count=8), 5, 12, 20.0),
    ("uci_only_ack1_csi20_qpsk", dict(modulation=2, target_code_rate=679.0, rb_count=10), 1, 20, 15.0),
    ("uci_only_csi60_2layer_dc", dict(bwp_size_rb=273, rb_start=134, rb_count=6, modulation=4,
                                      target_code_rate=378.0, nof_tx_layers=2, nof_rx_ports=2, dc_position=DC), 0, 60,
     25.0),
]


@pytest.mark.parametrize("case", UCI_ONLY_CASES, ids=[c[0] for c in UCI_ONLY_CASES])
def test_pusch_processor_uci_only_vs_reference(case):
    """a PUSCH PDU without codeword (tbs = 0) -- HARQ-ACK / CSI part 1 payloads and statuses and the
    CSI identical to the compiled pusch_processor_impl processing the same PDU without codeword; the result carries no
    transport block (TB CRC KO, no codeblocks).  Through the batch chain and the slot form next to a data PDU."""
    import torch

    name, over, n_ack, n_csi1, snr = case
    pdu = dict(BASE, **over, nof_harq_ack=n_ack, nof_csi_part1=n_csi1, beta_offset_harq_ack=8.0,
               beta_offset_csi_part1=6.25, alpha_scaling=1.0)
    nprb = pdu["bwp_size_rb"]
    nsubc = 12 * nprb
    rng = np.random.default_rng(len(name) + 50)
    ack = rng.integers(0, 2, n_ack).astype(np.uint8)
    csi1 = rng.integers(0, 2, n_csi1).astype(np.uint8)
    L, P = pdu["nof_tx_layers"], pdu["nof_rx_ports"]
    ch = (np.eye(L, P) + 0.2j * np.ones((L, P))).astype(np.complex64)
    tx = {k: v for k, v in pdu.items() if k != "dc_position"}
    grid, _ = pp.ue_transmit(np.zeros(0, np.uint8), tx, nsubc, channel=ch, snr_db=snr, seed=6, uci=(ack, csi1))
    _, want = pp.ref_pusch_process(grid, pdu, 0, iterations=6)
    assert want["nof_codeblocks_total"] == 0 and not want["tb_crc_ok"]
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=0)), nsubc)
    assert plan.nof_codeblocks == 0 and plan.tb_bytes == 0
    g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
    d_ack = torch.zeros((1, max(n_ack, 1)), dtype=torch.uint8, device="cuda:0")
    d_csi = torch.zeros((1, max(n_csi1, 1)), dtype=torch.uint8, device="cuda:0")
    _, res = proc.process_batch(g, plan, harq_ack=d_ack if n_ack else None, csi_part1=d_csi if n_csi1 else None)
    # the slot form: the UCI-only PDU next to a data PDU on its own grid
    dpdu = dict(BASE, bwp_size_rb=nprb, rb_start=0, rb_count=4, rnti=0x77, slot_index=pdu["slot_index"])
    dtbs = _tbs(dpdu)
    dpdu["base_graph"] = 2
    dtb = rng.integers(0, 256, dtbs // 8, dtype=np.uint8)
    dgrid, _ = pp.ue_transmit(dtb, dpdu, nsubc, snr_db=25.0, seed=8, nof_rx_ports=P)
    dplan = proc.plan(amd.make_pdu(**dict(dpdu, tbs=dtbs, nof_rx_ports=P)), nsubc)
    grids = torch.from_numpy(np.stack([grid, dgrid]).view(np.int32)).to("cuda:0")
    slot = amd.PuschSlot([(plan, 0), (dplan, 1)])
    uci = torch.zeros(max(slot.uci_total, 1), dtype=torch.uint8, device="cuda:0")
    tbs_s, offs, res_s = proc.process_slot(grids, slot, uci=uci)
    torch.cuda.synchronize()
    for tag, got, a_bits, c_bits in (
            ("batch", amd.pusch_processor.parse_results(res.cpu().numpy())[0], d_ack[0, :n_ack].cpu().numpy(),
             d_csi[0, :n_csi1].cpu().numpy()),
            ("slot", amd.pusch_processor.parse_results(res_s.cpu().numpy())[0],
             uci[:n_ack].cpu().numpy(), uci[n_ack:n_ack + n_csi1].cpu().numpy())):
        assert not got.data.tb_crc_ok and got.data.nof_codeblocks_total == 0, (name, tag)
        assert got.harq_ack_status == want["harq_ack_status"], (name, tag, got.harq_ack_status, want)
        assert got.csi_part1_status == want["csi_part1_status"], (name, tag, got.csi_part1_status, want)
        np.testing.assert_array_equal(a_bits, want["harq_ack"], err_msg=name + tag)
        np.testing.assert_array_equal(c_bits, want["csi_part1"], err_msg=name + tag)
        _check_csi(got, want, name + " " + tag)
    # the reference recovers what the UE sent; the data PDU of the slot decodes
    assert np.array_equal(want["harq_ack"], ack) and np.array_equal(want["csi_part1"], csi1), name
    got_d = amd.pusch_processor.parse_results(res_s.cpu().numpy())[1]
    assert got_d.data.tb_crc_ok and np.array_equal(tbs_s[offs[1]:offs[1] + dtbs // 8].cpu().numpy(), dtb)


def test_pusch_slot_per_pdu_slot_shared_plan():
    """PDUs of three slots that share one plan in one slot call each use their own slot's DM-RS
    (srs_amd_pusch_slot_pdu::has_slot): every transport block decodes, equal to the reference per slot."""
    import torch

    pdu = dict(BASE, bwp_size_rb=52, rb_count=52, nof_rx_ports=2, modulation=4, target_code_rate=490.0)
    tbs = _tbs(pdu)
    pdu["base_graph"] = 1 if tbs > 3824 else 2
    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=tbs)), 12 * 52)  # created for slot 0
    grids, tbs_sent, wants, slots = [], [], [], [5, 6, 9]
    for k, sl in enumerate(slots):
        p = dict(pdu, slot_index=sl)
        tb = np.random.default_rng(sl).integers(0, 256, tbs // 8, dtype=np.uint8)
        grid, _ = pp.ue_transmit(tb, p, 12 * 52, snr_db=25.0, seed=sl)
        grids.append(grid)
        tbs_sent.append(tb)
        wants.append(pp.ref_pusch_process(grid, p, tbs // 8, iterations=6))
    g = torch.from_numpy(np.stack(grids).view(np.int32)).to("cuda:0")
    # the fused route (new data, no soft buffer), then the batch-chain route (HARQ soft buffers kept)
    soft = [torch.zeros(plan.soft_bytes, dtype=torch.int8, device="cuda:0") for _ in range(3)]
    for route, pdus in (("fused", [(plan, k) for k in range(3)]), ("chain", [(plan, k, soft[k]) for k in range(3)])):
        slot = amd.PuschSlot(pdus, slots=[(1, sl) for sl in slots])
        out, offs, res = proc.process_slot(g, slot)
        torch.cuda.synchronize()
        for k, got in enumerate(amd.pusch_processor.parse_results(res.cpu().numpy())):
            want_tb, want = wants[k]
            assert got.data.tb_crc_ok and want["tb_crc_ok"], (route, k)
            assert np.array_equal(out[offs[k]:offs[k] + tbs // 8].cpu().numpy(), tbs_sent[k]), (route, k)
            assert got.data.ldpc_iterations_sum == want["iterations_sum"], (route, k)
            _check_csi(got, want, "%s slot %d" % (route, slots[k]))


def test_pusch_processor_harq_ack_only_pusch():
    """A PUSCH carrying only HARQ-ACK (no data, no CSI part 1).  Parity unpinned: the compiled reference
    pusch_processor_impl does not return for this PDU (reproduced on the CPU with the same grid; the reference's
    uplink_processor_impl.cpp:279-281 asserts that every PUSCH PDU has a codeword, so the path is unexercised there).
    Checked against the bits the UE sent, with the REs the HARQ-ACK leaves unused (reserved for a 1/2-bit HARQ-ACK)
    going to the discarded UL-SCH stream."""
    import torch

    proc = amd.PuschProcessor(amd.PuschProcessorConfig(dec_nof_iterations=6), device=0)
    for n_ack, snr in ((1, 10.0), (2, 10.0), (5, 12.0)):
        pdu = dict(BASE, modulation=2, target_code_rate=120.0, rb_count=4, nof_harq_ack=n_ack, nof_csi_part1=0,
                   beta_offset_harq_ack=8.0, alpha_scaling=1.0, rnti=0x99 + n_ack)
        ack = np.random.default_rng(n_ack).integers(0, 2, n_ack).astype(np.uint8)
        grid, _ = pp.ue_transmit(np.zeros(0, np.uint8), pdu, 12 * 51, snr_db=snr, seed=n_ack,
                                 uci=(ack, np.zeros(0, np.uint8)))
        plan = proc.plan(amd.make_pdu(**dict(pdu, tbs=0)), 12 * 51)
        g = torch.from_numpy(grid.view(np.int32)[None]).to("cuda:0")
        d_ack = torch.zeros((1, n_ack), dtype=torch.uint8, device="cuda:0")
        _, res = proc.process_batch(g, plan, harq_ack=d_ack)
        torch.cuda.synchronize()
        got = amd.pusch_processor.parse_results(res.cpu().numpy())[0]
        assert got.harq_ack_status in (0, 1) and not got.data.tb_crc_ok, (n_ack, got.harq_ack_status)
        np.testing.assert_array_equal(d_ack[0].cpu().numpy(), ack, err_msg=str(n_ack))

"""The channel-processor level of the boundary: the MI355X pusch_processor / pdsch_processor plug-ins
(integration/pusch_processor_hip, pdsch_processor_hip) and their throughput at the headline shape.

PUSCH: the plug-in (integration/pusch_processor_hip,
a pusch_processor_factory whose processors feed one slot collector that runs srs_amd_pusch_process_slot_ex) driven
as the reference's upper PHY drives a pusch_processor -- one process() call per PDU on a shared received grid
(uplink_processor_impl.cpp:270-326), results through pusch_processor_result_notifier, HARQ state in the reference's
rx_buffer -- against the REFERENCE's own pusch_processor_impl (oracle/_ref) called once per PDU on the same grid.

Bars: transport block bytes, TB CRC flags and LDPC iteration statistics (observations, sum, min, max) identical;
CSI within the estimator tolerances (SINR / EPRE / RSRP 0.05 dB, time alignment 2 ns); UCI payloads and statuses
identical, on_uci called exactly when the PDU carries UCI.
PDSCH: the plug-in (pdsch_processor::process per PDU on one resource_grid_writer) against the reference's
pdsch_processor_impl on the same PDUs and initial grid: the grids bit-identical.
"""
import ctypes
import os
import time

import numpy as np
import pytest

import srsran_project_amd as amd

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
from oracle import pusch_proc as pp

pytestmark = pytest.mark.gpu

ITERS = 6


@pytest.fixture(scope="module")
def phy():
    import torch

    torch.cuda.init()
    import oracle
    from oracle import phy as ophy

    return ophy, oracle


def _check(got, want, tag):
    assert got is not None, tag + ": not notified"
    assert got["tb_crc_ok"] == want["tb_crc_ok"], tag
    assert got["nof_codeblocks_total"] == want["nof_codeblocks_total"], tag
    for k in ("nof_observations", "iterations_sum", "iterations_min", "iterations_max"):
        assert got[k] == want[k], (tag, k, got[k], want[k])
    for k in ("sinr_db", "epre_db", "rsrp_db"):
        assert abs(got[k] - want[k]) <= 0.05, (tag, k, got[k], want[k])
    assert abs(got["time_alignment_s"] - want["time_alignment_s"]) <= 2e-9, (tag, "ta")


def _run_slot(ophy, oracle, plug, grid, pdus, bufs, ref_bufs):
    """process() per PDU on one grid, flush, wait; returns [(got, got_tb, want, want_tb)]."""
    g = ophy.Grid(grid)
    tickets = []
    for pdu in pdus:
        key = pdu["rnti"]
        if key not in bufs:
            C = pp.nof_codeblocks(pdu["tbs"], pdu["base_graph"])
            bufs[key], ref_bufs[key] = oracle.RefRxBuffer(C), oracle.RefRxBuffer(C)
        tickets.append(plug.process(g, amd.make_pdu(**pdu), pdu["tbs"] // 8, rx_buffer=bufs[key]))
    plug.flush()
    plug.wait()
    out = []
    for pdu, (t, tb) in zip(pdus, tickets):
        P = pdu["nof_rx_ports"]
        want_tb, want = pp.ref_pusch_process(grid[:P], pdu, pdu["tbs"] // 8, iterations=ITERS,
                                             rx_buffer=ref_bufs[pdu["rnti"]])
        got = plug.result(t, pdu.get("nof_harq_ack", 0), pdu.get("nof_csi_part1", 0))
        out.append((got, tb, want, want_tb))
    return out


def test_pusch_plugin_mixed_slots_vs_reference(phy):
    """every PDU kind of a slot (UCI on PUSCH, DFT-s-OFDM, a HARQ process rv 0 -> rv 2, plain PDUs) on
    one four-port grid, two consecutive slots, through pusch_processor::process of the plug-in, equal to the
    reference's pusch_processor_impl on the same grid and PDUs (HARQ state kept in one rx_buffer per UE on each
    side)."""
    ophy, oracle = phy
    from pusch_slot_cases import mixed_slot

    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    bufs, ref_bufs = {}, {}
    for slot_index, rv in ((3, 0), (4, 2)):
        grid, pdus, sent = mixed_slot(slot_index, rv, seed=slot_index)
        for pdu, (tb_sent, uci_sent), (got, tb, want, want_tb) in zip(
                pdus, sent, _run_slot(ophy, oracle, plug, grid, pdus, bufs, ref_bufs)):
            tag = "slot %d rnti %#x" % (slot_index, pdu["rnti"])
            _check(got, want, tag)
            assert np.array_equal(tb, want_tb), tag
            if pdu.get("nof_harq_ack", 0):
                assert got["nof_uci"] == 1, tag
                assert got["harq_ack_status"] == want["harq_ack_status"] == 1, tag
                assert got["csi_part1_status"] == want["csi_part1_status"] == 1, tag
                assert np.array_equal(got["harq_ack"], want["harq_ack"]), tag
                assert np.array_equal(got["csi_part1"], want["csi_part1"]), tag
            else:
                assert got["nof_uci"] == 0, tag
            if pdu["rnti"] == 0x5003:
                assert want["tb_crc_ok"] == (rv == 2), tag
            else:
                assert want["tb_crc_ok"] and np.array_equal(tb, tb_sent), tag
    s = plug.stats()
    assert s["pdus"] == 10 and s["errors"] == 0, s
    # one decoding per PDU: the failed rv 0 transmission's soft state comes from its only decoding
    assert s["harq_redecodes"] == 0 and s["harq_soft_downloads"] == 1 and s["retransmissions"] == 1, s


def test_pusch_plugin_two_cells_one_collector(phy):
    """Two cells (two processors of one factory, two grids, different slots) queued before one flush: the collector
    cuts the batch at the slot change and both cells' PDUs equal the reference."""
    ophy, oracle = phy
    from pusch_slot_cases import mixed_slot

    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    cell2 = ophy.PuschProcessorPlugin(sibling_of=plug)
    grid_a, pdus_a, _ = mixed_slot(6, 0, seed=11, kinds=["uci", "plain", "plain2"])
    grid_b, pdus_b, _ = mixed_slot(7, 0, seed=12, kinds=["tp", "plain", "plain2"])
    ga, gb = ophy.Grid(grid_a), ophy.Grid(grid_b)
    tickets = [(plug, plug.process(ga, amd.make_pdu(**p), p["tbs"] // 8), p, grid_a) for p in pdus_a]
    tickets += [(cell2, cell2.process(gb, amd.make_pdu(**p), p["tbs"] // 8), p, grid_b) for p in pdus_b]
    plug.flush()
    plug.wait()
    for proc, (t, tb), pdu, grid in tickets:
        P = pdu["nof_rx_ports"]
        want_tb, want = pp.ref_pusch_process(grid[:P], pdu, pdu["tbs"] // 8, iterations=ITERS)
        tag = "slot %d rnti %#x" % (pdu["slot_index"], pdu["rnti"])
        _check(proc.result(t, pdu.get("nof_harq_ack", 0), pdu.get("nof_csi_part1", 0)), want, tag)
        assert np.array_equal(tb, want_tb), tag
    s = plug.stats()
    assert s["batches"] >= 2 and s["pdus"] == len(tickets), s


def test_pusch_plugin_timer_flush(phy):
    """Without flush() the collector's timer (max_wait_us) runs the pending PDUs: the notifier is called."""
    ophy, oracle = phy
    from pusch_slot_cases import mixed_slot

    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS, max_wait_us=500)
    grid, pdus, sent = mixed_slot(2, 0, seed=21, kinds=["plain"])
    g = ophy.Grid(grid)
    t, tb = plug.process(g, amd.make_pdu(**pdus[0]), pdus[0]["tbs"] // 8)
    deadline = time.time() + 30
    got = None
    while got is None and time.time() < deadline:
        time.sleep(0.01)
        got = plug.result(t)
    assert got is not None and got["tb_crc_ok"] and np.array_equal(tb, sent[0][0])


def test_pusch_plugin_unsupported_pdu_reports_failure(phy):
    """A PDU the MI355X processor does not support (DM-RS type 2, which the reference's own validator also rejects)
    is notified as a failed transmission -- HARQ-ACK invalid through on_uci, on_sch with the TB CRC KO -- instead of
    stalling the upper PHY; the other PDUs of the slot are unaffected."""
    ophy, oracle = phy
    from pusch_slot_cases import mixed_slot

    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    grid, pdus, sent = mixed_slot(2, 0, seed=22, kinds=["uci", "plain"])
    g = ophy.Grid(grid)
    bad = dict(pdus[0], dmrs_type=2)
    t_bad, _ = plug.process(g, amd.make_pdu(**bad), bad["tbs"] // 8)
    t_ok, tb = plug.process(g, amd.make_pdu(**pdus[1]), pdus[1]["tbs"] // 8)
    plug.flush()
    plug.wait()
    got = plug.result(t_bad, bad["nof_harq_ack"], bad["nof_csi_part1"])
    assert got is not None and not got["tb_crc_ok"] and got["nof_uci"] == 1 and got["harq_ack_status"] == 2
    got = plug.result(t_ok)
    assert got["tb_crc_ok"] and np.array_equal(tb, sent[1][0])
    assert plug.stats()["errors"] == 1


# ---- PDSCH: the pdsch_processor plug-in (integration/pdsch_processor_hip) against pdsch_processor_impl ----

@pytest.mark.parametrize("bwp,ref_point", [((0, 273), 0), ((10, 263), 1)], ids=["crb0", "bwp10_prb0"])
def test_pdsch_plugin_slot_vs_reference(phy, bwp, ref_point):
    """VERDICT r3 #1 (PDSCH twin): four PDSCH PDUs of one grid (QPSK..256QAM, 1-4 layers, wideband precoding on four
    ports, reserved REs, DM-RS type 1 and 2, type-0 sparse allocation, data / DM-RS power offsets), each handed to the
    plug-in's pdsch_processor::process on one resource_grid_writer, one flush: the grid is bit-identical to the
    reference's pdsch_processor_impl processing the same PDUs on the same initial grid -- every written RE equal,
    every other RE untouched."""
    from pdsch_slot_cases import slot

    ophy, oracle = phy
    pdus, grid0 = slot(bwp=bwp, ref_point=ref_point)
    want = ophy.WriterGrid(grid0)
    for pdu, tb in pdus:
        ophy.ref_pdsch_process(want, pdu, tb)
    plug = ophy.PdschProcessorPlugin(device=0)
    got = ophy.WriterGrid(grid0)
    tickets = [plug.process(got, pdu, tb) for pdu, tb in pdus]
    plug.flush()
    plug.wait()
    assert all(plug.done(t) for t in tickets)
    w, g = want.read(), got.read()
    assert (w != grid0).sum() > 100000
    assert plug.stats()["errors"] == 0
    if not np.array_equal(g, w):
        # per-PDU diagnostics: mismatching REs inside each PDU's CRBs x symbols
        report = []
        for k, (pdu, tb) in enumerate(pdus):
            crbs = [i + pdu.bwp_start_rb for i in range(pdu.bwp_size_rb) if (pdu.vrb_mask[i // 8] >> (i % 8)) & 1]
            sub = np.zeros(g.shape[2], bool)
            for c in crbs:
                sub[12 * c:12 * c + 12] = True
            sy = slice(pdu.start_symbol_index, pdu.start_symbol_index + pdu.nof_symbols)
            d = (g[:, sy][:, :, sub] != w[:, sy][:, :, sub])
            dm = np.array([(pdu.dmrs_symbol_mask >> l) & 1 for l in range(14)][sy], bool)
            report.append((k, int(d.sum()), int(d[:, dm].sum()), int(d[:, ~dm].sum()), int(d.size),
                           int((g[:, sy][:, :, sub] == 0xFFFFFFFF).sum())))
        pytest.fail("grid differs in %d REs; per PDU (index, differing, in DM-RS symbols, in data symbols, REs, "
                    "sentinel): %s" % (int((g != w).sum()), report))


@pytest.mark.parametrize("device_grid", [False, True], ids=["host_grid", "device_grid"])
def test_pdsch_plugin_ptrs_and_prg_precoding_vs_reference(phy, device_grid):
    """PDSCH PDUs with PT-RS (frequency density 2 / 4, time density 1 / 2 / 4, every RE offset, power
    ratios, DM-RS type 1 and 2) and with precoding that differs between PRGs (2 to 7 PRGs), one grid, one flush: the
    grid is bit-identical to pdsch_processor_impl's -- the data filling the allocation over the PT-RS REs and
    stopping when the codeword (sized without them) runs out, the PT-RS overwriting its REs, data and DM-RS on the
    first PRG's weights, the PT-RS per PRG."""
    from pdsch_slot_cases import PTRS_PDUS, slot

    ophy, oracle = phy
    pdus, grid0 = slot(seed=17, slot_index=5, pdus=PTRS_PDUS)
    want = ophy.WriterGrid(grid0)
    for pdu, tb in pdus:
        ophy.ref_pdsch_process(want, pdu, tb)
    plug = ophy.PdschProcessorPlugin(device=0)
    got = ophy.DeviceGrid(grid0) if device_grid else ophy.WriterGrid(grid0)
    tickets = [plug.process(got, pdu, tb) for pdu, tb in pdus]
    plug.flush()
    plug.wait()
    assert all(plug.done(t) for t in tickets)
    assert plug.stats()["errors"] == 0
    w, g = want.read(), got.read()
    diff = np.argwhere(g != w)
    assert diff.size == 0, ("REs differ", len(diff), diff[:8].tolist())


def test_pdsch_plugin_two_slots_two_cells(phy):
    """Two cells (two writers) over two slots through one factory: each slot's PDUs land in their own writers,
    bit-identical to the reference, and the collector cuts between the slots."""
    from pdsch_slot_cases import slot

    ophy, oracle = phy
    plug = ophy.PdschProcessorPlugin(device=0)
    cases = [slot(seed=31, slot_index=3), slot(seed=32, slot_index=3), slot(seed=33, slot_index=4)]
    grids, wants = [], []
    for pdus, grid0 in cases:
        want = ophy.WriterGrid(grid0)
        for pdu, tb in pdus:
            ophy.ref_pdsch_process(want, pdu, tb)
        wants.append(want.read())
        g = ophy.WriterGrid(grid0)
        grids.append(g)
        for pdu, tb in pdus:
            plug.process(g, pdu, tb)
    plug.flush()
    plug.wait()
    for g, w in zip(grids, wants):
        np.testing.assert_array_equal(g.read(), w)
    s = plug.stats()
    assert s["batches"] >= 2 and s["pdus"] == 12, s


def _concurrent(*fns):
    """Wall seconds of the functions run at once on their own threads."""
    import threading

    th = [threading.Thread(target=f) for f in fns]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return time.perf_counter() - t0


def test_plugin_throughput_64_cells(phy):
    """Codeblocks/s THROUGH the plug-ins at the headline shape (64 cells of 100 MHz / 273 PRB, PUSCH 4 layers x 4
    rx MMSE 256QAM, PDSCH 4 layers x 4 ports 256QAM): per step, one process() per cell on the cell's resource grid,
    flush() at the slot boundary, wait for every notification.  Two grid kinds:
      host    the reference's reader / writer over host memory: grids staged over PCIe each step (row copies by the
              plug-ins' worker threads, two alternating buffer sets, completion on a separate thread);
      device  hip_resource_grid (integration/hip_resource_grid.h): the grids live in HBM (as the OFDM plug-ins produce
              / consume them) and the plug-ins work on them in place.
    Each kind is timed PUSCH alone, PDSCH alone, and both at once (two host threads, as the uplink and downlink
    processors run).  Written to gpurun_out/plugin_bench.json.  Floors: the device-grid PDSCH + PUSCH figure at least
    8 M codeblocks/s, and the host-grid one at least 2x round 4's 1.85 M."""
    import json
    import os
    import threading

    import torch

    import bench_pipeline as bp

    ophy, oracle = phy
    cells, warmup, steps = 64, 2, 10
    dev = torch.device("cuda:0")
    pl = bp.Pipeline(1, dev)
    pl.step(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    grid = pl.grid_ul[0].cpu().numpy().view(np.uint32)
    tb_ul = pl.tb_ul[0].cpu().numpy()
    tb_dl = pl.tb_dl[0].cpu().numpy()
    from oracle.phy import make_pdsch_pdu

    pdu_dl = make_pdsch_pdu(range(bp.NPRB), bp.dl_weights(), slot_index=bp.SLOT, rnti=bp.RNTI, qm=bp.QM, n_id=bp.N_ID,
                            dmrs_symbol_mask=bp.DMRS_MASK, scrambling_id=bp.N_ID, nof_cdm_groups_without_data=bp.NCDM,
                            start_symbol_index=bp.DL_START, nof_symbols=bp.DL_NSYM,
                            base_graph=bp.base_graph(pl.tbs_dl, bp.RATE / 1024), ratio_pdsch_dmrs_to_sss_dB=-3.0)
    c_ul, c_dl = pl.plan_ul.nof_segments, pl.plan_dl.nof_segments
    want_dl = pl.grid_dl[0].cpu().numpy().view(np.uint32)
    zeros = np.zeros((bp.DL_PORTS, 14, bp.NSUBC), np.uint32)
    plug = ophy.PuschProcessorPlugin(device=0, iterations=bp.LDPC_ITERS, mmse=True)
    dplug = ophy.PdschProcessorPlugin(device=0)
    res = dict(cells=cells, steps=steps)
    for kind in ("host", "device"):
        if kind == "host":
            ul = [ophy.Grid(grid) for _ in range(cells)]
            dl = [ophy.WriterGrid(zeros) for _ in range(cells)]
        else:
            ul = [ophy.DeviceGrid(grid, device=True) for _ in range(cells)]
            dl = [ophy.DeviceGrid(zeros) for _ in range(cells)]
        out = {}

        def run_ul():
            out["ul"] = plug.bench(ul, pl.pdu_ul, pl.tbs_ul // 8, warmup, steps)

        def run_dl():
            out["dl"] = dplug.bench(dl, pdu_dl, tb_dl, warmup, steps)

        s0 = plug.stats()
        run_ul()
        s1 = plug.stats()
        run_dl()
        dt_ul, ok, tbs = out["ul"]
        dt_dl = out["dl"]
        assert ok == cells * steps and all(np.array_equal(t, tb_ul) for t in tbs), kind
        # the plug-in's grid equals the Python-driven pipeline's PDSCH grid of the same transport block
        np.testing.assert_array_equal(dl[0].read(), want_dl, err_msg=kind)
        # both at once: the uplink and downlink processors on two threads (ctypes releases the GIL); the better of two
        # runs (the box's other tenants and the streams' hardware-queue mapping make single runs noisy)
        both_steps = min(_concurrent(run_ul, run_dl) for _ in range(2)) / (warmup + steps)
        res[kind] = dict(pusch_ms_per_step=dt_ul * 1e3, pdsch_ms_per_step=dt_dl * 1e3,
                         pusch_codeblocks_per_s=cells * c_ul / dt_ul, pdsch_codeblocks_per_s=cells * c_dl / dt_dl,
                         concurrent_ms_per_step=both_steps * 1e3,
                         pdsch_pusch_codeblocks_per_s=cells * (c_ul + c_dl) / both_steps)
        nb = max(s1["batches"] - s0["batches"], 1)
        res[kind]["pusch_host_us_per_batch"] = {k: round((s1[k] - s0[k]) / nb, 1)
                                               for k in ("stage_us", "set_wait_us", "wait_us", "notify_us", "stage_reads_us",
                                                         "stage_call_us", "stage_download_us")}
        if kind == "device":
            res[kind]["ul_grid_transfers"] = ul[0].transfers()
            res[kind]["dl_grid_transfers"] = dl[1].transfers()
    # device grids, two slots in flight (the uplink / downlink processors keep several slots in flight): step s
    # waits for step s - 2's notifications only, each slot on its own set of grids
    ul2 = [ophy.DeviceGrid(grid, device=True) for _ in range(2 * cells)]
    dl2 = [ophy.DeviceGrid(zeros) for _ in range(2 * cells)]
    out = {}

    def run_ul2():
        out["ul"] = plug.bench(ul2, pl.pdu_ul, pl.tbs_ul // 8, warmup, steps, depth=2)

    def run_dl2():
        out["dl"] = dplug.bench(dl2, pdu_dl, tb_dl, warmup, steps, depth=2)

    s0 = plug.stats()
    run_ul2()
    s1 = plug.stats()
    run_dl2()
    dt_ul, ok, tbs = out["ul"]
    dt_dl = out["dl"]
    assert ok == cells * steps and all(np.array_equal(t, tb_ul) for t in tbs), "pipelined"
    np.testing.assert_array_equal(dl2[cells + 3].read(), want_dl, err_msg="pipelined")
    both_steps = min(_concurrent(run_ul2, run_dl2) for _ in range(2)) / (warmup + steps)
    res["device_2_slots_in_flight"] = dict(
        pusch_ms_per_step=dt_ul * 1e3, pdsch_ms_per_step=dt_dl * 1e3, pusch_codeblocks_per_s=cells * c_ul / dt_ul,
        pdsch_codeblocks_per_s=cells * c_dl / dt_dl, concurrent_ms_per_step=both_steps * 1e3,
        pdsch_pusch_codeblocks_per_s=cells * (c_ul + c_dl) / both_steps,
        pusch_host_us_per_batch={k: round((s1[k] - s0[k]) / max(s1["batches"] - s0["batches"], 1), 1)
                                 for k in ("stage_us", "set_wait_us", "wait_us", "notify_us", "stage_reads_us",
                                                         "stage_call_us", "stage_download_us")})
    res["pusch_stats"], res["pdsch_stats"] = plug.stats(), dplug.stats()
    res["note"] = ("one process() per cell, flush, wait (device_2_slots_in_flight: wait for the slot before the "
                   "previous one); concurrent = the PUSCH and PDSCH benches on two host threads at once, codeblocks of "
                   "both over the wall time per step (warm-up steps included in that wall time)")
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/plugin_bench.json", "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    # device-resident grids: no grid crosses PCIe in the timed steps
    assert res["device"]["ul_grid_transfers"]["downloads"] == 0 and res["device"]["dl_grid_transfers"]["downloads"] <= 1
    # the device-grid PDSCH + PUSCH rate through the plug-ins at least 8 M codeblocks/s (r06:
    # 8.4-11.5 M one slot at a time over several boxes); host grids a regression floor (r06 2.9-4.4 M; r04 1.85 M)
    best = max(res["device"]["pdsch_pusch_codeblocks_per_s"],
               res["device_2_slots_in_flight"]["pdsch_pusch_codeblocks_per_s"])
    assert best >= 8e6, (res["device"], res["device_2_slots_in_flight"])
    assert res["host"]["pdsch_pusch_codeblocks_per_s"] >= 2.5e6, res["host"]


# ---- PDUs as the reference's FAPI adaptor produces them ----

FAPI_DC = 1638  # tx_direct_current_location: subcarrier 12 x 273 / 2 (scheduler default initial_ul_dc_offset = center)


def _fapi_ues():
    """(kind, FAPI fields) of one slot's PUSCH PDUs on a 273-PRB, four-antenna cell: every PDU carries the cell's
    tx_direct_current_location as the MAC -> FAPI translator sets it."""
    common = dict(bwp_start=0, bwp_size=273, numerology=1, sfn=0, num_layers=1, ul_dmrs_symb_pos=(1 << 2) | (1 << 11),
                  dmrs_type=1, nscid=0, num_dmrs_cdm_grps_no_data=2, start_symbol_index=0, nr_of_symbols=14,
                  tx_direct_current_location=FAPI_DC, has_data=1, rv_index=0, new_data=1, ldpc_base_graph=1,
                  tb_size_lbrm_bytes=159749, alpha_scaling=3, beta_offset_harq_ack=7, beta_offset_csi1=13,
                  beta_offset_csi2=13, num_rx_ant=4)
    return [
        ("dc_data", dict(common, rnti=0x4601, nid_pusch=21, scrambling_id=210, qm=4, target_code_rate=4900,
                         rb_start=110, rb_size=50, harq_process_id=1)),
        ("uci_data", dict(common, rnti=0x4602, nid_pusch=22, scrambling_id=220, qm=4, target_code_rate=4900,
                          rb_start=0, rb_size=60, harq_process_id=2, has_uci=1, harq_ack_bit_length=3,
                          csi_part1_bit_length=12)),
        ("uci_only", dict(common, rnti=0x4603, nid_pusch=23, scrambling_id=230, qm=2, target_code_rate=1200,
                          rb_start=200, rb_size=10, has_data=0, has_uci=1, harq_ack_bit_length=5,
                          csi_part1_bit_length=12)),
        ("tp", dict(common, rnti=0x4604, nid_pusch=24, qm=4, target_code_rate=4340, transform_precoding=1,
                    dmrs_identity=99, rb_start=60, rb_size=25, harq_process_id=3)),
        ("two_layer", dict(common, rnti=0x4605, nid_pusch=25, scrambling_id=250, nscid=1, qm=6,
                           target_code_rate=5670, num_layers=2, rb_start=160, rb_size=40, harq_process_id=4,
                           ul_dmrs_symb_pos=(1 << 2) | (1 << 7) | (1 << 11))),
        # DFT-s-OFDM over the DC (PRB 136 holds subcarrier 1638): contains_dc changes the geometry
        # (pusch_processor_impl.cpp:262-286, ulsch_info.cpp:353-357); it takes dc_data's place in even slots
        ("tp_dc", dict(common, rnti=0x4606, nid_pusch=26, qm=4, target_code_rate=4340, transform_precoding=1,
                       dmrs_identity=77, rb_start=125, rb_size=25, harq_process_id=5)),
    ]


def _default_kinds(slot):
    """dc_data and tp_dc both hold the DC PRB: odd slots carry dc_data, even slots tp_dc."""
    return [k for k, _ in _fapi_ues() if k != ("tp_dc" if slot % 2 else "dc_data")]


def _fapi_slot(ophy, slot, seed, kinds=None):
    """The slot's FAPI PDUs converted by convert_pusch_fapi_to_phy, the received grid (each UE from the reference's
    transmit classes, summed, AWGN) and what each UE sent."""
    from pusch_slot_cases import NSUBC, _bf16, _chan, _cplx, tbs_of
    from oracle.pusch_proc import ue_transmit, ue_transmit_tp

    rng = np.random.default_rng(seed)
    z = np.zeros((4, 14, NSUBC), np.complex128)
    out = []
    kinds = _default_kinds(slot) if kinds is None else kinds
    for u, (kind, f) in enumerate(_fapi_ues()):
        if kind not in kinds:
            continue
        pdu = dict(numerology=1, slot_index=slot, rnti=f["rnti"], bwp_start_rb=0, bwp_size_rb=273, modulation=f["qm"],
                   target_code_rate=f["target_code_rate"] / 10.0, rv=0, new_data=1, n_id=f["nid_pusch"],
                   nof_tx_layers=f["num_layers"], nof_rx_ports=4, dmrs_symbol_mask=f["ul_dmrs_symb_pos"], dmrs_type=1,
                   scrambling_id=f.get("scrambling_id", 0), n_scid=f["nscid"], nof_cdm_groups_without_data=2,
                   rb_start=f["rb_start"], rb_count=f["rb_size"], start_symbol_index=0, nof_symbols=14,
                   transform_precoding=f.get("transform_precoding", 0), n_rs_id=f.get("dmrs_identity", 0))
        tbs = tbs_of(pdu) if f["has_data"] else 0
        bg = 1 if tbs > 3824 or not tbs else 2
        f = dict(f, slot=slot, tb_size=tbs // 8, ldpc_base_graph=bg)
        fp = ophy.FapiPuschPdu(**f)
        assert fp.dc_position == FAPI_DC, kind  # the adaptor forwards the DC location to the PHY
        pdu.update(fp.params, base_graph=bg, tbs=tbs, nof_harq_ack=f.get("harq_ack_bit_length", 0),
                   nof_csi_part1=f.get("csi_part1_bit_length", 0))
        tb = rng.integers(0, 256, tbs // 8, dtype=np.uint8)
        uci = None
        if f.get("has_uci"):
            uci = (rng.integers(0, 2, pdu["nof_harq_ack"]).astype(np.uint8),
                   rng.integers(0, 2, pdu["nof_csi_part1"]).astype(np.uint8))
        if pdu["transform_precoding"]:
            g, _ = ue_transmit_tp(tb, pdu, NSUBC, channel=np.array([0.8, 0.3j, -0.5, 0.6 + 0.2j]))
        else:
            g, _ = ue_transmit(tb, pdu, NSUBC, channel=_chan(pdu["nof_tx_layers"], 4, 60 + u), uci=uci)
        zu = _cplx(g)
        z += zu / np.sqrt(float(np.mean(np.abs(zu[np.abs(zu) > 0]) ** 2)))
        out.append((kind, fp, tb, uci))
    sigma2 = 10 ** (-26.0 / 10)
    z += np.sqrt(sigma2 / 2) * (rng.normal(size=z.shape) + 1j * rng.normal(size=z.shape))
    return _bf16(z), out


def test_pusch_plugin_fapi_pdus_dc_uci_only_vs_reference(phy):
    """PUSCH PDUs produced by the reference's own FAPI -> PHY conversion
    (convert_pusch_fapi_to_phy, lib/fapi_adaptor/phy/messages/pusch.cpp, compiled into the oracle) from FAPI PDUs
    carrying tx_direct_current_location = 1638 -- a data PDU whose allocation contains the DC (slot 3), a DFT-s-OFDM PDU
    whose allocation contains the DC (slot 4), a data + UCI PDU, a UCI-only PDU (no data bit), a DFT-s-OFDM PDU off the
    DC, a two-layer PDU -- through the plug-in's pusch_processor::process,
    equal to the reference's pusch_processor_impl on the same converted PDUs and grid: TB, CRC, LDPC statistics, UCI
    payloads / statuses (on_uci alone for the UCI-only PDU), CSI."""
    ophy, oracle = phy
    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    for slot in (3, 4):
        grid, ues = _fapi_slot(ophy, slot, seed=slot)
        g = ophy.Grid(grid)
        tickets = [plug.process_fapi(g, fp) for _, fp, _, _ in ues]
        plug.flush()
        plug.wait()
        for (kind, fp, tb_sent, uci), (t, tb) in zip(ues, tickets):
            tag = "slot %d %s" % (slot, kind)
            want_tb, want = ophy.ref_pusch_process_fapi(g, fp, iterations=ITERS)
            got = plug.result(t, fp.fapi.harq_ack_bit_length, fp.fapi.csi_part1_bit_length)
            assert got is not None, tag + ": not notified"
            assert got["nof_uci"] == want["nof_uci"] == (1 if uci is not None else 0), tag
            if fp.tb_bytes:
                _check(got, want, tag)
                assert np.array_equal(tb, want_tb), tag
                assert want["tb_crc_ok"] and np.array_equal(want_tb, tb_sent), tag
            else:
                for k in ("sinr_db", "epre_db", "rsrp_db"):
                    assert abs(got[k] - want[k]) <= 0.05, (tag, k, got[k], want[k])
            if uci is not None:
                assert got["harq_ack_status"] == want["harq_ack_status"] == 1, tag
                assert got["csi_part1_status"] == want["csi_part1_status"] == 1, tag
                assert np.array_equal(got["harq_ack"], want["harq_ack"]) and np.array_equal(want["harq_ack"], uci[0])
                assert np.array_equal(got["csi_part1"], want["csi_part1"]) and np.array_equal(want["csi_part1"], uci[1])
    s = plug.stats()
    assert s["errors"] == 0 and s["pdus"] == 10, s


def test_pusch_plugin_three_slots_one_config(phy):
    """ADVICE r4 (high/medium): three slots of one UE with an identical PDU configuration (one cached plan) queued
    before a single flush: the collector cuts a batch at every slot change, each PDU carries its own slot, and every
    transport block equals the reference."""
    ophy, oracle = phy
    from pusch_slot_cases import mixed_slot

    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    runs = []
    for sl in (6, 7, 8):
        grid, pdus, sent = mixed_slot(sl, 0, seed=40, kinds=["plain"])
        g = ophy.Grid(grid)
        runs.append((grid, pdus[0], sent[0][0], g, plug.process(g, amd.make_pdu(**pdus[0]), pdus[0]["tbs"] // 8)))
    plug.flush()
    plug.wait()
    for grid, pdu, tb_sent, g, (t, tb) in runs:
        want_tb, want = pp.ref_pusch_process(grid[:pdu["nof_rx_ports"]], pdu, pdu["tbs"] // 8, iterations=ITERS)
        got = plug.result(t)
        _check(got, want, "slot %d" % pdu["slot_index"])
        assert got["tb_crc_ok"] and np.array_equal(tb, tb_sent) and np.array_equal(tb, want_tb)
    s = plug.stats()
    assert s["batches"] == 3 and s["pdus"] == 3, s


def _pdcch_grid(seed, ports, nsubc):
    g = np.random.default_rng(seed).integers(0, 2**32, (ports, 14, nsubc), dtype=np.uint64)
    return g.astype(np.uint32)


def test_pdcch_plugin_vs_reference(phy):
    """pdcch_processor_factory_hip's processors, driven through the reference's pdcch_processor
    interface, write exactly the grid pdcch_processor_impl writes -- on a host writer grid (the REs of the DCI's CRBs
    stored through get_view) and on a device-resident hip_resource_grid (written in place, read back once by the host
    reader) -- for every case PDU, and for five DCIs of two CORESETs on one grid."""
    from oracle import pdcch as op
    from tests.pdcch_cases import cases, slot_pdus

    ophy, _ = phy
    plug = ophy.PdcchProcessorPlugin(device=0)
    for i, (name, pdu) in enumerate(cases()):
        c = pdu.coreset
        nsubc = 12 * min(c.bwp_start_rb + c.bwp_size_rb + 2, 275)
        g0 = _pdcch_grid(i, pdu.dci.nof_ports + 1, nsubc)
        want = op.ref_process(g0.copy(), [pdu])
        wg = ophy.WriterGrid(g0)
        plug.process(wg, [pdu])
        assert np.array_equal(wg.read(), want), (name, "host grid")
        dg = ophy.DeviceGrid(g0)
        plug.process(dg, [pdu])
        assert np.array_equal(dg.read(), want), (name, "device grid")
        assert dg.transfers() == dict(downloads=1, uploads=1), name
        assert plug.validate(pdu) is None, name
    nsubc = 12 * 106
    pdus = [p for p in slot_pdus(1, nsubc)]
    g0 = _pdcch_grid(99, 2, nsubc)
    want = op.ref_process(g0.copy(), pdus)
    dg = ophy.DeviceGrid(g0, device=True)
    plug.process(dg, pdus)
    assert np.array_equal(dg.read(), want), "five DCIs, device grid"
    wg = ophy.WriterGrid(g0)
    plug.process(wg, pdus)
    assert np.array_equal(wg.read(), want), "five DCIs, host grid"
    s = plug.stats()
    n = len(cases())
    assert s == dict(pdus=2 * n + 2 * len(pdus), errors=0, device_grids=n + len(pdus)), s


def test_pdcch_plugin_validator_and_unsupported(phy):
    """The plug-in factory's validator rejects what pdcch_processor_validator_impl rejects (same messages); an invalid
    PDU handed to process anyway is logged and counted, and leaves the grid untouched."""
    from srsran_project_amd.pdcch import make_pdu
    from tests.pdcch_cases import INVALID

    ophy, _ = phy
    plug = ophy.PdcchProcessorPlugin(device=0)
    for name, kw, text in INVALID:
        pdu = make_pdu(np.ones(20, np.uint8), **kw)
        msg = plug.validate(pdu)
        assert msg is not None and text in msg, (name, msg)
    g0 = _pdcch_grid(3, 1, 12 * 52)
    wg = ophy.WriterGrid(g0)
    plug.process(wg, [make_pdu(np.ones(20, np.uint8), aggregation_level=3)])
    assert np.array_equal(wg.read(), g0)
    assert plug.stats()["errors"] == 1


def test_ssb_plugin_vs_reference(phy):
    """ssb_processor_factory_hip's processors, driven through the reference's ssb_processor interface, write exactly
    the grid ssb_processor_impl writes -- on a host writer grid (the block's PSS / SSS / PBCH / DM-RS REs stored
    through get_view) and on a device-resident hip_resource_grid -- for every case of tests/ssb_cases.py; PDUs the
    reference asserts on are refused by the validator, logged and counted, the grid untouched."""
    from oracle import ssb as oss
    from tests import ssb_cases

    ophy, _ = phy
    plug = ophy.SsbProcessorPlugin(device=0)
    for i, case in enumerate(ssb_cases.CASES):
        pdu = ssb_cases.pdu(case, seed=40 + i)
        g0 = ssb_cases.grid0(seed=50 + i)
        want = oss.ref_process(g0.copy(), [pdu])
        wg = ophy.WriterGrid(g0)
        plug.process(wg, [pdu])
        assert np.array_equal(wg.read(), want), (case[0], "host grid")
        dg = ophy.DeviceGrid(g0)
        plug.process(dg, [pdu])
        assert np.array_equal(dg.read(), want), (case[0], "device grid")
        assert plug.validate(pdu) is None, case[0]
    n = len(ssb_cases.CASES)
    assert plug.stats() == dict(pdus=2 * n, errors=0, device_grids=n), plug.stats()
    g0 = ssb_cases.grid0(seed=3)
    for case in ssb_cases.INVALID:
        pdu = ssb_cases.pdu(case)
        assert plug.validate(pdu) is not None, case[0]
        wg = ophy.WriterGrid(g0)
        plug.process(wg, [pdu])
        assert np.array_equal(wg.read(), g0), case[0]
    assert plug.stats()["errors"] == len(ssb_cases.INVALID)


def test_device_grid_concurrent_writers_vs_reference(phy):
    """the reference schedules PDCCH, PDSCH, SSB ... on separate executors that write one slot grid
    at once (downlink_processor_multi_executor_impl.cpp:81-217).  On one hip_resource_grid, from four threads at once:
    the PDCCH, SSB and PDSCH plug-ins (device writers, kernels on their own streams) and the reference's CPU
    pdsch_processor_impl (a host writer through the grid's resource_grid_writer), on disjoint REs.  The grid read
    back equals the reference processors' grid of the same PDUs, in every round (no device producer's REs lost, no
    host write lost to a device merge)."""
    import threading

    from oracle import pdcch as op
    from oracle import ssb as oss
    from pdsch_slot_cases import NSUBC, slot
    from tests import pdcch_cases, ssb_cases

    ophy, _ = phy
    # PDSCH A (host writer) on PRBs 100-159, PDSCH B (plug-in) on PRBs 180-259, symbols 2-13; the PDCCH CORESETs in
    # symbols 0-1; the SS/PBCH block in symbols 2-5 of PRBs below 40
    cases = [(2, 679.0, 1, (100, 160), 2, 12, (1 << 2) | (1 << 11), 1, 2, [], (0.0, 0.0)),
             (4, 490.0, 2, (180, 260), 2, 12, (1 << 3) | (1 << 10), 1, 2, [], (0.0, 0.0))]
    (pdu_a, tb_a), (pdu_b, tb_b) = slot(seed=23, slot_index=2, pdus=cases)[0]
    pdcch = [p for p in pdcch_cases.slot_pdus(1, NSUBC) if p.coreset.start_symbol_index == 0]
    ssb = ssb_cases.pdu(ssb_cases.CASES[0], seed=5)
    zeros = np.zeros((4, 14, NSUBC), np.uint32)
    ref = ophy.WriterGrid(zeros)
    ophy.ref_pdsch_process(ref, pdu_a, tb_a)
    ophy.ref_pdsch_process(ref, pdu_b, tb_b)
    want = oss.ref_process(op.ref_process(ref.read(), pdcch), [ssb])
    assert (want != 0).sum() > 50000
    pdsch_plug = ophy.PdschProcessorPlugin(device=0)
    pdcch_plug = ophy.PdcchProcessorPlugin(device=0)
    ssb_plug = ophy.SsbProcessorPlugin(device=0)
    for rnd in range(6):
        dg = ophy.DeviceGrid(zeros)
        errors = []

        def run(fn):
            try:
                fn()
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(repr(e))

        def pdsch_device():
            pdsch_plug.process(dg, pdu_b, tb_b)
            pdsch_plug.flush()
            pdsch_plug.wait()

        jobs = [pdsch_device, lambda: pdcch_plug.process(dg, pdcch), lambda: ssb_plug.process(dg, [ssb]),
                lambda: ophy.ref_pdsch_process(dg, pdu_a, tb_a)]
        th = [threading.Thread(target=run, args=(j,)) for j in (jobs if rnd % 2 == 0 else jobs[::-1])]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        got = dg.read()
        diff = np.argwhere(got != want)
        assert diff.size == 0, ("round", rnd, "REs differ", len(diff), diff[:8].tolist())
    assert pdsch_plug.stats()["errors"] == 0 and pdcch_plug.stats()["errors"] == 0 and ssb_plug.stats()["errors"] == 0


def test_pucch_plugin_vs_reference(phy):
    """pucch_processor_factory_hip's processor, driven through the reference's pucch_processor interface on host
    reader grids and device-resident hip_resource_grids: Format 0 / Format 1 batches / Format 2 messages (status,
    bits, payload) equal to the compiled pucch_detector_format0 / pucch_detector_format1 / pucch_processor_impl, CSI
    within the tolerances of tests/test_pucch_gpu.py; Formats 3 / 4 likewise against pucch_processor_impl."""
    from oracle import pucch as op
    from tests import pucch_cases as pc

    ophy, _ = phy
    plug = ophy.PucchProcessorPlugin(device=0)
    nprb = pc.NSUBC // 12
    n = nd = 0
    for i, (pdu, grid, _) in enumerate(pc.cases(n=8, seed=11)):
        want = op.ref_detect(grid, pdu)
        for g in (ophy.Grid(grid), ophy.DeviceGrid(grid)):
            got = plug.f0(g, pdu, nprb)
            assert (got.status, got.nof_sr, got.sr * got.nof_sr, list(got.harq_ack)[:got.nof_harq_ack]) == \
                (want.status, want.nof_sr, want.sr * want.nof_sr, list(want.harq_ack)[:want.nof_harq_ack]), i
            for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
                assert abs(getattr(got, k) - getattr(want, k)) <= 0.01, (i, k)
            n += 1
        nd += 1
    for i, (b, grid, _) in enumerate(pc.f1_cases(n=6, seed=12)):
        dense = np.ascontiguousarray(grid[[b.ports[k] for k in range(b.nof_ports)]])
        want = op.ref_detect_f1(grid, b)
        for k in range(b.nof_ports):
            b.ports[k] = k
        for g in (ophy.Grid(dense), ophy.DeviceGrid(dense)):
            got = plug.f1(g, b, nprb)
            for j, (x, w) in enumerate(zip(got, want)):
                assert x.status == w.status and list(x.harq_ack)[:w.nof_harq_ack] == list(w.harq_ack)[:w.nof_harq_ack], (i, j)
                np.testing.assert_allclose(x.detection_metric, w.detection_metric, rtol=1e-3)
                for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
                    assert abs(getattr(x, k) - getattr(w, k)) <= 0.01, (i, j, k)
            n += b.nof_entries
        nd += 1  # one device-grid read per batch
    for i, (pdu, grid, _) in enumerate(pc.f2_cases(n=8, seed=13)):
        want, want_pay = op.ref_process_f2(grid, pdu)
        for g in (ophy.Grid(grid), ophy.DeviceGrid(grid)):
            got, pay = plug.f2(g, pdu)
            assert got.status == want.status and np.array_equal(pay, want_pay), i
            for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
                assert abs(getattr(got, k) - getattr(want, k)) <= 0.02, (i, k)
            assert abs(got.time_alignment_s - want.time_alignment_s) <= 2.5 / (480e3 * 4096), i
            n += 1
        nd += 1
        assert plug.validate_f2(pdu) is None, i
    for i, (pdu, grid, _) in enumerate(pc.f34_cases(n=8, seed=14)):
        want, want_pay = op.ref_process_f34(grid, pdu)
        for g in (ophy.Grid(grid), ophy.DeviceGrid(grid)):
            got, pay = plug.f34(g, pdu)
            assert got.status == want.status and np.array_equal(pay, want_pay), (i, pdu.format)
            for k in ("sinr_dB", "rsrp_dB", "epre_dB"):
                assert abs(getattr(got, k) - getattr(want, k)) <= 0.02, (i, k)
            n += 1
        nd += 1
    # (one caller at a time: every device-grid call is a rendezvous batch of its own)
    s = plug.stats()
    assert (s["pdus"], s["errors"], s["device_grids"], s["batches"]) == (n, 0, nd, nd), s
    import srsran_project_amd as amd

    assert plug.validate_f2(amd.pucch.make_f2_pdu(nof_prb=2, nof_harq_ack=4, nof_csi_part2=3)) is not None
    assert plug.validate_f2(amd.pucch.make_f2_pdu(nof_prb=1, nof_symbols=1, nof_harq_ack=40)) is not None


def test_pucch_plugin_latency(phy):
    """Per-call latency of the synchronous pucch_processor::process through the plug-in (host reader grid and
    device-resident grid; Format 0 and Format 2), written to gpurun_out/pucch_plugin_latency.json; a floor that only
    catches a regression to per-row copies or extra synchronisations."""
    import json

    from tests import pucch_cases as pc

    ophy, _ = phy
    plug = ophy.PucchProcessorPlugin(device=0)
    pdu0, grid0, _ = pc.cases(n=1, seed=21)[0]
    pdu2, grid2, _ = pc.f2_cases(n=1, seed=22)[0]
    nprb = pc.NSUBC // 12
    out = {}
    for name, g0, g2 in (("host_grid", ophy.Grid(grid0), ophy.Grid(grid2)),
                         ("device_grid", ophy.DeviceGrid(grid0), ophy.DeviceGrid(grid2))):
        plug.latency_us(g0, pdu0=pdu0, grid_prb=nprb, reps=20)
        out[name] = dict(f0_us=round(plug.latency_us(g0, pdu0=pdu0, grid_prb=nprb), 1),
                         f2_us=round(plug.latency_us(g2, pdu2=pdu2), 1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pucch_plugin_latency.json"), "w") as f:
        json.dump(out, f)
    assert out["device_grid"]["f0_us"] < 1000 and out["host_grid"]["f2_us"] < 2000, out


def test_pucch_plugin_rendezvous_64_cells(phy):
    """the synchronous PUCCH calls of 64 cells (bench_pucch.cell_pdus: 8 F0 + 2 F1 batches of 12 + 4 F2
    + 2 F3 + 1 F4 per cell, 273 PRB, 4 ports, device-resident grids) from many PUCCH-executor threads, one
    pucch_processor::process per PDU as uplink_processor_impl posts them: the calls that wait together share one
    slot-form launch per format (the plug-in's rendezvous).  Bars: the results of 64 threads identical to those of one
    thread (every result back to its own caller), far fewer launches than calls; the message rate at 16 / 64 / 256
    threads beside 16 threads of the reference's pucch_processor_impl (one cell's PDUs per thread, concurrently).
    Written to gpurun_out/pucch_rendezvous.json."""
    import json
    import threading

    import oracle
    import srsran_project_amd as amd
    from bench_pucch import NPRB, PORTS, cell_pdus

    ophy, _ = phy
    ncell = 64
    rng = np.random.default_rng(31)
    grids = [rng.integers(0, 1 << 32, (PORTS, 14, 12 * NPRB), dtype=np.uint64).astype(np.uint32) for _ in range(ncell)]
    dgs = [ophy.DeviceGrid(g, device=True) for g in grids]
    f0, f1, f2, f34 = cell_pdus(amd, 0)
    msgs = len(f0) + sum(b.nof_entries for b in f1) + len(f2) + len(f34)
    plug = ophy.PucchProcessorPlugin(device=0)
    _, serial = plug.mt_bench(dgs, f0, f1, f2, f34, 1, 1, NPRB)
    s0 = plug.stats()
    _, many = plug.mt_bench(dgs, f0, f1, f2, f34, 64, 1, NPRB)
    s1 = plug.stats()
    for a, b, name in zip(serial, many, ("f0", "f1", "f2", "p2", "f34", "p34")):
        assert np.array_equal(a, b), name
    calls = ncell * (len(f0) + len(f1) + len(f2) + len(f34))
    assert s1["errors"] == 0 and s1["batches"] - s0["batches"] < calls // 4, (s0, s1)
    out = {"cells": ncell, "messages_per_cell": msgs}
    for threads in (16, 64, 256):
        plug.mt_bench(dgs, f0, f1, f2, f34, threads, 1, NPRB)  # warm-up
        b0 = plug.stats()
        dt, _ = plug.mt_bench(dgs, f0, f1, f2, f34, threads, 5, NPRB)
        b1 = plug.stats()
        nb = max(b1["batches"] - b0["batches"], 1)
        out["plugin_%d_threads" % threads] = dict(
            messages_per_s=5 * ncell * msgs / dt, calls_per_batch=5 * calls / nb,
            batch_host_us=(b1["batch_host_us"] - b0["batch_host_us"]) / nb,
            batch_wait_us=(b1["batch_wait_us"] - b0["batch_wait_us"]) / nb)
    # the reference: 16 threads, each one pucch_processor_impl over one cell's PDUs (srs_ref_pucch_time)
    from srsran_project_amd.pucch import PucchF0Pdu, PucchF1Batch, PucchF2Pdu, PucchF34Pdu

    f = oracle.REF.srs_ref_pucch_time
    f.restype = ctypes.c_double
    P = ctypes.c_void_p
    f.argtypes = [P, ctypes.c_uint, ctypes.c_uint, P, ctypes.c_uint, P, ctypes.c_uint, P, ctypes.c_uint, P,
                  ctypes.c_uint, ctypes.c_uint]
    a0, a1 = (PucchF0Pdu * len(f0))(*f0), (PucchF1Batch * len(f1))(*f1)
    a2, a34 = (PucchF2Pdu * len(f2))(*f2), (PucchF34Pdu * len(f34))(*f34)
    reps = max(1, int(1.0 / max(f(grids[0].ctypes.data, PORTS, 12 * NPRB, a0, len(f0), a1, len(f1), a2, len(f2), a34,
                                  len(f34), 1), 1e-6)))
    threads = [threading.Thread(target=f, args=(grids[t].ctypes.data, PORTS, 12 * NPRB, a0, len(f0), a1, len(f1), a2,
                                                len(f2), a34, len(f34), reps)) for t in range(16)]
    t0 = time.perf_counter()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    out["reference_16_threads"] = dict(messages_per_s=16 * reps * msgs / (time.perf_counter() - t0))
    out["plugin_256_vs_reference_16"] = out["plugin_256_threads"]["messages_per_s"] / \
        out["reference_16_threads"]["messages_per_s"]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pucch_rendezvous.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)


# ---- the OFDM demodulator plug-in feeding the PUSCH plug-in on the device ----

def _time_domain(oracle, grid, slot, fc):
    """Each port of the slot through the reference's OFDM modulator (CPU), 100 MHz, 4096-point DFT, scale 1/64."""
    u16 = np.ascontiguousarray(grid).view(np.uint16).reshape(grid.shape[0], 14, -1)
    return np.stack([oracle.ref_ofdm_modulate_slot(u16[p], slot % 2, 1, 273, 4096, 1 / 64, fc)
                     for p in range(grid.shape[0])])


@pytest.mark.parametrize("form", [1, 0], ids=["symbol_form", "slot_form"])
def test_ofdm_demodulator_plugin_feeds_pusch_plugin_on_device(phy, form):
    """The uplink chain through the reference interfaces with the grid resident in HBM: the OFDM demodulator plug-in
    (ofdm_symbol_demodulator called per port and symbol as puxch_processor_impl.cpp:73-82 does; or the slot form)
    writes a hip_resource_grid's device copy in place, the PUSCH plug-in reads it there.  Bars: zero grid transfers
    (no download, no upload) up to the PUSCH results; the demodulated grid within one bf16 ulp of the reference's
    ofdm_slot_demodulator_impl on the same samples; the PUSCH plug-in equal to the reference's pusch_processor_impl on
    that grid (TB, CRC, LDPC statistics, UCI, CSI); end to end, the transport blocks and UCI the UEs sent, as the
    reference's chain (its demodulator, then pusch_processor_impl) also returns."""
    from pusch_slot_cases import NSUBC

    ophy, oracle = phy
    slot, fc = 3, 3.5e9
    grid, ues = _fapi_slot(ophy, slot, seed=17, kinds=["dc_data", "uci_data", "tp", "two_layer"])
    x = _time_domain(oracle, grid, slot, fc)
    dg = ophy.DeviceGrid(shape=(4, 14, NSUBC))
    ophy.ofdm_demodulate(dg, x, slot % 2, 1, 273, 4096, fc, scale=1 / 64, form=form)
    plug = ophy.PuschProcessorPlugin(device=0, iterations=ITERS)
    tickets = [plug.process_fapi(dg, fp) for _, fp, _, _ in ues]
    plug.flush()
    plug.wait()
    assert dg.transfers() == dict(downloads=0, uploads=0)
    assert plug.stats()["device_grids"] >= 1 and plug.stats()["errors"] == 0
    got_grid = dg.read()  # (the first host access: one download)
    want_grid = np.stack([oracle.ref_ofdm_demodulate_slot(x[p], slot % 2, 1, 273, 4096, 1 / 64, fc)
                          for p in range(4)]).view(np.uint32)
    a = (got_grid.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    b = (want_grid.view(np.uint16).astype(np.uint32) << 16).view(np.float32)
    tol = 2.0 ** -7 * np.maximum(np.abs(a), np.abs(b)) + 3e-5 * np.sqrt(np.mean(b ** 2))
    assert (np.abs(a - b) <= tol).all() and (got_grid == want_grid).mean() >= 0.99
    same, ref_chain = ophy.Grid(got_grid), ophy.Grid(want_grid)
    for (kind, fp, tb_sent, uci), (t, tb) in zip(ues, tickets):
        got = plug.result(t, fp.fapi.harq_ack_bit_length, fp.fapi.csi_part1_bit_length)
        want_tb, want = ophy.ref_pusch_process_fapi(same, fp, iterations=ITERS)
        _check(got, want, kind)
        assert np.array_equal(tb, want_tb) and got["tb_crc_ok"] and np.array_equal(tb, tb_sent), kind
        chain_tb, chain = ophy.ref_pusch_process_fapi(ref_chain, fp, iterations=ITERS)
        assert chain["tb_crc_ok"] and np.array_equal(chain_tb, tb), kind
        if uci is not None:
            assert np.array_equal(got["harq_ack"], uci[0]) and np.array_equal(got["csi_part1"], uci[1]), kind
            assert np.array_equal(chain["harq_ack"], uci[0]) and np.array_equal(chain["csi_part1"], uci[1]), kind


def _random_grid(seed, ports=4):
    from oracle import ofdm as oofdm
    from pusch_slot_cases import NSUBC

    rng = np.random.default_rng(seed)
    return np.stack([oofdm.random_grid(rng, 14, NSUBC) for _ in range(ports)]).view(np.uint32)


@pytest.mark.parametrize("form", [1, 0], ids=["symbol_form", "slot_form"])
def test_ofdm_modulator_plugin_reads_device_grid(phy, form):
    """The downlink end of the chain: a grid written on the device (as the PDSCH plug-in leaves it) modulated by the
    OFDM modulator plug-in in place -- every port of the slot in one launch at the first call, later calls served from
    that launch -- with zero grid transfers; samples within 2e-5 x RMS of the reference's ofdm_slot_modulator_impl on
    the same grid.  The symbol form again on the same grid rewritten on the device and through the host writer: the
    plug-in's per-slot samples follow the grid's content (no stale slot)."""
    ophy, oracle = phy
    slot, fc = 1, 3.5e9
    g0, g1 = _random_grid(21), _random_grid(22)

    def want(g):
        u16 = g.view(np.uint16).reshape(4, 14, -1)
        return np.stack([oracle.ref_ofdm_modulate_slot(u16[p], slot, 1, 273, 4096, 1 / 64, fc) for p in range(4)])

    w0, w1 = want(g0), want(g1)
    rms = float(np.sqrt(np.mean(np.abs(w0) ** 2)))
    dg = ophy.DeviceGrid(g0, device=True)
    got = ophy.ofdm_modulate(dg, 4, slot, 1, 273, 4096, fc, 1 / 64, w0.shape[1], form=form)
    assert dg.transfers() == dict(downloads=0, uploads=0)
    assert np.max(np.abs(got - w0)) <= 2e-5 * rms
    if form == 1:
        for on_host in (False, True):
            dg = ophy.DeviceGrid(g0, device=True)
            y0, y1 = ophy.ofdm_modulate_twice(dg, 4, slot, 1, 273, 4096, fc, 1 / 64, w0.shape[1], g1, on_host)
            assert np.max(np.abs(y0 - w0)) <= 2e-5 * rms, on_host
            assert np.max(np.abs(y1 - w1)) <= 2e-5 * rms, on_host
            # (a host write after device writes merges the device's changes into the host mirror first: one download)
            assert dg.transfers()["downloads"] == int(on_host), on_host


def test_ofdm_symbol_plugin_rate(phy):
    """Symbol-form OFDM as the lower PHY drives it (one ofdm_symbol_(de)modulator per sector, one call per port and
    symbol): 16 sector threads through the plug-ins on device-resident grids -- the demodulator staging its symbols
    and launching a slot at a time (the timed region ends when every kernel has completed), the modulator launching
    every port of a slot at its first call on a grid rewritten on the device every slot -- beside 16 threads of the
    reference's ofdm_symbol_(de)modulator_impl (generic DFT), 100 MHz / 4096-point / 4 ports; also one sector alone
    (host time per call).  Zero grid transfers.  Written to gpurun_out/ofdm_symbol_plugin_rate.json."""
    import json

    ophy, oracle = phy
    rng = np.random.default_rng(5)
    x = (rng.normal(size=(4, 61440)) + 1j * rng.normal(size=(4, 61440))).astype(np.complex64) * 0.1
    g = _random_grid(23)
    out = {}
    for kind, modulate in (("demodulator", False), ("modulator", True)):
        ophy.ofdm_symbol_bench(1, 1, 1, 273, 4096, x, 2, modulate=modulate, grid=g)  # warm-up (code objects, pinned)
        res = {}
        for name, plugin, threads, slots in (("plugin_1_sector", 1, 1, 200), ("plugin_16_sectors", 1, 16, 100),
                                             ("reference_16_threads", 0, 16, 4)):
            dt, us_call, xfer = ophy.ofdm_symbol_bench(plugin, threads, 1, 273, 4096, x, slots, modulate=modulate,
                                                       grid=g)
            assert xfer == 0
            res[name] = dict(symbols_per_s=threads * slots * 14 * 4 / dt, host_us_per_call=us_call,
                             slot_us_per_sector=1e6 * dt / slots, threads=threads)
        res["plugin_vs_reference_16"] = res["plugin_16_sectors"]["symbols_per_s"] / res["reference_16_threads"][
            "symbols_per_s"]
        out[kind] = res
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/ofdm_symbol_plugin_rate.json", "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)

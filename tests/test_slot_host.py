"""Host logic of the heterogeneous slot forms (no GPU): the sch_slot workload's plans (TS 38.212 7.2.2
base-graph rule, TBS from the reference's tbs_calculator restatement) and the SlotUes descriptor arrays
(C layout of srs_amd_pusch_ue / srs_amd_pdsch_ue, buffer extents)."""
import ctypes

import bench_slot
import srsran_project_amd as amd


def test_descriptor_layout_matches_c():
    # srs_amd_sch_plan (19 x uint32 = 76 B) then two uint64 at 8-byte alignment
    assert ctypes.sizeof(amd.SchPlan) == 76
    for kind in (amd.PuschUe, amd.PdschUe):
        assert ctypes.sizeof(kind) == 96
        assert kind.plan.offset == 0
    assert amd.PuschUe.llr_offset.offset == 80 and amd.PuschUe.tb_offset.offset == 88
    assert amd.PdschUe.tb_offset.offset == 80 and amd.PdschUe.cw_offset.offset == 88


def test_slot_plans_and_extents():
    plans = bench_slot.make_slot(amd, 4, 8, 3)
    assert len(plans) == 32
    for p in plans:
        rate = p.tbs / p.cw_length
        want_bg = 2 if (p.tbs <= 292 or (p.tbs <= 3824 and rate <= 0.67) or rate <= 0.25) else 1
        # the plan's BG follows the target-rate rule; the realised rate can differ slightly from the target
        assert p.base_graph in (1, 2) and p.nof_segments >= 1 and p.cw_length == p.nof_ch_symbols * p.modulation_order
        assert p.base_graph == want_bg or abs(rate - 0.67) < 0.1 or abs(rate - 0.25) < 0.1
    ues, pos, tpos = [], 0, 0
    for p in plans:
        ues.append((p, pos, tpos))
        pos += p.cw_length + 3
        tpos += p.tbs // 8 + 1
    d = amd.SlotUes(amd.PuschUe, ues)
    assert d.n == 32 and d.data_end == pos - 3 and d.out_end == tpos - 1
    assert d.arr[5].llr_offset == ues[5][1] and d.arr[5].plan.tbs == plans[5].tbs
    e = amd.SlotUes(amd.PdschUe, [(p, t, c) for (p, c, t) in ues])
    assert e.data_end == tpos - 1 and e.out_end == max(c + (p.cw_length + 7) // 8 for p, c, _ in ues)

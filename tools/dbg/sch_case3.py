import sys, ctypes, numpy as np, torch
sys.path.insert(0, '.')
import srsran_project_amd as amd, oracle, oracle.sch as osch
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes
dec = amd.PuschDecoder("simd")
explicit = sys.argv[1] == "1"
for ci in range(6):
    tbs, bg, qm, lay, nre, rv, nref = SCH_CASES[ci]
    p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre); op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
    tbl = tb_bytes(p.tbs, 7 * ci)
    llrs = noisy_llrs(osch.pdsch_encode(tbl, op), 10, 4, seed=0)[None]
    C = p.nof_segments
    cb_it = torch.zeros(C, dtype=torch.int32, device="cuda")
    soft = torch.zeros(amd.soft_buffer_size(p), dtype=torch.int8, device="cuda") if explicit else None
    d_tb, res = dec.decode_batch(torch.from_numpy(llrs).cuda(), p, amd.PuschDecoder.config(), cb_iterations=cb_it, soft=soft)
    torch.cuda.synchronize()
    h = osch.HarqBuffer(op); out = np.zeros(tbs // 8, np.uint8)
    o = osch.pusch_decode(llrs[0], op, h, out, 6, "simd")
    print(ci, "gpu", res.cpu().numpy()[0], cb_it.cpu().numpy(), "oracle", o[0], o[1])
    if soft is not None:
        rows = soft.cpu().numpy().reshape(C, -1)
        N = h.soft[0].size
        print("   soft rows equal", [bool(np.array_equal(rows[r, :N], h.soft[r])) for r in range(C)])

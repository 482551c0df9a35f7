import sys, numpy as np, torch
sys.path.insert(0, '.')
import srsran_project_amd as amd, oracle, oracle.sch as osch
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes
dec = amd.PuschDecoder("simd")
for ci in range(int(sys.argv[1]) + 1):
    tbs, bg, qm, lay, nre, rv, nref = SCH_CASES[ci]
    p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre); op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
    n = int(sys.argv[2])
    tbl = [tb_bytes(p.tbs, 7 * ci + k) for k in range(n)]
    llrs = np.stack([noisy_llrs(osch.pdsch_encode(tbl[k], op), 10, 4 + 4 * k, seed=k) for k in range(n)])
    C = p.nof_segments
    cb_it = torch.zeros(n * C, dtype=torch.int32, device="cuda")
    d_tb, res = dec.decode_batch(torch.from_numpy(llrs).cuda(), p, amd.PuschDecoder.config(), cb_iterations=cb_it)
    torch.cuda.synchronize()
    for k in range(n):
        h = osch.HarqBuffer(op); out = np.zeros(tbs // 8, np.uint8)
        o = osch.pusch_decode(llrs[k], op, h, out, 6, "simd")
        g = res.cpu().numpy()[k]
        same = bool(g[0]) == o[0] and np.array_equal(d_tb.cpu().numpy()[k], out)
        print(ci, k, "gpu", g, cb_it.cpu().numpy().reshape(n, C)[k], "oracle", o[0], o[1], "same", same)

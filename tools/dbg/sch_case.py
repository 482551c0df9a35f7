import sys, numpy as np, torch
sys.path.insert(0, '.')
import srsran_project_amd as amd, oracle, oracle.sch as osch
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes
ci = int(sys.argv[1])
tbs, bg, qm, lay, nre, rv, nref = SCH_CASES[ci]
p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre); op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
print(op)
tb = tb_bytes(tbs, 7 * ci)
llr = noisy_llrs(osch.pdsch_encode(tb, op), 10, 4, seed=0)
dec = amd.PuschDecoder("simd")
C = p.nof_segments
cb_it = torch.zeros(C, dtype=torch.int32, device="cuda")
soft = torch.zeros(amd.soft_buffer_size(p), dtype=torch.int8, device="cuda")
d_tb, res = dec.decode_batch(torch.from_numpy(llr[None]).cuda(), p, amd.PuschDecoder.config(), cb_iterations=cb_it, soft=soft)
torch.cuda.synchronize()
print("gpu", res.cpu().numpy(), cb_it.cpu().numpy())
h = osch.HarqBuffer(op); out = np.zeros(tbs // 8, np.uint8)
print("oracle", osch.pusch_decode(llr, op, h, out, 6, "simd"))
rows = soft.cpu().numpy().reshape(C, -1)
N = h.soft[0].size
for r in range(C):
    print(r, "soft equal", np.array_equal(rows[r, :N], h.soft[r]), np.flatnonzero(rows[r, :N] != h.soft[r])[:10])

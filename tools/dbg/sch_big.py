import sys, numpy as np, torch
sys.path.insert(0, '.')
import srsran_project_amd as amd, oracle, oracle.sch as osch
from tests.sch_cases import tb_bytes, noisy_llrs
nre = 273 * 12 * 12
p = amd.sch_plan(8 * 78000, 1, 0, 8, 0, 2, nre * 2); op = p.as_dict()
print(op)
enc = amd.PdschEncoder(); dec = amd.PuschDecoder()
rows = torch.from_numpy(np.stack([tb_bytes(p.tbs, k) for k in range(2)])).cuda()
cw = enc.encode_batch(rows, p)
torch.cuda.synchronize()
cwb = np.unpackbits(cw.cpu().numpy(), axis=1)[:, :p.cw_length]
want = osch.pdsch_encode(rows[0].cpu().numpy(), op)
print("encode equal oracle", np.array_equal(cwb[0], want), np.flatnonzero(cwb[0] != want)[:10])
llrs = torch.from_numpy(((1 - 2 * cwb.astype(np.int16)) * 40).astype(np.int8)).cuda()
cb_it = torch.zeros(2 * p.nof_segments, dtype=torch.int32, device="cuda")
d_tb, res = dec.decode_batch(llrs.contiguous(), p, amd.PuschDecoder.config(), cb_iterations=cb_it)
torch.cuda.synchronize()
print(res.cpu().numpy(), cb_it.cpu().numpy()[:80])
print("tb equal", torch.equal(d_tb, rows))
h = osch.HarqBuffer(op); out = np.zeros(p.tbs // 8, np.uint8)
o = osch.pusch_decode(llrs[0].cpu().numpy(), op, h, out, 6, "simd")
print("oracle", o[0], o[1][:10], np.array_equal(out, rows[0].cpu().numpy()))

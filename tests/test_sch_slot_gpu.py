"""GPU parity: heterogeneous slot decoding / encoding (srs_amd_pusch_decode_slot, srs_amd_pdsch_encode_slot).
Decoding: the new transmissions of
UEs with different plans (TBS, base graph, lifting size, Qm, layers, rv, limited buffer) decoded as
one launch sequence -- against oracle/sch.py per UE, itself bit-exact with the reference's
pusch_decoder_impl (tests/test_oracle_vs_ref.py).  Bar: bit-exact TB bytes, TB CRC status and
LDPC statistics for every UE, whatever its position, alignment or bucket in the batch."""
import numpy as np
import pytest

import oracle.sch as osch
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes

pytestmark = pytest.mark.gpu

# (tbs, base graph, Qm, layers, channel symbols, rv, Nref): SCH_CASES plus high-rate BG1 Z = 384
# codeblocks of the 100 MHz slot (the LDPC high-rate kernel's bucket, CRC24B) with different Qm / F.
SLOT_CASES = SCH_CASES + [
    (8 * 20000, 1, 8, 2, 21504, 0, 0),     # 256QAM R ~ 0.93, C = 19
    (8 * 9000, 1, 6, 2, 12960, 0, 0),      # 64QAM high rate, C = 9
    (8 * 30000, 1, 8, 4, 32256, 0, 0),     # 256QAM 4 layers, C = 29
    (8 * 6000, 1, 4, 1, 13000, 2, 0),      # rv 2 new data (k0 != 0: whole soft row)
    # one mixed-Z bucket, same rv / Qm / Nref / F = 0, equal dematcher write ends: Z = 32 with E > Ncb
    # (whole row, 66 x 32 = 2112) and Z = 64 whose bounded prefix is also 2112 = 33 x 64 -- their
    # rate-matching geometries must stay apart
    (688, 1, 2, 1, 1100, 0, 0),
    (1392, 1, 2, 1, 1025, 0, 0),
]


def _ues(seed, order):
    import srsran_project_amd as amd

    rng = np.random.default_rng(seed)
    ues, llr_chunks, want_tbs, pos, tpos = [], [], [], 0, 0
    for k, ci in enumerate(order):
        tbs, bg, qm, lay, nre, rv, nref = SLOT_CASES[ci]
        p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre)
        op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
        tb = tb_bytes(tbs, 1000 * seed + k)
        sigma = [3, 6, 9, 30][k % 4]  # easy ... undecodable
        llr = noisy_llrs(osch.pdsch_encode(tb, op), 10, sigma, seed=7 * seed + k)
        pos += int(rng.integers(0, 40))  # arbitrary (also odd) codeword offsets
        tpos += int(rng.integers(0, 9))
        ues.append((p, pos, tpos, op, llr, tb))
        pos += llr.size
        tpos += tbs // 8
    flat = np.zeros(pos + 64, np.int8)
    for p, lo, _, _, llr, _ in ues:
        flat[lo:lo + llr.size] = llr
    return ues, flat, tpos


@pytest.fixture(scope="module")
def decs():
    import srsran_project_amd as amd

    return {"simd": amd.PuschDecoder("simd"), "generic": amd.PuschDecoder("generic")}


@pytest.mark.parametrize("arith", ["simd", "generic"])
@pytest.mark.parametrize("early", [True, False])
def test_decode_slot_matches_oracle(decs, arith, early):
    import torch

    import srsran_project_amd as amd

    n = len(SLOT_CASES)
    # every case twice, interleaved so buckets and plans alternate along the batch
    order = list(range(n)) + list(reversed(range(n)))
    ues, flat, tb_total = _ues(3 + int(early), order)
    cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6, use_early_stop=early)
    d_tb, res = decs[arith].decode_slot(torch.from_numpy(flat).cuda(), [(u[0], u[1], u[2]) for u in ues], cfg)
    torch.cuda.synchronize()
    d_tb, res = d_tb.cpu().numpy(), res.cpu().numpy()
    for u, (p, _, to, op, llr, tb) in enumerate(ues):
        h = osch.HarqBuffer(op)
        out = np.zeros(p.tbs // 8, np.uint8)
        ok, iters, stats = osch.pusch_decode(llr, op, h, out, 6, arith, use_early_stop=early)
        msg = "UE %d (case %d)" % (u, order[u])
        assert bool(res[u, 0]) == ok, msg
        assert res[u, 1] == p.nof_segments, msg
        assert (res[u, 2], res[u, 3], res[u, 4]) == (sum(stats), min(stats), max(stats)), msg
        assert res[u, 5] == sum(i is not None for i in iters), msg
        np.testing.assert_array_equal(d_tb[to:to + p.tbs // 8], out, err_msg=msg)
        if u % 4 == 0 and SLOT_CASES[order[u]][5] == 0:
            assert ok and np.array_equal(out, tb), msg


def test_decode_slot_equals_uniform_batches(decs):
    """A slot of many UEs equals decoding each UE alone through srs_amd_pusch_decode_batch."""
    import torch

    import srsran_project_amd as amd

    order = [8, 9, 3, 10, 8, 4, 9, 7, 10, 8, 11, 5]
    ues, flat, _ = _ues(11, order)
    cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6)
    d_tb, res = decs["simd"].decode_slot(torch.from_numpy(flat).cuda(), [(u[0], u[1], u[2]) for u in ues], cfg)
    for u, (p, _, to, _, llr, _) in enumerate(ues):
        tb1, res1 = decs["simd"].decode_batch(torch.from_numpy(llr[None, :].copy()).cuda(), p, cfg)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(res[u].cpu().numpy(), res1[0].cpu().numpy(), err_msg="UE %d" % u)
        np.testing.assert_array_equal(d_tb[to:to + p.tbs // 8].cpu().numpy(), tb1[0].cpu().numpy(),
                                      err_msg="UE %d" % u)


def test_decode_slot_rejects_retransmissions(decs):
    import torch

    import srsran_project_amd as amd

    p = amd.sch_plan(*[SLOT_CASES[1][i] for i in (0, 1, 5, 2, 6, 3, 4)])
    llrs = torch.zeros(p.cw_length, dtype=torch.int8, device="cuda")
    with pytest.raises(ValueError):
        decs["simd"].decode_slot(llrs, [(p, 0, 0)], amd.PuschDecoder.config(new_data=False))
    tbs, res = decs["simd"].decode_slot(llrs, [], amd.PuschDecoder.config())
    assert res.shape[0] == 0


@pytest.fixture(scope="module")
def enc():
    import srsran_project_amd as amd

    return amd.PdschEncoder()


def test_encode_slot_matches_oracle(enc):
    """PDSCH side: the codewords of UEs with different plans encoded as one launch sequence
    (srs_amd_pdsch_encode_slot), each bit-exact with oracle/sch.py's pdsch_encoder_impl restatement;
    bytes between the codewords untouched."""
    import torch

    import srsran_project_amd as amd

    n = len(SLOT_CASES)
    order = list(range(n)) + list(reversed(range(n))) + [8, 10, 8]
    rng = np.random.default_rng(5)
    ues, tb_chunks, tpos, cpos = [], [], 0, 0
    for k, ci in enumerate(order):
        tbs, bg, qm, lay, nre, rv, nref = SLOT_CASES[ci]
        p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre)
        op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
        tpos += int(rng.integers(0, 9))
        cpos += int(rng.integers(1, 9))  # a gap byte before every codeword
        ues.append((p, tpos, cpos, op, tb_bytes(tbs, 500 + k)))
        tpos += tbs // 8
        cpos += (p.cw_length + 7) // 8
    flat = np.zeros(tpos + 16, np.uint8)
    for p, to, _, _, tb in ues:
        flat[to:to + tb.size] = tb
    out = torch.full((cpos + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    enc.encode_slot(torch.from_numpy(flat).cuda(), [(u[0], u[1], u[2]) for u in ues], out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    covered = np.zeros(got.size, bool)
    for u, (p, _, co, op, tb) in enumerate(ues):
        nb = (p.cw_length + 7) // 8
        bits = np.unpackbits(got[co:co + nb])
        np.testing.assert_array_equal(bits[:p.cw_length], osch.pdsch_encode(tb, op),
                                      err_msg="UE %d (case %d)" % (u, order[u]))
        assert not bits[p.cw_length:].any(), "UE %d: padding bits" % u
        covered[co:co + nb] = True
    assert (got[~covered] == 0xA5).all(), "bytes outside the codewords written"


def test_encode_slot_equals_uniform_batch(enc):
    """Many UEs of one plan through encode_slot equal srs_amd_pdsch_encode_batch."""
    import torch

    import srsran_project_amd as amd

    tbs, bg, qm, lay, nre, rv, nref = SLOT_CASES[10]
    p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre)
    m, tbb, cwb = 6, tbs // 8, (p.cw_length + 7) // 8
    rows = np.stack([tb_bytes(tbs, 900 + k) for k in range(m)])
    d_rows = torch.from_numpy(rows).cuda()
    want = enc.encode_batch(d_rows, p).cpu().numpy()
    got = enc.encode_slot(d_rows.reshape(-1), [(p, k * tbb, k * cwb) for k in range(m)]).cpu().numpy()
    for k in range(m):
        np.testing.assert_array_equal(got[k * cwb:(k + 1) * cwb], want[k, :cwb], err_msg="TB %d" % k)


@pytest.mark.parametrize("early", [True, False])
def test_realistic_slot_equals_per_ue(decs, enc, early):
    """A slot as bench.py --workload sch_slot builds it (4 cells x 8 UEs: random PRB split, MCS QPSK..256QAM,
    1-4 layers; ~20 lifting sizes, mixed-Z decoder launches) encodes and decodes exactly as one per-plan
    batch per UE."""
    import torch

    import bench_slot
    import srsran_project_amd as amd

    plans = bench_slot.make_slot(amd, 4, 8, 77)
    tx, rx, tpos, cpos = [], [], 0, 0
    for p in plans:
        tx.append((p, tpos, cpos))
        rx.append((p, 8 * cpos, tpos))
        tpos += p.tbs // 8
        cpos += (p.cw_length + 7) // 8
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    tbs = torch.randint(0, 256, (tpos,), device="cuda", generator=g, dtype=torch.uint8)
    cws = enc.encode_slot(tbs, tx)
    bits = ((cws[:, None] >> torch.arange(7, -1, -1, device="cuda", dtype=torch.uint8)) & 1).reshape(-1).float()
    sigma = torch.rand(bits.shape, device="cuda", generator=g) * 12  # from clean to undecodable
    llrs = ((1 - 2 * bits) * 10 + sigma * torch.randn(bits.shape, device="cuda", generator=g)).round()
    llrs = llrs.clamp(-120, 120).to(torch.int8)
    cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6, use_early_stop=early)
    d_tb, res = decs["simd"].decode_slot(llrs, rx, cfg)
    torch.cuda.synchronize()
    for u, ((p, to, co), (_, lo, _)) in enumerate(zip(tx, rx)):
        cw1 = enc.encode_batch(tbs[to:to + p.tbs // 8].view(1, -1), p)
        nb = (p.cw_length + 7) // 8
        assert torch.equal(cw1[0, :nb], cws[co:co + nb]), "UE %d codeword" % u
        tb1, res1 = decs["simd"].decode_batch(llrs[lo:lo + p.cw_length].view(1, -1), p, cfg)
        assert torch.equal(res[u], res1[0]), "UE %d: %s vs %s" % (u, res[u].tolist(), res1[0].tolist())
        assert torch.equal(d_tb[to:to + p.tbs // 8], tb1[0]), "UE %d TB" % u


def _every_z_cases():
    """One transport block per (base graph, lifting size, layers): C = 1 with the lifting size Z selected
    (BG1: TBS + 24 just above 22 (Z_prev); BG2: TBS > 640 so K_b = 10), the PDSCH PDU shapes of the plug-in tests
    (1-4 layers, QPSK..256QAM), codeword of about TBS / 0.6 bits."""
    import srsran_project_amd as amd

    out = []
    zs = list(amd.LIFTING_SIZES)
    for bg, kb, crc, lo in ((1, 22, 24, 0), (2, 10, 24, 656)):
        for i, Z in enumerate(zs):
            kmax = kb * Z - crc
            kmin = kb * zs[i - 1] - crc + 1 if i else 8
            tbs = (kmax // 8) * 8
            if tbs < max(kmin, lo + 8) or tbs > (8424 if bg == 1 else 3816):
                continue
            lay, qm = 1 + i % 4, (2, 4, 6, 8)[(i // 4) % 4]
            nre = -(-int(tbs / 0.6) // (lay * qm)) * lay
            out.append((tbs, bg, qm, lay, nre, 0, 0))
    # segmented: Z = 352, C = 6, 3 layers 16QAM (the pdsch_processor plug-in test's third PDU)
    out.append((44040, 1, 4, 3, 23040, 0, 0))
    return out


@pytest.mark.parametrize("case", _every_z_cases())
def test_encode_every_lifting_size(enc, case):
    """Every lifting size of both base graphs (one transport block each, 1-4 layers) through the batch and slot
    encoders, bit-exact with the reference's pdsch_encoder_impl (oracle.ref_pdsch_encode, the compiled reference)."""
    import torch

    import oracle
    import srsran_project_amd as amd

    tbs, bg, qm, lay, nre, rv, nref = case
    p = amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre)
    op = osch.plan(tbs, bg, rv, qm, nref, lay, nre)
    assert p.as_dict()["lifting_size"] == op["lifting_size"]
    tb = tb_bytes(tbs, 77 + tbs)
    want = oracle.ref_pdsch_encode(tb, op)
    d_tb = torch.from_numpy(tb[None]).cuda()
    got_b = enc.encode_batch(d_tb, p)
    out = torch.zeros((p.cw_length + 7) // 8 + 8, dtype=torch.uint8, device="cuda")
    enc.encode_slot(torch.from_numpy(tb).cuda(), [(p, 0, 0)], out=out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(np.unpackbits(got_b[0].cpu().numpy())[:p.cw_length], want, err_msg="batch")
    np.testing.assert_array_equal(np.unpackbits(out.cpu().numpy())[:p.cw_length], want, err_msg="slot")


def test_encode_slot_mixed_lifting_sizes_in_one_launch(enc):
    """The transport blocks of one PDSCH slot with four different geometries -- Z = 288 (C = 2, 1 layer QPSK),
    Z = 384 (C = 9, 2 layers 64QAM), Z = 352 (C = 6, 3 layers 16QAM), Z = 384 (C = 23, 4 layers 256QAM) -- encoded by
    one srs_amd_pdsch_encode_slot call, each bit-exact with the reference's pdsch_encoder_impl."""
    import torch

    import oracle
    import srsran_project_amd as amd

    cases = [(11528, 1, 2, 1, 8640), (73776, 1, 6, 2, 2 * 10980), (44040, 1, 4, 3, 3 * 7680),
             (192624, 1, 8, 4, 4 * 7800)]
    ues, tbs_flat, tpos, cpos, want = [], [], 0, 0, []
    for k, (tbs, bg, qm, lay, nch) in enumerate(cases):
        p = amd.sch_plan(tbs, bg, 0, qm, 25344, lay, nch)
        op = osch.plan(tbs, bg, 0, qm, 25344, lay, nch)
        tb = tb_bytes(tbs, 900 + k)
        want.append(oracle.ref_pdsch_encode(tb, op))
        ues.append((p, tpos, cpos))
        tbs_flat.append(np.concatenate([tb, np.zeros((-tb.size) % 64, np.uint8)]))
        tpos += tbs_flat[-1].size
        cpos += ((p.cw_length + 511) // 512) * 64
    out = torch.zeros(cpos, dtype=torch.uint8, device="cuda")
    enc.encode_slot(torch.from_numpy(np.concatenate(tbs_flat)).cuda(), ues, out=out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for k, ((p, _, co), w) in enumerate(zip(ues, want)):
        bits = np.unpackbits(got[co:co + (p.cw_length + 7) // 8])[:p.cw_length]
        assert np.array_equal(bits, w), (k, int((bits != w).sum()), int(np.flatnonzero(bits != w)[0]))


@pytest.mark.parametrize("case", [(40, 2, 2, 34), (64, 2, 3, 54), (304, 8, 2, 64), (96, 4, 4, 20)])
def test_small_z_codeblock_stages(enc, case):
    """Small lifting sizes (C = 1) stage by stage: the single and batch LDPC encoders (whole codeblock), then the
    single and batch rate matchers on the oracle's codeblock, against oracle/sch.py's restatement."""
    import torch

    import oracle
    import srsran_project_amd as amd

    tbs, qm, lay, nch = case
    op = osch.plan(tbs, 1, 0, qm, 0, lay, nch)
    Z, F, E, K = op["lifting_size"], op["nof_filler_bits"], op["cw_length"], op["segment_length"]
    tb = np.unpackbits(tb_bytes(tbs, 77 + tbs))
    c = oracle.crc_bits(osch._tb_crc_poly(op), tb)
    L = op["nof_tb_crc_bits"]
    msg = np.zeros(K, np.uint8)
    msg[:tbs + L] = np.concatenate([tb, [(c >> (L - 1 - k)) & 1 for k in range(L)]])
    want_cb = oracle.ldpc_encode(msg, 1, Z)
    cfg = amd.LdpcEncoderConfiguration(base_graph=1, lifting_size=Z)
    e1 = amd.LdpcEncoder()
    got1 = e1.encode(msg, cfg)
    d = np.flatnonzero(got1[:want_cb.size] != want_cb)
    assert d.size == 0, "single encoder Z %d: %s" % (Z, d[:8].tolist())
    gotb = e1.encode_batch(torch.from_numpy(np.packbits(msg)).cuda().reshape(1, -1).contiguous(), cfg).cpu().numpy()
    d = np.flatnonzero(np.unpackbits(gotb[0])[:want_cb.size] != want_cb)
    assert d.size == 0, "batch encoder Z %d: %s" % (Z, d[:8].tolist())
    want = osch.unpack_bits(oracle.rate_match(want_cb, 1, Z, 0, qm, E, 0, F), E)
    meta = amd.CodeblockMetadata(base_graph=1, lifting_size=Z, rv=0, modulation_order=qm, Nref=0, nof_filler_bits=F)
    rm = amd.LdpcRateMatcher()
    got = np.unpackbits(rm.rate_match(E, want_cb, meta))[:E]
    d = np.flatnonzero(got != want)
    assert d.size == 0, "single rate matcher Z %d F %d E %d: %s" % (Z, F, E, d[:8].tolist())
    got = np.unpackbits(rm.rate_match_batch(torch.from_numpy(np.packbits(want_cb)).cuda().reshape(1, -1).contiguous(), [E], meta)
                        .cpu().numpy())[:E]
    d = np.flatnonzero(got != want)
    assert d.size == 0, "batch rate matcher Z %d F %d E %d: %s" % (Z, F, E, d[:8].tolist())

"""GPU parity: the MI355X PDSCH encoder and PUSCH decoder (transport-block chain,
through the C-ABI) vs oracle/sch.py, itself bit-exact with the reference's
pdsch_encoder_impl / pusch_decoder_impl (tests/test_oracle_vs_ref.py).
Bar: bit-exact codewords, transport blocks, TB CRC status, per-codeblock
iteration counts and LDPC statistics; HARQ combining across transmissions."""
import numpy as np
import pytest

import oracle.sch as osch
from tests.sch_cases import SCH_CASES, noisy_llrs, tb_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    import srsran_project_amd as amd

    return amd.PdschEncoder()


@pytest.fixture(scope="module")
def decs():
    import srsran_project_amd as amd

    return {"simd": amd.PuschDecoder("simd"), "generic": amd.PuschDecoder("generic")}


def _plan(case):
    import srsran_project_amd as amd

    tbs, bg, qm, lay, nre, rv, nref = case
    return amd.sch_plan(tbs, bg, rv, qm, nref, lay, nre), osch.plan(tbs, bg, rv, qm, nref, lay, nre)


@pytest.mark.parametrize("overlap", ["0", "1"])
@pytest.mark.parametrize("ci", range(len(SCH_CASES)))
def test_pdsch_encode(enc, ci, overlap, monkeypatch):
    """Host and batch forms against the oracle; the batch with and without the TB-CRC overlap on a helper stream
    (SRSRAN_AMD_PDSCH_OVERLAP)."""
    import torch

    monkeypatch.setenv("SRSRAN_AMD_PDSCH_OVERLAP", overlap)

    p, op = _plan(SCH_CASES[ci])
    assert p.as_dict() == op
    tbs = p.tbs
    tb = tb_bytes(tbs, ci)
    want = osch.pdsch_encode(tb, op)
    np.testing.assert_array_equal(enc.encode(tb, p), want)
    # Batch of 5 TBs in padded rows.
    rows = np.stack([tb_bytes(tbs, 100 * ci + k) for k in range(5)])
    padded = np.zeros((5, tbs // 8 + 13), np.uint8)
    padded[:, :tbs // 8] = rows
    out = enc.encode_batch(torch.from_numpy(padded).cuda(), p)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for k in range(5):
        np.testing.assert_array_equal(np.unpackbits(got[k])[:p.cw_length], osch.pdsch_encode(rows[k], op),
                                      err_msg="TB %d" % k)


@pytest.mark.parametrize("arith", ["simd", "generic"])
@pytest.mark.parametrize("early", [True, False])
def test_pusch_decode_batch(decs, arith, early):
    import torch

    import srsran_project_amd as amd

    for ci, case in enumerate(SCH_CASES):
        p, op = _plan(case)
        n = 4
        tbs = [tb_bytes(p.tbs, 7 * ci + k) for k in range(n)]
        # Noise from easy (k = 0) to undecodable (k = 3).
        llrs = np.stack([noisy_llrs(osch.pdsch_encode(tbs[k], op), 10, 4 + 4 * k, seed=k) for k in range(n)])
        cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6, use_early_stop=early)
        C = p.nof_segments
        cb_it = torch.zeros(n * C, dtype=torch.int32, device="cuda")
        d_tb, res = decs[arith].decode_batch(torch.from_numpy(llrs).cuda(), p, cfg, cb_iterations=cb_it)
        torch.cuda.synchronize()
        d_tb, res, cb_it = d_tb.cpu().numpy(), res.cpu().numpy(), cb_it.cpu().numpy().reshape(n, C)
        for k in range(n):
            h = osch.HarqBuffer(op)
            out = np.zeros(p.tbs // 8, np.uint8)
            ok, iters, stats = osch.pusch_decode(llrs[k], op, h, out, 6, arith, use_early_stop=early)
            msg = "case %d TB %d" % (ci, k)
            assert bool(res[k, 0]) == ok, msg
            assert res[k, 1] == C
            assert (res[k, 2], res[k, 3], res[k, 4]) == (sum(stats), min(stats), max(stats)), msg
            assert res[k, 5] == sum(i is not None for i in iters), msg
            np.testing.assert_array_equal(cb_it[k], [-1 if i is None else i for i in iters], err_msg=msg)
            np.testing.assert_array_equal(d_tb[k], out, err_msg=msg)
            if k == 0 and case[5] == 0:
                assert ok and np.array_equal(out, tbs[k]), msg


def test_pusch_harq_combining(decs):
    """Two transmissions of one TB through caller-owned device soft buffers:
    rv 0 too noisy, rv 2 combined; then a new_data transmission resets."""
    import torch

    import srsran_project_amd as amd

    tbs_bits, bg, qm, lay, nre = 8 * 1056, 1, 2, 1, 6000
    tb = tb_bytes(tbs_bits, 99)
    dec = decs["simd"]
    p0, op0 = _plan((tbs_bits, bg, qm, lay, nre, 0, 0))
    p2, op2 = _plan((tbs_bits, bg, qm, lay, nre, 2, 0))
    soft = torch.zeros(amd.soft_buffer_size(p0), dtype=torch.int8, device="cuda")
    h = osch.HarqBuffer(op0)
    out = np.zeros(tbs_bits // 8, np.uint8)
    d_tb = torch.zeros((1, tbs_bits // 8), dtype=torch.uint8, device="cuda")
    for p, op, new, sigma in ((p0, op0, True, 9), (p2, op2, False, 5)):
        llr = noisy_llrs(osch.pdsch_encode(tb, op), 8, sigma, seed=p.rv)
        ok, _, _ = osch.pusch_decode(llr, op, h, out, 6, "simd", new_data=new)
        cfg = amd.PuschDecoder.config(new_data=new)
        _, res = dec.decode_batch(torch.from_numpy(llr[None]).cuda(), p, cfg, tbs=d_tb, soft=soft)
        torch.cuda.synchronize()
        assert bool(res[0, 0].item()) == ok
        np.testing.assert_array_equal(d_tb[0].cpu().numpy(), out)
    assert ok and np.array_equal(out, tb)
    # Host form with a host soft buffer gives the same.
    hs = np.zeros(amd.soft_buffer_size(p0), np.int8)
    out2 = np.zeros(tbs_bits // 8, np.uint8)
    for p, op, new, sigma in ((p0, op0, True, 9), (p2, op2, False, 5)):
        llr = noisy_llrs(osch.pdsch_encode(tb, op), 8, sigma, seed=p.rv)
        r = dec.decode(llr, p, hs, out2, amd.PuschDecoder.config(new_data=new))
    assert r.tb_crc_ok == 1 and np.array_equal(out2, tb)


def test_pusch_harq_partial_retransmission(decs):
    """A retransmission after a partially decoded first transmission: codeblocks whose CRC passed are only
    rate dematched, not decoded again (pusch_decoder_impl.cpp:330-345); their statistic is the iteration
    count of the decoding that passed.  TB, CRC verdict, CB CRC count and LDPC statistics vs the oracle."""
    import torch

    import srsran_project_amd as amd

    tbs_bits, bg, qm, lay, nre = 8 * 4000, 1, 4, 1, 12000
    tb = tb_bytes(tbs_bits, 7)
    dec = decs["simd"]
    p0, op0 = _plan((tbs_bits, bg, qm, lay, nre, 0, 0))
    p2, op2 = _plan((tbs_bits, bg, qm, lay, nre, 2, 0))
    C = p0.nof_segments
    assert C >= 3
    E, off = amd.sch_segments(p0)
    soft = torch.zeros(amd.soft_buffer_size(p0), dtype=torch.int8, device="cuda")
    h = osch.HarqBuffer(op0)
    out = np.zeros(tbs_bits // 8, np.uint8)
    d_tb = torch.zeros((1, tbs_bits // 8), dtype=torch.uint8, device="cuda")
    cb_it = torch.zeros(C, dtype=torch.int32, device="cuda")
    for k, (p, op, new) in enumerate(((p0, op0, True), (p0, op0, False), (p2, op2, False))):
        llr = noisy_llrs(osch.pdsch_encode(tb, op), 8, 3, seed=10 + k)
        if k == 0:  # codeblock 1 lost in the first transmission
            llr[off[1]:off[1] + E[1]] = 0
        ok, iters, stats = osch.pusch_decode(llr, op, h, out, 6, "simd", new_data=new)
        _, res = dec.decode_batch(torch.from_numpy(llr[None]).cuda(), p, amd.PuschDecoder.config(new_data=new),
                                  tbs=d_tb, soft=soft, cb_iterations=cb_it)
        torch.cuda.synchronize()
        res = res.cpu().numpy()
        msg = "transmission %d" % k
        assert bool(res[0, 0]) == ok, msg
        assert res[0, 2] == sum(stats) and res[0, 3] == min(stats) and res[0, 4] == max(stats), (msg, res[0], stats)
        assert res[0, 5] == sum(h.crc), msg
        got = cb_it.cpu().numpy()
        for i in range(C):
            want = iters[i] if iters[i] is not None else (h.its[i] if h.crc[i] else -1)
            assert got[i] == want, (msg, i, got, iters)
        if k == 0:
            assert not ok and iters[1] is None and all(iters[i] is not None for i in range(C) if i != 1)
        np.testing.assert_array_equal(d_tb[0].cpu().numpy(), out, err_msg=msg)
    assert ok and np.array_equal(out, tb)


def test_pipeline_slot_roundtrip(enc, decs):
    """configs[3] transport block (273 PRB, 14 symbols with 2 DM-RS, 2 layers,
    256QAM MCS 27, R = 948/1024, TBS 590128): 8 TBs encoded and decoded back
    from clean LLRs on the device."""
    import torch

    import srsran_project_amd as amd

    tbs = amd.tbs_calculator_calculate(14, 24, 0, 8, 948, 2, 0, 273)
    assert tbs == 590128
    p = amd.sch_plan(tbs, 1, 0, 8, 0, 2, 273 * 144 * 2)
    rows = torch.from_numpy(np.stack([tb_bytes(p.tbs, k) for k in range(8)])).cuda()
    cw = enc.encode_batch(rows, p)
    bits = torch.from_numpy(np.unpackbits(cw.cpu().numpy(), axis=1)[:, :p.cw_length].astype(np.int8)).cuda()
    llrs = (1 - 2 * bits) * 40
    d_tb, res = decs["simd"].decode_batch(llrs.contiguous(), p, amd.PuschDecoder.config())
    torch.cuda.synchronize()
    assert res[:, 0].all().item()
    assert torch.equal(d_tb, rows)


# High-rate BG1 Z = 384 transport blocks whose new-data rows the high-rate decoder builds from the codeword itself
# (rate dematching fused into its load, decode_args::cw_llrs): fillers of 56..416 bits, Qm 2..8, 1..4 layers,
# short and long segments, the headline 4-layer 256QAM TB.  (tbs, Qm, layers, channel symbols)
FUSED_DEMATCH_CASES = [
    (160136, 2, 1, 87093),
    (40024, 4, 1, 10887),
    (72808, 6, 1, 13064),
    (72808, 6, 2, 13064),
    (160136, 8, 4, 21776),
    (1179864, 8, 4, 156744),
]


@pytest.mark.parametrize("ci", range(len(FUSED_DEMATCH_CASES)))
def test_pusch_decode_dematch_fused(decs, ci, monkeypatch):
    """decode_batch with internal soft rows (new data, rv 0, no circular wrap, prefix 24 Z): the fused
    dematch-in-decoder path against the oracle (pusch_decoder_impl restatement) and against the separate dematch
    launch (SRSRAN_AMD_DEMATCH_FUSED=0): TBs, CRC verdicts, statistics and per-codeblock iterations bit-exact."""
    import torch

    import srsran_project_amd as amd

    tbs, qm, lay, nre = FUSED_DEMATCH_CASES[ci]
    p, op = _plan((tbs, 1, qm, lay, nre, 0, 0))
    assert p.lifting_size == 384 and amd.decoder_llr_prefix(p, True, True) == 24 * 384
    n = 2 if tbs > 500000 else 3
    tb = [tb_bytes(p.tbs, 31 * ci + k) for k in range(n)]
    # easy, near-threshold, undecodable
    llrs = np.stack([noisy_llrs(osch.pdsch_encode(tb[k], op), 12, (2, 5, 12)[k], seed=ci * 10 + k) for k in range(n)])
    C = p.nof_segments
    cfg = amd.PuschDecoder.config(nof_ldpc_iterations=6)
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SRSRAN_AMD_DEMATCH_FUSED", mode)
        cb_it = torch.zeros(n * C, dtype=torch.int32, device="cuda")
        d_tb, res = decs["simd"].decode_batch(torch.from_numpy(llrs).cuda(), p, cfg, cb_iterations=cb_it)
        torch.cuda.synchronize()
        outs[mode] = (d_tb.cpu().numpy(), res.cpu().numpy(), cb_it.cpu().numpy().reshape(n, C))
    for a, b in zip(outs["1"], outs["0"]):
        np.testing.assert_array_equal(a, b)
    d_tb, res, cb_it = outs["1"]
    for k in range(n):
        h = osch.HarqBuffer(op)
        out = np.zeros(p.tbs // 8, np.uint8)
        ok, iters, stats = osch.pusch_decode(llrs[k], op, h, out, 6, "simd")
        msg = "case %d TB %d" % (ci, k)
        assert bool(res[k, 0]) == ok, msg
        assert (res[k, 2], res[k, 3], res[k, 4]) == (sum(stats), min(stats), max(stats)), msg
        np.testing.assert_array_equal(cb_it[k], [-1 if i is None else i for i in iters], err_msg=msg)
        np.testing.assert_array_equal(d_tb[k], out, err_msg=msg)
    assert bool(res[0, 0]) and np.array_equal(d_tb[0], tb[0])

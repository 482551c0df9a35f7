"""GPU parity: MI355X LDPC decoder (through the C-ABI) vs the CPU oracle.

Bar: bit-exact -- decoded bits, iteration counts / CRC verdicts and the final
int8 soft bits must equal oracle/srs_oracle.c, which is itself pinned to the
reference's decoders (tests/test_oracle_vs_ref.py).  Cases follow the
reference's tests/unittests/phy/upper/channel_coding/ldpc/ldpc_enc_dec_test.cpp
(all base graphs / lifting-size families, shortened lengths 24Z..66Z in 3 steps,
zero and almost-zero LLR codeblocks) plus CRC early stop, filler bits,
force_decoding, ragged batches and large batches.
"""
import numpy as np
import pytest

import oracle
from tests.ldpc_cases import noisy_codeblocks

pytestmark = pytest.mark.gpu

# every kernel class: Z not a multiple of 4 (one row per lane), the packed runtime-Z kernel with 1, 2 and 3 waves
# per codeblock (Z <= 128, <= 256, > 256), BG1 Z = 384 (compile-time kernels)
ZS = [2, 3, 4, 5, 7, 9, 11, 12, 13, 15, 16, 36, 44, 64, 104, 128, 144, 208, 240, 256, 288, 352, 384]


@pytest.fixture(scope="module")
def amd():
    import srsran_project_amd as amd

    return amd


@pytest.fixture(autouse=True, params=["auto", "full", "nopk"])
def full_length_kernel(request, monkeypatch):
    """Every case three times: the launch's own kernel choice (small batches of full-length BG1 Z=384 codeblocks go
    to ldpc_decode_kernel, other graphs with Z a multiple of 4 to the packed runtime-Z kernel),
    SRSRAN_AMD_LDPC_FULL=1, which sends every BG1 Z=384 launch the high-rate kernel does not take through the packed
    full-length kernel whatever the batch size, and SRSRAN_AMD_LDPC_PK=0, which keeps every other graph on the
    one-row-per-lane ldpc_decode_kernel."""
    monkeypatch.delenv("SRSRAN_AMD_LDPC_FULL", raising=False)
    monkeypatch.delenv("SRSRAN_AMD_LDPC_PK", raising=False)
    if request.param == "full":
        monkeypatch.setenv("SRSRAN_AMD_LDPC_FULL", "1")
    elif request.param == "nopk":
        monkeypatch.setenv("SRSRAN_AMD_LDPC_PK", "0")
    return request.param


def _gpu_decode(amd, dec, llrs, bg, Z, iters, crc=None, filler=0, lens=None, want_soft=False):
    import torch

    cfg = amd.LdpcDecoderConfiguration(base_graph=bg, lifting_size=Z, nof_filler_bits=filler,
                                       nof_crc_bits=24 if crc in (0, 1, 2) else 16, max_iterations=iters)
    d_llrs = torch.from_numpy(np.ascontiguousarray(llrs)).cuda()
    d_lens = None if lens is None else torch.from_numpy(np.asarray(lens, np.int32)).cuda()
    soft = None
    if want_soft:
        soft = torch.zeros((llrs.shape[0], oracle.BG_N_FULL[bg] * Z), dtype=torch.int8, device="cuda")
    out, it = dec.decode_batch(d_llrs, cfg, crc, llr_lens=d_lens, soft_out=soft)
    torch.cuda.synchronize()
    return out.cpu().numpy(), it.cpu().numpy(), (soft.cpu().numpy() if want_soft else None)


def _check(amd, dec, arith, llrs, bg, Z, iters, crc=None, filler=0, lens=None):
    out, it, soft = _gpu_decode(amd, dec, llrs, bg, Z, iters, crc, filler, lens, want_soft=True)
    for i in range(llrs.shape[0]):
        L = llrs.shape[1] if lens is None else lens[i]
        r, o, s = oracle.ldpc_decode(llrs[i, :L], bg, Z, iters, arith, crc, filler,
                                     24 if crc in (0, 1, 2) else 16, want_soft=True)
        assert (-1 if r is None else r) == it[i], (bg, Z, i, r, it[i])
        np.testing.assert_array_equal(out[i], o, err_msg="bits bg%d Z%d cb%d" % (bg, Z, i))
        np.testing.assert_array_equal(soft[i], s, err_msg="soft bg%d Z%d cb%d" % (bg, Z, i))


@pytest.mark.parametrize("arith", ["simd", "generic"])
@pytest.mark.parametrize("bg", [1, 2])
def test_parity_all_families(amd, bg, arith):
    dec = amd.LdpcDecoder(arith)
    for Z in ZS:
        msgs, llrs = noisy_codeblocks(bg, Z, 3, seed=Z * 7 + bg)
        _check(amd, dec, arith, llrs, bg, Z, iters=6)


@pytest.mark.parametrize("bg", [1, 2])
def test_parity_shortened_lengths(amd, bg):
    # ldpc_enc_dec_test.cpp: create_range(min_cb_length, max_cb_length, 3).
    dec = amd.LdpcDecoder("simd")
    for Z in (5, 52, 160, 320, 384):
        lo = (24 if bg == 1 else 12) * Z
        hi = oracle.BG_N_SHORT[bg] * Z
        step = (hi - lo) // 3
        for L in list(range(lo, hi, step)) + [hi]:
            msgs, llrs = noisy_codeblocks(bg, Z, 2, length=L, seed=L)
            _check(amd, dec, "simd", llrs, bg, Z, iters=8)


def test_noiseless_one_iteration_recovers_message(amd):
    # ldpc_enc_dec_test.cpp LDPCDecTest: fixed amplitude 10, one iteration.
    dec = amd.LdpcDecoder("simd")
    for bg in (1, 2):
        for Z in (2, 13, 384):
            msgs, llrs = noisy_codeblocks(bg, Z, 4, snr_amp=10, noise=0.0, seed=Z)
            out, it, _ = _gpu_decode(amd, dec, llrs, bg, Z, 1)
            K = oracle.BG_K[bg] * Z
            for i in range(4):
                np.testing.assert_array_equal(oracle.unpack_bits(out[i], K), msgs[i])


def test_zero_and_almost_zero_llrs(amd):
    # LDPCDecTestZeroLLR / LDPCDecTestAlmostZeroLLR: message of all ones, no value.
    dec = amd.LdpcDecoder("simd")
    for bg in (1, 2):
        Z = 16
        K = oracle.BG_K[bg] * Z
        N = oracle.BG_N_SHORT[bg] * Z
        zero = np.zeros((1, N), np.int8)
        almost = np.zeros((1, N), np.int8)
        lo = (24 if bg == 1 else 12) * Z
        for b in range(lo + 2, N, 3):
            almost[0, b] = 1 if b % 2 == 0 else -1
        for llrs in (zero, almost):
            out, it, _ = _gpu_decode(amd, dec, llrs, bg, Z, 1)
            assert it[0] == -1
            assert (oracle.unpack_bits(out[0], K) == 1).all()
            _check(amd, dec, "simd", llrs, bg, Z, 1)


@pytest.mark.parametrize("crc", [3, 1, 0])
def test_crc_early_stop(amd, crc):
    dec = amd.LdpcDecoder("simd")
    bg, Z = (1, 384) if crc != 3 else (2, 16)
    msgs, llrs = noisy_codeblocks(bg, Z, 8, noise=9.0, seed=crc + 11, crc_poly=crc)
    # make two codeblocks undecodable
    rng = np.random.default_rng(5)
    llrs[3] = rng.integers(-3, 4, llrs.shape[1]).astype(np.int8)
    _check(amd, dec, "simd", llrs, bg, Z, iters=10, crc=crc)
    _, it, _ = _gpu_decode(amd, dec, llrs, bg, Z, 10, crc)
    assert it[3] == -1 and (it[[0, 1, 2, 4, 5, 6, 7]] >= 1).all()


def test_filler_bits(amd):
    dec = amd.LdpcDecoder("simd")
    bg, Z, F = 1, 104, 200
    msgs, llrs = noisy_codeblocks(bg, Z, 4, seed=3)
    _check(amd, dec, "simd", llrs, bg, Z, iters=5, crc=0, filler=F)


def test_force_decoding_short_input(amd):
    dec = amd.LdpcDecoder("simd", force_decoding=True)
    bg, Z = 1, 32
    K = 22 * Z
    N = 66 * Z
    llrs = np.zeros((2, N), np.int8)
    llrs[0, : K // 2] = 5  # input_size < K
    llrs[1, : K + 3 * Z] = -7
    out, it, _ = _gpu_decode(amd, dec, llrs, bg, Z, 3)
    assert it[0] == -1 and (oracle.unpack_bits(out[0], K) == 1).all()
    r, o, _ = oracle.ldpc_decode(llrs[1], bg, Z, 3, force_decoding=True)
    np.testing.assert_array_equal(out[1], o)


def test_ragged_batch_and_tail(amd):
    # Per-codeblock lengths, including lengths that are not a multiple of Z
    # (ldpc_decoder_impl.cpp:204 tail handling).
    dec = amd.LdpcDecoder("simd")
    bg, Z = 2, 26
    N = oracle.BG_N_SHORT[bg] * Z
    msgs, llrs = noisy_codeblocks(bg, Z, 6, seed=9)
    lens = [N, 12 * Z, 12 * Z + 5, 30 * Z + 1, N - 3, 20 * Z]
    _check(amd, dec, "simd", llrs, bg, Z, iters=4, lens=lens)


def test_large_batch_grid_stride(amd):
    dec = amd.LdpcDecoder("simd")
    dec.set_max_slots(64)  # force the persistent grid-stride loop
    bg, Z = 1, 384
    msgs, llrs = noisy_codeblocks(bg, Z, 16, seed=77)
    big = np.concatenate([llrs] * 20)  # 320 codeblocks over 64 workgroups
    out, it, _ = _gpu_decode(amd, dec, big, bg, Z, 8)
    ref = [oracle.ldpc_decode(llrs[i], bg, Z, 8)[1] for i in range(16)]
    for i in range(big.shape[0]):
        np.testing.assert_array_equal(out[i], ref[i % 16])


def test_host_single_call_matches_reference_shape(amd):
    dec = amd.create_ldpc_decoder_factory_hip("auto").create()
    bg, Z = 1, 208
    msgs, llrs = noisy_codeblocks(bg, Z, 2, seed=1, crc_poly=1)
    cfg = amd.LdpcDecoderConfiguration(base_graph=bg, lifting_size=Z, nof_crc_bits=24, max_iterations=8)
    for i in range(2):
        out = np.zeros((22 * Z + 7) // 8, np.uint8)
        r = dec.decode(out, llrs[i], amd.CrcGeneratorPoly.CRC24B, cfg)
        r2, o2, _ = oracle.ldpc_decode(llrs[i], bg, Z, 8, crc_poly=1, nof_crc_bits=24)
        assert r == r2
        np.testing.assert_array_equal(out, o2)


def test_invalid_configuration_raises(amd):
    dec = amd.LdpcDecoder("simd")
    out = np.zeros(100, np.uint8)
    with pytest.raises(ValueError):
        dec.decode(out, np.zeros(100, np.int8), None, amd.LdpcDecoderConfiguration(lifting_size=17))
    with pytest.raises(ValueError):
        dec.decode(np.zeros((22 * 4 + 7) // 8, np.uint8), np.zeros(50, np.int8), None,
                   amd.LdpcDecoderConfiguration(lifting_size=4))  # input shorter than K + 2Z
    with pytest.raises(ValueError):
        dec.decode(np.zeros((22 * 4 + 7) // 8, np.uint8), np.zeros(200, np.int8), None,
                   amd.LdpcDecoderConfiguration(lifting_size=4, max_iterations=0))


# ---- high-rate BG1 / Z = 384 kernel (ldpc_decode_hr_kernel): rows of at most 24 Z LLRs, so at most
# four layers; selected by the launch for those rows (ldpc_decoder.hip, ldpc_decode_hr_eligible).
HR_LEN = 24 * 384


def _high_rate_rows(n, seed, noise, crc=None, zero_from=None, filler=0):
    msgs, llrs = noisy_codeblocks(1, 384, n, length=HR_LEN, noise=noise, seed=seed, crc_poly=crc)
    if filler:
        llrs[:, 20 * 384 - filler:20 * 384] = 127  # the rate dematcher's +inf filler LLRs
    if zero_from is not None:
        for i, z in enumerate(zero_from):
            llrs[i, z:] = 0
    return msgs, llrs


@pytest.mark.parametrize("arith", ["simd", "generic"])
def test_high_rate_kernel_parity(amd, arith):
    dec = amd.LdpcDecoder(arith)
    # near threshold (several iterations, some failures), moderate, noiseless-ish
    for seed, noise, crc in ((1, 11.0, 1), (2, 7.0, 1), (3, 2.0, 1), (4, 9.0, None), (5, 10.0, 0)):
        _, llrs = _high_rate_rows(12, seed, noise, crc)
        _check(amd, dec, arith, llrs, 1, 384, iters=6, crc=crc)


def test_high_rate_kernel_fillers_and_trimming(amd):
    dec = amd.LdpcDecoder("simd")
    _, llrs = _high_rate_rows(6, 21, 8.0, crc=1, filler=136)
    _check(amd, dec, "simd", llrs, 1, 384, iters=5, crc=1, filler=136)
    # trailing zeros: the decoder trims at the last non-zero LLR (23 Z + 5, 22 Z + 2 Z - 1, ...)
    _, llrs = _high_rate_rows(4, 22, 6.0, crc=1, zero_from=[23 * 384 + 5, 24 * 384 - 1, 22 * 384, 21 * 384 + 7])
    _check(amd, dec, "simd", llrs, 1, 384, iters=4, crc=1)
    # infinite soft bits anywhere in the row (saturated LLRs)
    _, llrs = _high_rate_rows(4, 23, 30.0)
    llrs[:, ::97] = np.where(llrs[:, ::97] >= 0, 127, -127)
    _check(amd, dec, "simd", llrs, 1, 384, iters=3)


def test_high_rate_kernel_force_decoding(amd):
    dec = amd.LdpcDecoder("simd", force_decoding=True)
    llrs = np.zeros((3, HR_LEN), np.int8)
    llrs[0, :100] = 5  # input_size < K: no value, all ones
    llrs[1, : 22 * 384 + 3] = -9
    llrs[2] = _high_rate_rows(1, 31, 6.0)[1][0]
    out, it, _ = _gpu_decode(amd, dec, llrs, 1, 384, 3)
    assert it[0] == -1 and (oracle.unpack_bits(out[0], 22 * 384) == 1).all()
    for i in (1, 2):
        r, o, _ = oracle.ldpc_decode(llrs[i], 1, 384, 3, force_decoding=True)
        np.testing.assert_array_equal(out[i], o)
        assert (-1 if r is None else r) == it[i]


def test_high_rate_kernel_grid_stride_and_offsets(amd):
    import torch

    dec = amd.LdpcDecoder("simd")
    dec.set_max_slots(48)
    _, llrs = _high_rate_rows(16, 41, 9.0, crc=1)
    big = np.concatenate([llrs] * 10)
    # rows with a stride larger than the length (PUSCH soft-buffer rows) and an odd output stride
    rows = np.zeros((big.shape[0], 26112), np.int8)
    rows[:, :HR_LEN] = big
    d = torch.from_numpy(rows).cuda()[:, :HR_LEN]
    cfg = amd.LdpcDecoderConfiguration(base_graph=1, lifting_size=384, nof_crc_bits=24, max_iterations=6)
    out = torch.zeros((big.shape[0], 1061), dtype=torch.uint8, device="cuda")
    out, it = dec.decode_batch(d, cfg, amd.CrcGeneratorPoly.CRC24B, out=out[:, 1:1057])
    torch.cuda.synchronize()
    out, it = out.cpu().numpy(), it.cpu().numpy()
    for i in range(16):
        r, o, _ = oracle.ldpc_decode(llrs[i], 1, 384, 6, crc_poly=1, nof_crc_bits=24)
        for k in range(10):
            np.testing.assert_array_equal(out[16 * k + i], o)
            assert it[16 * k + i] == (-1 if r is None else r)


@pytest.mark.parametrize("bg", [1, 2])
def test_packed_kernel_repeating_lanes(amd, bg):
    """Lifting sizes whose half Z / 2 is not a multiple of 64 with two or three waves per codeblock: the lanes past
    Z / 2 repeat a row pair of another wave and must not scatter (a repeating wave that gathered after the owner's
    scatter wrote different soft bits, intermittently).  48 noisy codeblocks per size, soft bits included."""
    dec = amd.LdpcDecoder("simd")
    for Z in (144, 160, 176, 208, 224, 240, 288, 320, 352):
        msgs, llrs = noisy_codeblocks(bg, Z, 48, seed=Z * 13 + bg)
        _check(amd, dec, "simd", llrs, bg, Z, iters=6)

"""Golden vectors produced by the reference decoders/encoder themselves
(tests/golden/make_golden.py): the oracle must reproduce them on the CPU; the
GPU decoder must reproduce them through the C-ABI (gpu marker)."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ldpc_golden.npz")


def cases():
    z = np.load(GOLDEN)
    keys = sorted({k.split("_")[0] for k in z.files})
    for k in keys:
        bg, Z, iters, crc, filler, generic = z[k + "_cfg"].tolist()
        yield k, dict(bg=bg, Z=Z, iters=iters, crc=None if crc < 0 else crc, filler=filler,
                      arith="generic" if generic else "simd", msg=z[k + "_msg"], cw=z[k + "_cw"],
                      llr=z[k + "_llr"], out=z[k + "_out"], it=int(z[k + "_iters"][0]))


def test_oracle_encoder_reproduces_golden():
    for k, c in cases():
        K = oracle.BG_K[c["bg"]] * c["Z"]
        N = oracle.BG_N_SHORT[c["bg"]] * c["Z"]
        m = oracle.unpack_bits(c["msg"], K)
        np.testing.assert_array_equal(oracle.ldpc_encode(m, c["bg"], c["Z"]), oracle.unpack_bits(c["cw"], N), err_msg=k)


def test_oracle_decoder_reproduces_golden():
    for k, c in cases():
        nb = 24 if c["crc"] in (0, 1, 2) else 16
        r, out, _ = oracle.ldpc_decode(c["llr"], c["bg"], c["Z"], c["iters"], c["arith"], c["crc"], c["filler"], nb)
        assert (-1 if r is None else r) == c["it"], k
        np.testing.assert_array_equal(out, c["out"], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("full", ["auto", "1", "nopk"])
def test_gpu_decoder_reproduces_golden(full, monkeypatch):
    # "1": BG1 Z=384 vectors (configs[1]) through the packed full-length kernel whatever the batch size;
    # "nopk": every other graph on the one-row-per-lane kernel instead of the packed runtime-Z kernel
    monkeypatch.delenv("SRSRAN_AMD_LDPC_FULL", raising=False)
    monkeypatch.delenv("SRSRAN_AMD_LDPC_PK", raising=False)
    if full == "1":
        monkeypatch.setenv("SRSRAN_AMD_LDPC_FULL", "1")
    elif full == "nopk":
        monkeypatch.setenv("SRSRAN_AMD_LDPC_PK", "0")
    import torch

    import srsran_project_amd as amd

    decs = {"simd": amd.LdpcDecoder("simd"), "generic": amd.LdpcDecoder("generic")}
    for k, c in cases():
        nb = 24 if c["crc"] in (0, 1, 2) else 16
        cfg = amd.LdpcDecoderConfiguration(base_graph=c["bg"], lifting_size=c["Z"], nof_filler_bits=c["filler"],
                                           nof_crc_bits=nb, max_iterations=c["iters"])
        llr = torch.from_numpy(c["llr"][None, :].copy()).cuda()
        out, it = decs[c["arith"]].decode_batch(llr, cfg, c["crc"])
        torch.cuda.synchronize()
        assert int(it.cpu()[0]) == c["it"], k
        np.testing.assert_array_equal(out.cpu().numpy()[0], c["out"], err_msg=k)

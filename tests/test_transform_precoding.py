"""Transform deprecoding (DFT-s-OFDM PUSCH, transform_precoder_dft_impl.cpp:31-84).

CPU: the numpy restatement (oracle/transform_precoding.py) against the reference's own
transform_precoder_dft_impl compiled into oracle/_ref, and the C-ABI's PRB validity rule.
GPU: the MI355X deprecoder (srs_amd_transform_deprecode*, through the C-ABI) against the float64
restatement and the reference, every valid PRB count.  Tolerance (float DFT, as the reference's
generic float DFT): |gpu - exact| <= 2e-6 * sqrt(M) * RMS(input) per output; noise means within 2e-5
relative, invalid variances passed through unchanged."""
import numpy as np
import pytest

import oracle.transform_precoding as otp

VALID = [m for m in range(1, 276) if otp.nof_prbs_valid(m)]


def _symbol(M, seed):
    rng = np.random.default_rng(seed)
    return ((rng.normal(size=M) + 1j * rng.normal(size=M)) * 0.7).astype(np.complex64)


def _noise(M, seed):
    rng = np.random.default_rng(seed)
    nv = rng.uniform(0.01, 2.0, M).astype(np.float32)
    nv[rng.integers(0, M, 3)] = 0.0
    nv[rng.integers(0, M, 2)] = np.inf
    nv[rng.integers(0, M, 1)] = -0.5
    nv[rng.integers(0, M, 1)] = np.nan
    return nv


@pytest.mark.skipif(otp.REF is None, reason="oracle/_ref not built")
@pytest.mark.parametrize("m", [1, 2, 3, 5, 8, 12, 25, 45, 75, 96, 135, 180, 240, 270])
def test_oracle_matches_reference(m):
    M = 12 * m
    y = _symbol(M, m)
    ref = otp.ref_deprecode(y)
    np.testing.assert_allclose(ref, otp.deprecode(y), atol=2e-6 * np.sqrt(M) * np.sqrt(np.mean(np.abs(y) ** 2)))
    nv = _noise(M, m)
    np.testing.assert_allclose(otp.ref_deprecode_noise(nv), otp.deprecode_noise(nv), rtol=2e-5)


@pytest.mark.skipif(otp.REF is None, reason="oracle/_ref not built")
def test_prb_validity_matches_reference():
    import srsran_project_amd as amd

    for n in range(0, 300):
        assert amd.transform_precoding_nof_prbs_valid(n) == otp.ref_nof_prbs_valid(n) == otp.nof_prbs_valid(n), n


@pytest.mark.gpu
def test_gpu_deprecode_every_valid_size():
    import torch

    import srsran_project_amd as amd

    tp = amd.TransformPrecoder()
    for m in VALID:
        M = 12 * m
        rows = 3
        ys = np.stack([_symbol(M, 1000 * m + r) for r in range(rows)])
        nvs = np.stack([_noise(M, 2000 * m + r) for r in range(rows)])
        # padded rows (stride > M)
        d_y = torch.zeros((rows, M + 8), dtype=torch.complex64, device="cuda")
        d_y[:, :M] = torch.from_numpy(ys).cuda()
        d_nv = torch.zeros((rows, M + 4), dtype=torch.float32, device="cuda")
        d_nv[:, :M] = torch.from_numpy(nvs).cuda()
        tp.deprecode_batch(d_y, d_nv, nof_subc=M)
        torch.cuda.synchronize()
        got, gnv = d_y.cpu().numpy(), d_nv.cpu().numpy()
        for r in range(rows):
            exact = otp.deprecode(ys[r])
            tol = 2e-6 * np.sqrt(M) * np.sqrt(np.mean(np.abs(ys[r]) ** 2))
            assert np.abs(got[r, :M] - exact).max() <= tol, (m, r, np.abs(got[r, :M] - exact).max(), tol)
            assert (got[r, M:] == 0).all(), "padding written"
            np.testing.assert_allclose(gnv[r, :M], otp.deprecode_noise(nvs[r]), rtol=2e-5, err_msg="M_rb %d" % m)
        if m in (1, 45, 270) and otp.REF is not None:
            ref = otp.ref_deprecode(ys[0])
            assert np.abs(got[0, :M] - ref).max() <= 2 * tol


@pytest.mark.gpu
def test_gpu_host_forms_and_errors():
    import srsran_project_amd as amd

    tp = amd.TransformPrecoder()
    y = _symbol(12 * 20, 5)
    np.testing.assert_allclose(tp.deprecode_ofdm_symbol(y), otp.deprecode(y), atol=2e-5)
    nv = _noise(12 * 20, 6)
    np.testing.assert_allclose(tp.deprecode_ofdm_symbol_noise(nv), otp.deprecode_noise(nv), rtol=2e-5)
    for bad in (12 * 7, 12 * 11, 13, 0, 12 * 280):
        with pytest.raises(ValueError):
            tp.deprecode_ofdm_symbol(np.zeros(bad, np.complex64))

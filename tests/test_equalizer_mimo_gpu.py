"""GPU tests of the L-layer equalizers the open reference does not implement -- ZF 3x4 / 4x4 and MMSE
2x2 / 2x4 / 3x4 / 4x4 (channel_equalizer_generic_impl.cpp:197-247 asserts for them): PARITY UNPINNED.
Checked against the fp64 solve of the same model (oracle/equalizer.py equalize_mimo), which itself reduces to the
pinned ZF equalizers where they overlap (test_oracle_properties.py).

Tolerance (the contract): per RE, |gpu_l - exact_l| <= r * ||exact_RE|| + 1e-6 on the symbols and
|gpu - exact| <= 2 r * exact on the noise variances, r = 1e-4 + 4e-6 * kappa, kappa the condition number of the
float32 solve (Gram matrix for ZF; A = ts^2 H^H H + sigma^2 I scaled by 1 / min(mu) for the unbiased MMSE) -- the
float32 Cholesky + substitution error bound (~n u kappa, u = 6e-8) with a margin of 16.
Abnormal inputs (zero / NaN / infinite channel, invalid noise variance) give exactly zero symbols and infinite
variances."""
import numpy as np
import pytest

from oracle import equalizer as E
from oracle.ofdm import float_to_bf16

pytestmark = pytest.mark.gpu

MIMO = [(4, 3, "zf"), (4, 4, "zf"), (2, 2, "mmse"), (4, 2, "mmse"), (4, 3, "mmse"), (4, 4, "mmse")]


@pytest.fixture(scope="module")
def amd():
    import srsran_project_amd as amd

    return amd


def _eq(amd, algo):
    return amd.ChannelEqualizer(getattr(amd.ChannelEqualizerAlgorithmType, algo))


def _close(got, gotn, want, wantn, kappa):
    r = 1e-4 + 4e-6 * kappa[:, None]
    scale = np.linalg.norm(want, axis=1)[:, None]
    err = np.abs(got - want)
    bad = err > r * scale + 1e-6
    assert not bad.any(), (np.argwhere(bad)[:5], got[bad][:5], want[bad][:5], kappa[np.any(bad, axis=1)][:5])
    fin = np.isfinite(wantn)
    assert np.array_equal(np.isfinite(gotn), fin)
    rv = np.broadcast_to(2 * r, wantn.shape)
    assert np.all(np.abs(gotn[fin] - wantn[fin]) <= rv[fin] * wantn[fin])


@pytest.mark.parametrize("ports,layers,algo", MIMO)
def test_mimo_equalizer_random_channels(amd, ports, layers, algo):
    rng = np.random.default_rng(ports * 100 + layers * 10 + len(algo))
    eq = _eq(amd, algo)
    assert eq.is_supported(ports, layers) and E.is_supported_mimo(algo, ports, layers)
    assert not E.is_supported(algo, ports, layers)  # the open reference asserts for this topology
    for nre, tx, snr in ((1, 1.0, 20.0), (257, 0.5, 5.0), (3276 * 14, 1.0, 30.0), (4096, 0.8, 15.0)):
        s, h, nv, _ = E.random_channel(rng, nre, ports, layers, snr)
        got, gotn = eq.equalize(s, h, nv, tx)
        want, wantn, kap = E.equalize_mimo(s, h, nv, tx, layers, algo)
        _close(got, gotn, want, wantn, kap)


@pytest.mark.parametrize("ports,layers,algo", MIMO)
def test_mimo_equalizer_recovers_symbols(amd, ports, layers, algo):
    """High SNR, well-conditioned channels: the equalized symbols are the transmitted QPSK points."""
    rng = np.random.default_rng(5)
    s, h, nv, x = E.random_channel(rng, 2048, ports, layers, 40.0)
    got, gotn = _eq(amd, algo).equalize(s, h, nv, 1.0)
    _, _, kap = E.equalize_mimo(s, h, nv, 1.0, layers, algo)
    ok = kap < 1000
    assert ok.mean() > 0.5
    # within 6 standard deviations of the post-equalization noise the equalizer itself reports
    assert np.all(np.abs(got[ok] - x[ok]) < 6 * np.sqrt(gotn[ok]) + 0.02)
    assert np.median(gotn[ok]) < 0.01


@pytest.mark.parametrize("ports,layers,algo", MIMO)
def test_mimo_equalizer_abnormal_inputs(amd, ports, layers, algo):
    rng = np.random.default_rng(99)
    eq = _eq(amd, algo)
    s, h, nv, _ = E.random_channel(rng, 64, ports, layers)
    h = h.copy()
    # RE 0: zero channel on every path; RE 1: NaN on the first path; RE 2: infinity; RE 3: two equal layers
    h[:, :, 0:2] = 0
    h[0, 0, 2:4] = float_to_bf16(np.array([np.nan, 0.0], np.float32))
    h[0, 0, 4:6] = float_to_bf16(np.array([np.inf, 1.0], np.float32))
    h[1, :, 6:8] = h[0, :, 6:8]
    got, gotn = eq.equalize(s, h, nv, 1.0)
    want, wantn, kap = E.equalize_mimo(s, h, nv, 1.0, layers, algo)
    for re in (0, 1, 2):
        assert got[re].tolist() == [0] * layers and np.all(np.isinf(gotn[re])), re
    if algo == "zf":  # singular Gram matrix: no ZF solution
        assert got[3].tolist() == [0] * layers and np.all(np.isinf(gotn[3]))
    sel = np.arange(64) >= (3 if algo == "mmse" else 4)
    _close(got[sel], gotn[sel], want[sel], wantn[sel], kap[sel])
    for bad in ([0.0] * ports, [np.inf] + [0.02] * (ports - 1), [np.nan] * ports):
        got, gotn = eq.equalize(s, h, np.array(bad, np.float32), 1.0)
        assert np.all(got == 0) and np.all(np.isinf(gotn))


def test_mimo_equalizer_batch_device(amd):
    import torch

    rng = np.random.default_rng(1)
    eq = _eq(amd, "mmse")
    s, h, nv, _ = E.random_channel(rng, 3276 * 12, 4, 4, 25.0)
    ds = torch.from_numpy(s.view(np.int16)).cuda()
    dh = torch.from_numpy(h.view(np.int16)).cuda()
    got, gotn = eq.equalize_batch(ds, dh, nv, 0.8)
    torch.cuda.synchronize()
    want, wantn, kap = E.equalize_mimo(s, h, nv, 0.8, 4, "mmse")
    _close(got.cpu().numpy(), gotn.cpu().numpy(), want, wantn, kap)

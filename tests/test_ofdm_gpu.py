"""GPU parity: MI355X OFDM modulator / demodulator and DFT processor (through
the C-ABI) vs the CPU oracle oracle/ofdm.py, itself pinned to the reference's
ofdm_modulator_impl / ofdm_demodulator_impl / dft_processor_generic_impl
(tests/test_oracle_vs_ref.py).

Tolerances (float path, stated here as the contract):
  * time-domain samples and DFT outputs: max |gpu - exact| <= 2e-5 x RMS(exact)
    (the reference's own float DFT sits at ~1.5e-6 x RMS);
  * resource grids (cbf16): every value equal to the exactly computed value
    rounded half-to-even, except values within float error of a bf16 rounding
    tie, which may differ by one bf16 ulp (< 0.1 % of values).
Cases: the configurations of the reference's ofdm_modulator_test_data.h /
ofdm_demodulator_test_data.h (numerology 0-3, 256-4096 points, normal and
extended CP), the 100 MHz numerology-1 4096-point 273-PRB case, 1536/3072/6144
points, window offsets, multi-port multi-slot batches.
"""
import numpy as np
import pytest

from oracle import ofdm as ref

pytestmark = pytest.mark.gpu

CASES = [
    (0, 12, 256, False, 0.81158, 2740100000), (0, 24, 512, False, 0.67645, 2196700000),
    (0, 48, 1024, False, 0.356, 1552000000), (0, 96, 2048, False, 0.93184, 97900000),
    (0, 192, 4096, False, 0.87523, 1424700000), (1, 12, 256, False, -0.77438, 2686500000),
    (1, 96, 2048, False, 0.17815, 1462800000), (1, 192, 4096, False, -0.54681, 619800000),
    (2, 12, 256, True, 0.73538, 837900000), (2, 48, 1024, True, -0.12453, 383700000),
    (2, 192, 4096, True, -0.82195, 605900000), (3, 48, 1024, False, -0.64012, 622100000),
    (3, 192, 4096, False, 0.73052, 2633100000), (1, 273, 4096, False, 1.0, 3500000000),
    (1, 106, 1536, False, 0.5, 1800000000), (1, 217, 3072, False, 0.25, 2100000000),
    (1, 273, 6144, False, 0.7, 3300000000), (0, 24, 384, False, 1.3, 900000000),
    (1, 51, 768, False, 0.9, 1900000000), (2, 10, 128, False, 0.4, 700000000),
    (3, 264, 8192, False, 0.6, 28000000000),
]


@pytest.fixture(scope="module")
def amd():
    import srsran_project_amd as amd

    return amd


def _rms(x):
    return float(np.sqrt(np.mean(np.abs(x) ** 2)))


def _check_grid(got, rx, slot, mu, bw, N, scale, fc, off, ext):
    want = ref.demodulate_slot(rx, slot, mu, bw, N, scale, fc, off, ext)
    diff = np.abs(got.astype(np.int32) - want.astype(np.int32))
    assert diff.max() <= 1 and np.mean(diff != 0) < 1e-3, (N, mu, off, diff.max(), np.mean(diff != 0))


@pytest.mark.parametrize("case", CASES)
def test_modulate_demodulate_slot(amd, case):
    mu, bw, N, ext, scale, fc = case
    rng = np.random.default_rng(N + 7 * bw + mu)
    ns = 12 if ext else 14
    mcfg = amd.OfdmModulatorConfiguration(numerology=mu, bw_rb=bw, dft_size=N, cp=int(ext), scale=scale,
                                          center_freq_Hz=fc)
    mod = amd.OfdmSlotModulator(mcfg)
    for slot in sorted({0, (1 << mu) - 1}):
        assert mod.get_slot_size(slot) == ref.slot_size(slot, mu, N, ext)
        g = ref.random_grid(rng, ns, bw * 12)
        y = mod.modulate(g, slot)
        want = ref.modulate_slot(g, slot, mu, bw, N, scale, fc, ext)
        assert np.max(np.abs(y - want)) <= 2e-5 * _rms(want), (case, slot)
        rx = (want + (rng.normal(0, 0.05, want.size) + 1j * rng.normal(0, 0.05, want.size)) * _rms(want))
        rx = rx.astype(np.complex64)
        for off in (0, 3):
            dcfg = amd.OfdmDemodulatorConfiguration(numerology=mu, bw_rb=bw, dft_size=N, cp=int(ext), scale=scale,
                                                    center_freq_Hz=fc, nof_samples_window_offset=off)
            dem = amd.OfdmSlotDemodulator(dcfg)
            _check_grid(dem.demodulate(rx, slot), rx, slot, mu, bw, N, scale, fc, off, ext)


def test_batches_ports_and_slots(amd):
    """4 ports x 5 consecutive slots starting mid-subframe, 100 MHz mu=1 4096 points."""
    import torch

    mu, bw, N, scale, fc = 1, 273, 4096, 0.8, 3.5e9
    rng = np.random.default_rng(3)
    nslots, nports, first = 5, 4, 1
    grids = np.stack([np.stack([ref.random_grid(rng, 14, bw * 12) for _ in range(nports)]) for _ in range(nslots)])
    mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(mu, bw, N, 0, scale, fc))
    dem = amd.OfdmSlotDemodulator(amd.OfdmDemodulatorConfiguration(mu, bw, N, 0, scale, fc, 0))
    d_grid = torch.from_numpy(grids.view(np.int16)).cuda()
    samples = mod.modulate_batch(d_grid, first_slot=first)
    back = dem.demodulate_batch(samples, first_slot=first)
    torch.cuda.synchronize()
    s_host = samples.cpu().numpy()
    g_host = back.cpu().numpy().view(np.uint16)
    for s in range(nslots):
        slot = (first + s) % 2
        n = ref.slot_size(slot, mu, N)
        for p in range(nports):
            want = ref.modulate_slot(grids[s, p], slot, mu, bw, N, scale, fc)
            got = s_host[s, p, :n]
            assert np.max(np.abs(got - want)) <= 2e-5 * _rms(want), (s, p)
            _check_grid(g_host[s, p], got, slot, mu, bw, N, scale, fc, 0, False)


@pytest.mark.parametrize("N", [128, 256, 384, 512, 768, 1024, 1536, 2048, 3072, 4096, 6144, 8192])
def test_dft_processor(amd, N):
    import torch

    rng = np.random.default_rng(N)
    for direction in (amd.DftDirection.DIRECT, amd.DftDirection.INVERSE):
        dft = amd.DftProcessor(N, direction)
        x = (rng.normal(size=N) + 1j * rng.normal(size=N)).astype(np.complex64)
        dft.get_input()[:] = x
        exact = np.fft.ifft(x.astype(complex)) * N if direction else np.fft.fft(x.astype(complex))
        y = dft.run()
        assert np.max(np.abs(y - exact)) <= 2e-5 * _rms(exact), (N, direction)
        xb = (rng.normal(size=(9, N)) + 1j * rng.normal(size=(9, N))).astype(np.complex64)
        yb = dft.run_batch(torch.from_numpy(xb).cuda())
        torch.cuda.synchronize()
        yb = yb.cpu().numpy()
        eb = np.fft.ifft(xb.astype(complex), axis=1) * N if direction else np.fft.fft(xb.astype(complex), axis=1)
        assert np.max(np.abs(yb - eb)) <= 2e-5 * _rms(eb), (N, direction)


def test_invalid_configurations(amd):
    with pytest.raises(ValueError):  # DFT not larger than the grid
        amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(1, 273, 2048, 0, 1.0, 0.0))
    with pytest.raises(ValueError):  # scale must be normal
        amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(1, 52, 1024, 0, 0.0, 0.0))
    with pytest.raises(ValueError):  # window offset too large
        amd.OfdmSlotDemodulator(amd.OfdmDemodulatorConfiguration(1, 52, 1024, 0, 1.0, 0.0, 72))
    with pytest.raises(ValueError):
        amd.DftProcessor(1000)
    mod = amd.OfdmSlotModulator(amd.OfdmModulatorConfiguration(1, 52, 1024, 0, 1.0, 0.0))
    with pytest.raises(ValueError):
        mod.modulate(np.zeros((14, 2 * 624), np.uint16), 2)  # slot index beyond the subframe

"""GPU parity: MI355X modulation mapper, soft demapper and scrambling (through
the C-ABI) vs the CPU oracle oracle/srs_oracle_mod.c, itself bit-exact with an
x86-64-v3 build of the reference (tests/test_oracle_vs_ref.py).  Bar:
bit-exact symbols, LLRs and scrambled bits, including AVX2-block / scalar-tail
boundaries, near-zero symbols and invalid noise variances."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

QMS = [0, 1, 2, 4, 6, 8]


@pytest.fixture(scope="module")
def mod():
    import srsran_project_amd as amd

    return amd.Modulator()


@pytest.mark.parametrize("qm", QMS)
def test_modulate_and_demodulate(mod, qm):
    rng = np.random.default_rng(qm)
    bps = 1 if qm < 2 else qm
    for nsym in (1, 3, 4, 15, 16, 17, 33, 3276 * 12 + 5):
        bits = rng.integers(0, 256, (nsym * bps + 7) // 8).astype(np.uint8)
        sym = mod.modulate(bits, nsym, qm)
        want = oracle.modulate(bits, nsym, qm)
        np.testing.assert_array_equal(sym.view(np.uint32), want.view(np.uint32), err_msg="mod qm %d n %d" % (qm, nsym))
        rx = (want + (rng.normal(size=nsym) + 1j * rng.normal(size=nsym)) * 0.35).astype(np.complex64)
        rx[rng.random(nsym) < 0.02] = 0
        nv = rng.uniform(0.003, 2.0, nsym).astype(np.float32)
        nv[rng.random(nsym) < 0.03] = 0.0
        nv[rng.random(nsym) < 0.02] = -1.0
        np.testing.assert_array_equal(mod.demodulate_soft(rx, nv, qm), oracle.demodulate(rx, nv, qm),
                                      err_msg="demod qm %d n %d" % (qm, nsym))


def test_device_batches(mod):
    import torch

    rng = np.random.default_rng(7)
    nsym = 3276 * 14
    for qm in (2, 8):
        bits = rng.integers(0, 256, nsym * qm // 8).astype(np.uint8)
        d = mod.modulate_batch(torch.from_numpy(bits).cuda(), nsym, qm)
        nv = torch.full((nsym,), 0.1, dtype=torch.float32, device="cuda")
        llr = mod.demodulate_soft_batch(d, nv, qm)
        torch.cuda.synchronize()
        want = oracle.modulate(bits, nsym, qm)
        np.testing.assert_array_equal(d.cpu().numpy().view(np.uint32), want.view(np.uint32))
        np.testing.assert_array_equal(llr.cpu().numpy(), oracle.demodulate(want, np.full(nsym, 0.1, np.float32), qm))


def test_scrambling(mod):
    import torch

    rng = np.random.default_rng(9)
    for c_init in (0, 1, 0x5A5A5A5, 2 ** 31 - 1):
        for n in (1, 7, 31, 32, 33, 1000, 250001):
            bits = rng.integers(0, 2, n).astype(np.uint8)
            c = oracle.prbs(c_init, n)
            out = mod.scramble_bits(np.packbits(bits), n, c_init)
            np.testing.assert_array_equal(np.unpackbits(out)[:n], bits ^ c, err_msg=str((c_init, n)))
            llr = rng.integers(-127, 128, n).astype(np.int8)
            want = np.where(c == 1, -llr.astype(np.int16), llr.astype(np.int16)).astype(np.int8)
            np.testing.assert_array_equal(mod.descramble_llrs(llr, c_init), want)
    x = torch.from_numpy(rng.integers(-100, 100, 1 << 20).astype(np.int8)).cuda()
    y = mod.descramble_llrs_batch(x, 77)
    torch.cuda.synchronize()
    c = oracle.prbs(77, 1 << 20)
    xn = x.cpu().numpy()
    np.testing.assert_array_equal(y.cpu().numpy(), np.where(c == 1, -xn, xn))


def test_invalid(mod):
    with pytest.raises(ValueError):
        mod.modulate(np.zeros(4, np.uint8), 4, 3)

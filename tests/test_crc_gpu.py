"""GPU parity: MI355X CRC calculator (through the C-ABI) vs the CPU oracle
(srs_oracle_crc_bits, pinned to the reference's crc_calculator_generic_impl in
tests/test_oracle_vs_ref.py::test_crc_matches_reference).  Follows the
reference's crc_calculator_test.cpp: byte, bit and bit_buffer forms, every
polynomial, sizes {8, 16, 32, 257, 997, 6012}; plus batched rows, the in-place
attachment used by codeblock segmentation and a transport-block-sized row.
Bar: bit-exact."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

POLYS = [0, 1, 2, 3, 4, 5]
ORDER = {0: 24, 1: 24, 2: 24, 3: 16, 4: 11, 5: 6}
SIZES = [8, 16, 32, 257, 997, 6012]


@pytest.fixture(scope="module")
def calcs():
    import srsran_project_amd as amd

    return {p: amd.CrcCalculator(p, max_bits=1 << 21) for p in POLYS}


@pytest.mark.parametrize("poly", POLYS)
def test_reference_sizes(calcs, poly):
    rng = np.random.default_rng(poly)
    c = calcs[poly]
    assert c.order == ORDER[poly]
    for n in SIZES:
        data = rng.integers(0, 256, n).astype(np.uint8)
        bits = np.unpackbits(data)
        assert c.calculate_byte(data) == oracle.crc_bits(poly, bits), ("byte", n)
        b1 = rng.integers(0, 2, n).astype(np.uint8)
        assert c.calculate_bit(b1) == oracle.crc_bits(poly, b1), ("bit", n)
        assert c.calculate(np.packbits(b1), n) == oracle.crc_bits(poly, b1), ("bit_buffer", n)


def test_empty_and_tiny(calcs):
    for p in POLYS:
        assert calcs[p].calculate(np.zeros(0, np.uint8), 0) == 0
        for n in range(1, 20):
            b = np.ones(n, np.uint8)
            assert calcs[p].calculate_bit(b) == oracle.crc_bits(p, b), (p, n)


def test_batch_and_attach(calcs):
    import torch

    rng = np.random.default_rng(11)
    for p in (0, 1, 3, 5):
        for n in (1, 100, 8424, 8448 - 24):
            rows = 37
            stride = (n + ORDER[p] + 7) // 8 + 3
            host = rng.integers(0, 256, (rows, stride)).astype(np.uint8)
            d = torch.from_numpy(host).cuda()
            got = calcs[p].calculate_batch(d, n).cpu().numpy().view(np.uint32)
            bits = np.unpackbits(host, axis=1)
            want = np.array([oracle.crc_bits(p, bits[r, :n]) for r in range(rows)], np.uint32)
            np.testing.assert_array_equal(got, want, err_msg="poly %d n %d" % (p, n))
            calcs[p].attach_batch(d, n)
            out = np.unpackbits(d.cpu().numpy(), axis=1)
            L = ORDER[p]
            for r in range(rows):
                crc_bits = [(int(want[r]) >> (L - 1 - k)) & 1 for k in range(L)]
                np.testing.assert_array_equal(out[r, n:n + L], crc_bits)
                # bits outside [n, n+L) untouched
                np.testing.assert_array_equal(out[r, :n], bits[r, :n])
                np.testing.assert_array_equal(out[r, n + L:], bits[r, n + L:])
                # a message followed by its CRC divides evenly: CRC of the whole is 0
                assert oracle.crc_bits(p, out[r, :n + L]) == 0


def test_transport_block_row(calcs):
    """One ~1.2 Mbit row (a large TB CRC24A) through the device form."""
    import torch

    rng = np.random.default_rng(5)
    n = 1_213_032
    host = rng.integers(0, 256, (1, (n + 7) // 8)).astype(np.uint8)
    got = calcs[0].calculate_batch(torch.from_numpy(host).cuda(), n).cpu().numpy().view(np.uint32)[0]
    assert got == oracle.crc_bits(0, np.unpackbits(host[0])[:n])


def test_invalid_arguments(calcs):
    import srsran_project_amd as amd

    with pytest.raises(Exception):
        amd.CrcCalculator(9)
    with pytest.raises(Exception):
        calcs[0].calculate(np.zeros(1 << 19, np.uint8), (1 << 21) + 1)

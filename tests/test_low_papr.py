"""Low-PAPR base sequences (include/srsran_amd/low_papr.h, the transform-precoded PUSCH DM-RS): every length
the reference generates, every sequence group u and sequence number v, bit-exact (float bits) against the
compiled low_papr_sequence_generator_impl (oracle/_ref).  Host code: runs on the CPU."""
import re

import numpy as np
import pytest

import oracle
import srsran_project_amd as amd

pytestmark = pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref/libsrsran_ref.so not built")


def _sizes():
    text = open("srsran_project_amd/csrc/low_papr_tables.inc").read()
    return [int(x) for x in re.findall(r"\d+", text.split("SRS_LOW_PAPR_SIZES[82] = {")[1].split("}")[0])]


def test_low_papr_matches_reference_bit_exact():
    from oracle.chest import ref_low_papr

    n = 0
    for M in _sizes():
        for u in range(30):
            for v in ((0, 1) if M >= 72 else (0,)):
                got, want = amd.low_papr_sequence(M, u, v), ref_low_papr(M, u, v)
                np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="M%d u%d v%d" % (M, u, v))
                n += 1
    assert n == 4650


def test_low_papr_properties_and_errors():
    for M in (6, 30, 36, 1632):
        s = amd.low_papr_sequence(M, 7)
        assert np.allclose(np.abs(s), 1.0, atol=1e-6)
    assert amd.low_papr_length_valid(1650) is False and amd.low_papr_length_valid(1620) is True
    for M, u, v in ((7, 0, 0), (36, 30, 0), (36, 0, 1), (72, 0, 2)):
        with pytest.raises(ValueError):
            amd.low_papr_sequence(M, u, v)

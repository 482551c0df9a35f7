"""GPU parity: the MI355X UCI decoder (include/srsran_amd/uci_decoder.h) against the compiled reference
uci_decoder_impl (short_block_detector_impl for 1-11 bits, the polar chain with CRC6 / CRC11 for 12-1706 bits, one
or two codeblocks): message bits and uci_status identical on encoded payloads through noise from clean to
undecodable, and on too-short / all-zero inputs."""
import numpy as np
import pytest

import oracle
from oracle import pusch_proc as pp

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(oracle.REF is None, reason="oracle/_ref not built")]


def _llrs(bits, rng, amp, sigma):
    b = np.where(bits > 1, rng.integers(0, 2, bits.size), bits).astype(np.int16)  # placeholders: any bit
    x = (1 - 2 * b) * amp + rng.normal(0, sigma, bits.size)
    return np.clip(np.round(x), -120, 120).astype(np.int8)


@pytest.mark.parametrize("K", list(range(1, 12)) + [12, 19, 20, 40, 200, 400, 1013])
def test_uci_decode_matches_reference(K):
    import srsran_project_amd as amd

    dec = amd.UciDecoder(device=0)
    rng = np.random.default_rng(K)
    n_valid = 0
    for trial in range(24):
        qm = int(rng.choice([1, 2, 4, 6, 8]))
        if K <= 11:
            E = qm * int(rng.integers(max(1, 20 // qm), 200 // qm + 2))
        else:
            E = max(int((K + 11) * rng.uniform(1.3, 3.0)), 1100 if K >= 360 and trial % 2 else 0)
            E -= E % qm
        msg = rng.integers(0, 2, K).astype(np.uint8)
        cw = pp.uci_encode(msg, E, qm)
        sigma = [0.0, 20.0, 60.0, 200.0][trial % 4]
        llrs = _llrs(cw, rng, 40, sigma)
        if trial == 5:
            llrs[:] = 0  # too few non-zero soft bits
        got, gst = dec.decode(llrs, K, qm)
        want, wst = pp.ref_uci_decode(llrs, K, qm)
        assert gst == wst, (K, E, qm, trial, gst, wst)
        np.testing.assert_array_equal(got, want, err_msg="K%d E%d qm%d trial %d" % (K, E, qm, trial))
        n_valid += wst == amd.UCI_VALID
    assert n_valid >= 6

"""GPU parity: MI355X polar encode / decode chains (through the C-ABI) vs the
CPU oracle oracle/srs_oracle_polar.c, itself pinned to the reference's polar
classes (tests/test_oracle_vs_ref.py).  Bar: bit-exact.  Codes: PDCCH DCI sizes
at every aggregation level (nMax 9) and UCI sizes with and without
parity-check bits (nMax 10), repetition / puncturing / shortening, channel
interleaver on and off; LLRs include +-infinity and zeros."""
import numpy as np
import pytest

import oracle
from tests.test_oracle_vs_ref import polar_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    import srsran_project_amd as amd

    return amd


def _llrs(rng, cw):
    E = cw.size
    llr = np.clip(np.round((1 - 2.0 * cw) * 5 + rng.normal(0, 7, E)), -120, 120).astype(np.int8)
    llr[rng.random(E) < 0.03] = 127
    llr[rng.random(E) < 0.03] = -127
    llr[rng.random(E) < 0.02] = 0
    return llr


def test_polar_single_codewords(amd):
    rng = np.random.default_rng(1)
    for K, E, nMax in polar_cases():
        try:
            oracle.polar_code(K, E, nMax)
        except ValueError:
            continue
        for ibil in (0, 1):
            code = amd.PolarCode(K, E, nMax, ibil)
            N, kmask, pc = oracle.polar_code(K, E, nMax)
            assert code.get_N() == N and code.get_nPC() == pc.size
            np.testing.assert_array_equal(code.get_K_set(), kmask)
            m = rng.integers(0, 2, K).astype(np.uint8)
            cw = code.encode(m)
            np.testing.assert_array_equal(cw, oracle.polar_encode_chain(m, E, nMax, ibil), err_msg=str((K, E, ibil)))
            llr = _llrs(rng, cw)
            np.testing.assert_array_equal(code.decode(llr), oracle.polar_decode_chain(llr, K, nMax, ibil),
                                          err_msg=str((K, E, ibil)))


@pytest.mark.parametrize("K,E,nMax,ibil", [(57, 864, 9, 0), (140, 1728, 9, 0), (22, 300, 10, 1), (400, 1100, 10, 1),
                                           (1000, 8192, 10, 1)])
def test_polar_batches(amd, K, E, nMax, ibil):
    import torch

    rng = np.random.default_rng(K + E)
    n = 777
    code = amd.PolarCode(K, E, nMax, ibil)
    msgs = rng.integers(0, 2, (n, K)).astype(np.uint8)
    cws = code.encode_batch(torch.from_numpy(msgs).cuda())
    torch.cuda.synchronize()
    cws = cws.cpu().numpy()
    llrs = np.stack([_llrs(rng, cws[i]) for i in range(n)])
    dec = code.decode_batch(torch.from_numpy(llrs).cuda())
    torch.cuda.synchronize()
    dec = dec.cpu().numpy()
    for i in range(0, n, 7):
        np.testing.assert_array_equal(cws[i], oracle.polar_encode_chain(msgs[i], E, nMax, ibil))
        np.testing.assert_array_equal(dec[i], oracle.polar_decode_chain(llrs[i], K, nMax, ibil))
    # noiseless: decoding returns the message
    clean = ((1 - 2 * cws.astype(np.int16)) * 20).astype(np.int8)
    back = code.decode_batch(torch.from_numpy(clean).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(back.cpu().numpy(), msgs)


def test_polar_invalid(amd):
    with pytest.raises(ValueError):
        amd.PolarCode(20, 200, 9)  # K below the downlink range
    with pytest.raises(ValueError):
        amd.PolarCode(27, 200, 10)  # K in the excluded 26..30 range
    with pytest.raises(ValueError):
        amd.PolarCode(100, 100, 10)  # E must exceed K

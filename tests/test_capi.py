"""C-ABI library checks that run without a GPU: it loads, exports every
function declared in include/srsran_amd/*.h, and its host-only entry points
behave."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "srsran_amd", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(srs_amd_\w+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_functions():
    assert "srs_amd_ldpc_decode_batch" in declared_functions()


def test_library_exports_every_declared_symbol():
    from srsran_project_amd import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_gfx950_code_object():
    from srsran_project_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_host_only_entry_points():
    import srsran_project_amd as amd

    assert amd.message_length(1, 384) == 8448
    assert amd.codeblock_length(1, 384) == 25344
    assert amd.message_length(2, 52) == 520
    assert amd.codeblock_length(2, 52) == 2600
    assert amd.message_length(1, 17) == 0
    assert amd.message_length(3, 8) == 0


def test_create_without_gpu_fails_loudly():
    import torch

    import srsran_project_amd as amd

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(Exception):
        amd.LdpcDecoder("simd")


def test_invalid_decoder_type():
    import srsran_project_amd as amd

    with pytest.raises(ValueError):
        amd.create_ldpc_decoder_factory_hip("neon")


def test_polar_construction_host_only():
    """The product's polar_code::set restatement equals the oracle (which is
    pinned to the reference) -- host-only entry point, no device needed."""
    import oracle
    import srsran_project_amd as amd
    from tests.test_oracle_vs_ref import polar_cases

    for K, E, nMax in polar_cases():
        try:
            want = oracle.polar_code(K, E, nMax)
        except ValueError:
            with pytest.raises(ValueError):
                amd.polar_code_construct(K, E, nMax)
            continue
        got = amd.polar_code_construct(K, E, nMax)
        assert got[0] == want[0]
        np.testing.assert_array_equal(got[1], want[1])
        np.testing.assert_array_equal(got[2], want[2])


def test_polar_interleaver_host_only():
    import oracle
    import srsran_project_amd as amd

    rng = np.random.default_rng(4)
    for K in (1, 20, 164):
        b = rng.integers(0, 2, K).astype(np.uint8)
        for d in (0, 1):
            np.testing.assert_array_equal(amd.polar_interleave(b, d), oracle.polar_interleave(b, d))
    with pytest.raises(ValueError):
        amd.polar_interleave(np.zeros(165, np.uint8))


def test_tbs_calculator_golden():
    """srs_amd_tbs_calculate vs the reference's 256 TBS calculator test vectors
    (tests/golden/tbs_calculator.json, extracted by tools/gen_tbs_golden.py)."""
    import json

    import srsran_project_amd as amd

    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "tbs_calculator.json")))["cases"]
    assert len(cases) == 256
    for c in cases:
        got = amd.tbs_calculator_calculate(c["nof_symb_sh"], c["nof_dmrs_prb"], c["nof_oh_prb"], c["qm"],
                                           np.float32(float(c["target_code_rate"])), c["nof_layers"],
                                           c["tb_scaling_field"], c["n_prb"])
        assert got == c["tbs"], c


def test_sch_plan_host_only():
    """The product's segmentation geometry equals oracle/sch.py (pinned to the reference)."""
    import random

    import oracle.sch as osch
    import srsran_project_amd as amd

    rnd = random.Random(1)
    for _ in range(2000):
        bg, qm, lay = rnd.choice([1, 2]), rnd.choice([1, 2, 4, 6, 8]), rnd.choice([1, 2, 3, 4])
        tbs, nre = 8 * rnd.randint(1, 159000), lay * rnd.randint(1, 40000)
        want = osch.plan(tbs, bg, 0, qm, 0, lay, nre)
        if want["nof_segments"] > 162 or (want["rm_length_short"] == 0 and want["nof_short_segments"] > 0):
            with pytest.raises(ValueError):
                amd.sch_plan(tbs, bg, 0, qm, 0, lay, nre)
            continue
        assert amd.sch_plan(tbs, bg, 0, qm, 0, lay, nre).as_dict() == want


def test_integration_plugins_built_against_reference_headers():
    """integration/_build/libsrsran_amd_hal.so -- the srsRAN plug-ins over the C-ABI (hal::hw_accelerator_pusch_dec
    and its factory, the PDSCH encoder plug-in, the ldpc_decoder / dft_processor / channel_equalizer factories), compiled against the reference's own headers -- exists, links
    with no undefined symbols (-Wl,--no-undefined) and exports the factory entry points."""
    import subprocess

    path = os.path.join(os.path.dirname(__file__), "..", "integration", "_build", "libsrsran_amd_hal.so")
    if not os.path.exists(path):
        pytest.skip("integration plug-ins not built (the reference headers are needed)")
    out = subprocess.run(["nm", "-D", "-C", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    assert "srsran::hip::create_hip_pusch_dec_acc_factory(srsran::hip::pusch_dec_accelerator_config const&)" in out
    assert "srsran::hip::create_ldpc_decoder_factory_hip(" in out
    assert "srsran::hip::create_hip_pdsch_enc_acc_factory(srsran::hip::pdsch_enc_accelerator_config const&)" in out
    assert "srsran::hip::create_dft_processor_factory_hip(int)" in out
    assert "srsran::hip::create_channel_equalizer_factory_hip(srsran::channel_equalizer_algorithm_type, int)" in out
    ctypes.CDLL(path)  # loads with libsrsran_amd.so found through its rpath


def test_channel_processor_plugins_take_only_reference_interface_symbols():
    """integration/_build/libsrsran_amd_phy.so -- the pusch / pdsch / pdcch / ssb / pucch processor plug-ins -- exports its factory
    entry points and leaves undefined only the vtables / typeinfo of the reference's factory interfaces (their key
    function, create(srslog::basic_logger&), lives in the srsRAN library the plug-in is linked into) and
    rb_allocation::get_crb_mask; with the
    reference's compiled factories loaded first (oracle/_ref/libsrsran_ref.so) it loads."""
    import subprocess

    root = os.path.join(os.path.dirname(__file__), "..")
    path = os.path.join(root, "integration", "_build", "libsrsran_amd_phy.so")
    ref = os.path.join(root, "oracle", "_ref", "libsrsran_ref.so")
    if not os.path.exists(path) or not os.path.exists(ref):
        pytest.skip("channel-processor plug-ins not built (the reference headers are needed)")
    out = subprocess.run(["nm", "-D", "-C", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    assert "srsran::hip::create_pusch_processor_factory_hip(srsran::hip::pusch_processor_hip_config const&)" in out
    assert "srsran::hip::create_pdsch_processor_factory_hip(srsran::hip::pdsch_processor_hip_config const&)" in out
    assert "srsran::hip::create_pdcch_processor_factory_hip(srsran::hip::pdcch_processor_hip_config const&)" in out
    assert "srsran::hip::create_ssb_processor_factory_hip(srsran::hip::ssb_processor_hip_config const&)" in out
    assert "srsran::hip::create_pucch_processor_factory_hip(srsran::hip::pucch_processor_hip_config const&)" in out
    undef = subprocess.run(["nm", "-D", "-C", "-u", path], capture_output=True, text=True, check=True).stdout
    ref_syms = sorted({l.split(" U ")[-1].strip() for l in undef.splitlines() if "srsran::" in l or "srslog::" in l})
    allowed = {"vtable for srsran::pusch_processor_factory", "typeinfo for srsran::pusch_processor_factory",
               "vtable for srsran::pdsch_processor_factory", "typeinfo for srsran::pdsch_processor_factory",
               "vtable for srsran::pdcch_processor_factory", "typeinfo for srsran::pdcch_processor_factory",
               "vtable for srsran::ssb_processor_factory", "typeinfo for srsran::ssb_processor_factory",
               "vtable for srsran::pucch_processor_factory", "typeinfo for srsran::pucch_processor_factory",
               "srsran::pucch_processor_factory::create(srslog::detail::logger_impl<srslog::basic_logger_channels, "
               "srslog::basic_levels>&)",
               "srsran::rb_allocation::get_crb_mask(unsigned int, unsigned int) const"}
    assert set(ref_syms) <= allowed, ref_syms
    ctypes.CDLL(ref, mode=ctypes.RTLD_GLOBAL)
    ctypes.CDLL(path)

"""The REFERENCE's full PDSCH + PUSCH slot chain (oracle/ref_chain.cpp) --
TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and the end-to-end
pipeline parity test. Implementations are the ones the reference's "auto"
software factories pick on the running host (ref_builders.h)."""
import ctypes as _c
import os

import numpy as np

from . import REF, _ptr


class RefChainConfig(_c.Structure):
    """srs_ref_chain_config (oracle/ref_chain.cpp)."""

    _fields_ = [(n, _c.c_uint32) for n in ("numerology", "slot", "nof_prb", "dft_size", "rnti", "n_id", "qm",
                                           "dmrs_symbol_mask", "nof_cdm_groups_without_data", "dl_layers",
                                           "dl_ports", "dl_start", "dl_nsym", "dl_tbs", "dl_bg")] + \
        [("dl_weights", _c.c_float * 32), ("dl_dmrs_amplitude", _c.c_float)] + \
        [(n, _c.c_uint32) for n in ("ul_layers", "ul_ports", "ul_start", "ul_nsym", "ul_tbs", "ul_bg",
                                    "ul_iterations")] + \
        [("ul_target_code_rate", _c.c_float), ("choice", _c.c_int32), ("ul_td", _c.c_int32)]


if REF is not None and hasattr(REF, "srs_ref_chain_run"):
    _CP = _c.POINTER(RefChainConfig)
    REF.srs_ref_chain_slot_size.restype = _c.c_uint
    REF.srs_ref_chain_slot_size.argtypes = [_CP]
    REF.srs_ref_chain_run.restype = _c.c_int
    REF.srs_ref_chain_run.argtypes = [_CP, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_void_p,
                                      _c.c_void_p]
    REF.srs_ref_chain_many.restype = _c.c_double
    REF.srs_ref_chain_many.argtypes = [_CP, _c.c_void_p, _c.c_void_p, _c.c_uint, _c.c_uint, _c.c_void_p,
                                       _c.c_void_p]

STAGES = ["pdsch_encode", "pdsch_modulate+dmrs", "ofdm_modulate", "ofdm_demodulate", "pusch_process"]


def make_config(**kw):
    c = RefChainConfig()
    w = kw.pop("dl_weights")
    for k, v in kw.items():
        setattr(c, k, v)
    w = np.asarray(w, np.complex64)
    flat = np.zeros(32, np.float32)
    flat[:2 * w.size] = w.reshape(-1).view(np.float32)
    c.dl_weights[:] = flat.tolist()
    return c


def slot_size(cfg):
    return REF.srs_ref_chain_slot_size(_c.byref(cfg))


def run(cfg, tb_dl, ul_samples):
    """One cell-slot. Returns (dl grid uint32 [dl_ports][14][nsubc], dl samples complex64 [dl_ports][n],
    ul tb bytes, tb_crc_ok, ldpc iterations)."""
    n = slot_size(cfg)
    nsubc = cfg.nof_prb * 12
    grid = np.zeros((cfg.dl_ports, 14, nsubc), np.uint32)
    samp = np.zeros((cfg.dl_ports, n), np.complex64)
    tb = np.zeros(cfg.ul_tbs // 8, np.uint8)
    res = np.zeros(2, np.float64)
    ul = np.ascontiguousarray(ul_samples, np.complex64)
    tbd = np.ascontiguousarray(tb_dl, np.uint8)
    REF.srs_ref_chain_run(_c.byref(cfg), _ptr(tbd), _ptr(ul), _ptr(grid), _ptr(samp), _ptr(tb), _ptr(res))
    return grid, samp, tb, bool(res[0]), int(res[1])


def many(cfg, tb_dl, ul_samples, nof_slots, threads):
    """CPU baseline: nof_slots cell-slots on `threads` threads. Returns (wall s, stage seconds dict summed over
    all slots, slots with TB CRC ok, LDPC iterations summed)."""
    st = np.zeros(5, np.float64)
    cnt = np.zeros(2, np.uint32)
    ul = np.ascontiguousarray(ul_samples, np.complex64)
    tbd = np.ascontiguousarray(tb_dl, np.uint8)
    wall = REF.srs_ref_chain_many(_c.byref(cfg), _ptr(tbd), _ptr(ul), nof_slots, threads, _ptr(st), _ptr(cnt))
    return wall, dict(zip(STAGES, st.tolist())), int(cnt[0]), int(cnt[1])


def host_cores():
    """(logical CPUs this process may use, physical cores among them) from the affinity mask and sysfs."""
    cpus = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in cpus:
        try:
            base = "/sys/devices/system/cpu/cpu%d/topology/" % c
            with open(base + "core_id") as f:
                core = f.read().strip()
            with open(base + "physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", str(c)))
    return len(cpus), len(cores)

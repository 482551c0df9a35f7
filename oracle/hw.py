"""TEST INFRASTRUCTURE: the reference's hardware-accelerated PUSCH decoder (pusch_decoder_hw_impl, compiled from
/root/reference) driving the MI355X plug-in (integration/hip_accelerator_pusch_dec.cpp) -- oracle/hw_harness.cpp,
built into oracle/_ref/libsrsran_ref_hw.so.  Loading it initialises the GPU (the plug-in allocates its HARQ
buffers in HBM), so only GPU tests use it."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
HW_PATH = os.path.join(_HERE, "_ref", "libsrsran_ref_hw.so")
HAL_PATH = os.path.join(_HERE, "..", "integration", "_build", "libsrsran_amd_hal.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(HW_PATH):
            raise ImportError("oracle/_ref/libsrsran_ref_hw.so not built (make -C integration && make -C oracle)")
        L = ctypes.CDLL(HW_PATH)
        P, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        L.srs_ref_hw_ctx_create.restype = P
        L.srs_ref_hw_ctx_create.argtypes = [i, i]
        L.srs_ref_hw_ctx_destroy.argtypes = [P]
        L.srs_ref_hw_ctx_sibling.restype = P
        L.srs_ref_hw_ctx_sibling.argtypes = [P, i]
        L.srs_ref_hw_rx_buffer_create.restype = P
        L.srs_ref_hw_rx_buffer_create.argtypes = [u, u]
        L.srs_ref_hw_rx_buffer_destroy.argtypes = [P]
        L.srs_ref_hw_pusch_decode.restype = i
        L.srs_ref_hw_pusch_decode.argtypes = [P, P, P, u, P, u] + [u] * 6 + [i, i, P]
        # adapter_harness.cpp
        f, d = ctypes.c_float, ctypes.c_double
        L.srs_ref_hw_pdsch_encode.restype = i
        L.srs_ref_hw_pdsch_encode.argtypes = [i, i, P, u] + [u] * 6 + [P]
        L.srs_ref_hw_pdsch_enc_forced_failure.restype = i
        L.srs_ref_hw_pdsch_enc_forced_failure.argtypes = [i]
        L.srs_ref_hip_ofdm_modulate_slot.restype = i
        L.srs_ref_hip_ofdm_modulate_slot.argtypes = [i, u, u, u, i, f, d, u, P, P]
        L.srs_ref_hip_ofdm_demodulate_slot.restype = i
        L.srs_ref_hip_ofdm_demodulate_slot.argtypes = [i, u, u, u, i, u, f, d, u, P, P]
        L.srs_ref_hip_pusch_demodulate.restype = i
        L.srs_ref_hw_ofdm_plugin.restype = i
        L.srs_ref_hw_ofdm_plugin.argtypes = [i, i, u, u, u, i, u, f, d, d, u, P, P]
        L.srs_ref_hw_ofdm_bench.restype = d
        L.srs_ref_hw_ofdm_bench.argtypes = [i, i, i, u, u, u, u, P, P, P]
        L.srs_ref_hip_pusch_demodulate.argtypes = [i, P, u, u, P, u, P, u, u, i, P, u, u, u, i, u, i, i, i, P, u, P]
        L.srs_ref_hip_ldpc_pusch_decode.restype = i
        L.srs_ref_hip_ldpc_pusch_decode.argtypes = [i, P, P, u, P, u] + [u] * 6 + [i] * 4 + [P]
        _lib = L
    return _lib


class HwPuschDecoder:
    """pusch_decoder_hw_impl + the MI355X hal::hw_accelerator_pusch_dec (external HARQ in HBM)."""

    def __init__(self, device=0, generic=False, sibling_of=None):
        if sibling_of is not None:  # another accelerator of the same factory (shared HBM HARQ pool)
            self.h = lib().srs_ref_hw_ctx_sibling(sibling_of.h, int(generic))
            self._base = sibling_of  # keeps the factory's owner alive
        else:
            self.h = lib().srs_ref_hw_ctx_create(int(device), int(generic))

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_hw_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HwRxBuffer:
    """rx_buffer of one HARQ process; its codeblocks have absolute ids abs_base + index (HARQ rows in HBM)."""

    def __init__(self, nof_cbs, abs_base):
        self.h = lib().srs_ref_hw_rx_buffer_create(int(nof_cbs), int(abs_base))

    def __del__(self):
        if getattr(self, "h", None):
            lib().srs_ref_hw_rx_buffer_destroy(self.h)
            self.h = None


def hw_pusch_decode(dec, llrs, p, rxbuf, tb_out, max_iterations=6, use_early_stop=True, new_data=True):
    """Returns (tb_crc_ok, nof_cbs, nof_obs, iteration sum, min, max), as oracle.ref_pusch_decode."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    res = np.zeros(6, np.float64)
    r = lib().srs_ref_hw_pusch_decode(dec.h, rxbuf.h, llrs.ctypes.data, llrs.size, tb_out.ctypes.data, tb_out.size,
                                      p["base_graph"], p["rv"], p["modulation_order"], p["Nref"], p["nof_layers"],
                                      max_iterations, int(use_early_stop), int(new_data), res.ctypes.data)
    if r != 0:
        raise RuntimeError("pusch_decoder_hw_impl did not notify")
    return bool(res[0]), int(res[1]), int(res[2]), int(round(res[3])), int(res[4]), int(res[5])


def _p(a):
    return a.ctypes.data


def hw_pdsch_encode(tb_bytes, p, cb_mode=False, device=0):
    """The reference's pdsch_encoder_hw_impl with the MI355X hal::hw_accelerator_pdsch_enc (TB mode, or CB mode).
    p: an oracle.sch.plan() dict. Codeword bits, one per byte (as oracle.ref_pdsch_encode)."""
    tb = np.ascontiguousarray(tb_bytes, dtype=np.uint8)
    cw = np.zeros(p["cw_length"], np.uint8)
    lib().srs_ref_hw_pdsch_encode(device, int(cb_mode), _p(tb), tb.size, p["base_graph"], p["rv"],
                                  p["modulation_order"], p["Nref"], p["nof_layers"], p["nof_ch_symbols"], _p(cw))
    return cw


def hip_ofdm_modulate_slot(grid_u16, slot, numerology, bw_rb, dft_size, scale, fc, n, device=0):
    """ofdm_slot_modulator_impl (one port) with the MI355X dft_processor; n = the slot size in samples."""
    g = np.ascontiguousarray(grid_u16, dtype=np.uint16)
    out = np.zeros(n, np.complex64)
    if lib().srs_ref_hip_ofdm_modulate_slot(device, numerology, bw_rb, dft_size, 0, scale, fc, slot, _p(g), _p(out)):
        raise ValueError("the MI355X dft_processor refused size %d" % dft_size)
    return out


def hip_ofdm_demodulate_slot(samples, slot, numerology, bw_rb, dft_size, scale, fc, device=0):
    """ofdm_slot_demodulator_impl (one port) with the MI355X dft_processor; grid uint16 [14][2 * 12 * bw_rb]."""
    x = np.ascontiguousarray(samples, dtype=np.complex64)
    grid = np.zeros((14, 2 * bw_rb * 12), np.uint16)
    if lib().srs_ref_hip_ofdm_demodulate_slot(device, numerology, bw_rb, dft_size, 0, 0, scale, fc, slot, _p(x),
                                              _p(grid)):
        raise ValueError("the MI355X dft_processor refused size %d" % dft_size)
    return grid


OFDM_PLUGIN_MODES = {"slot_mod": 0, "symbol_mod": 1, "slot_demod": 2, "symbol_demod": 3}


def ofdm_plugin(mode, data, slot, numerology, bw_rb, dft_size, scale, fc, fc2=None, extended_cp=False,
                window_offset=0, n=None, device=0):
    """One port of one slot through the ofdm_modulator_factory / ofdm_demodulator_factory plug-ins of
    integration/ofdm_modulator_hip.h ("slot_mod" / "symbol_mod": data = grid uint16 [nsymb][2 * 12 * bw_rb], returns
    n complex samples; "slot_demod" / "symbol_demod": data = samples, returns the grid). fc2: the symbol forms call
    set_center_frequency(fc2) first."""
    ns = 12 if extended_cp else 14
    fc2 = fc if fc2 is None else fc2
    if OFDM_PLUGIN_MODES[mode] < 2:
        grid = np.ascontiguousarray(data, dtype=np.uint16)
        samples = np.zeros(n, np.complex64)
    else:
        samples = np.ascontiguousarray(data, dtype=np.complex64)
        grid = np.zeros((ns, 2 * bw_rb * 12), np.uint16)
    if lib().srs_ref_hw_ofdm_plugin(device, OFDM_PLUGIN_MODES[mode], numerology, bw_rb, dft_size, int(extended_cp),
                                    window_offset, scale, fc, fc2, slot, _p(grid), _p(samples)):
        raise ValueError("the OFDM plug-in factory refused the configuration")
    return samples if OFDM_PLUGIN_MODES[mode] < 2 else grid


def ofdm_bench(plugin, demod, numerology, bw_rb, dft_size, calls, device=0):
    """Seconds for `calls` one-port slot (de)modulations through the plug-in (plugin=True) or the reference's
    ofdm_slot_(de)modulator_impl over the generic DFT on this thread (plugin=False)."""
    rng = np.random.default_rng(1)
    grid = rng.integers(0, 1 << 16, (14, 2 * bw_rb * 12), dtype=np.uint16) & 0x3fff  # small finite bf16 values
    samples = np.zeros(1 << 20, np.complex64)
    gout = np.zeros_like(grid)
    return lib().srs_ref_hw_ofdm_bench(device, int(plugin), int(demod), numerology, bw_rb, dft_size, calls, _p(grid),
                                       _p(samples), _p(gout))


def hip_pusch_demodulate(grid, estimates, noise_vars, rnti, n_id, qm, crbs, start_symbol, nof_symbols, dmrs_symb_mask,
                         dmrs_type2, nof_cdm_groups_without_data, nof_layers, mmse=False, device=0):
    """pusch_demodulator_impl with the MI355X channel_equalizer (arguments as oracle.pusch_demod.ref_pusch_demodulate)."""
    from .pusch_demod import data_re_mask

    P, _, nsubc = grid.shape
    mask = data_re_mask(nsubc, crbs, start_symbol, nof_symbols, dmrs_symb_mask, dmrs_type2,
                        nof_cdm_groups_without_data)
    nllr = int(mask.sum()) * nof_layers * qm
    g = np.ascontiguousarray(grid, np.uint32)
    e = np.ascontiguousarray(estimates, np.uint32)
    nv = np.ascontiguousarray(noise_vars, np.float32)
    cr = np.zeros(nsubc // 12, np.uint8)
    cr[list(crbs)] = 1
    out = np.zeros(nllr, np.int8)
    sinr = np.zeros(15, np.float32)
    r = lib().srs_ref_hip_pusch_demodulate(device, _p(g), P, nsubc, _p(e), nof_layers, _p(nv), rnti, n_id, qm, _p(cr),
                                           start_symbol, nof_symbols, dmrs_symb_mask, int(dmrs_type2),
                                           nof_cdm_groups_without_data, int(mmse), 0, 0, _p(out), nllr, _p(sinr))
    if r < 0:
        raise RuntimeError("pusch_demodulator_impl with the MI355X equalizer failed (%d)" % r)
    return out


def hip_ldpc_pusch_decode(llrs, p, rxbuf, tb_out, max_iterations=6, generic=False, use_early_stop=True,
                          force_decoding=False, new_data=True, device=0):
    """The reference's pusch_decoder_impl whose pusch_codeblock_decoder runs the MI355X ldpc_decoder adapter
    (integration/ldpc_decoder_hip). rxbuf: an oracle.RefRxBuffer. Result as oracle.ref_pusch_decode."""
    llrs = np.ascontiguousarray(llrs, dtype=np.int8)
    res = np.zeros(6, np.float64)
    r = lib().srs_ref_hip_ldpc_pusch_decode(device, rxbuf.h, _p(llrs), llrs.size, _p(tb_out), tb_out.size,
                                            p["base_graph"], p["rv"], p["modulation_order"], p["Nref"],
                                            p["nof_layers"], max_iterations, int(force_decoding), int(use_early_stop),
                                            int(new_data), int(generic), _p(res))
    if r != 0:
        raise RuntimeError("pusch_decoder_impl did not notify")
    return bool(res[0]), int(res[1]), int(res[2]), int(round(res[3])), int(res[4]), int(res[5])

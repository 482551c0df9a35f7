"""TEST INFRASTRUCTURE: the MI355X channel-processor plug-ins (integration/pusch_processor_hip, libsrsran_amd_phy.so)
driven as the reference's upper PHY drives a pusch_processor (oracle/phy_harness.cpp in
oracle/_ref/libsrsran_ref_hw.so).  Loading it initialises the GPU on first use, so only GPU tests use it."""
import ctypes

import numpy as np

from srsran_project_amd.pdsch_modulator import RePattern

from . import hw as _hw

_declared = False


def lib():
    global _declared
    L = _hw.lib()
    if not _declared:
        P, u, i, d = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_double
        L.srs_ref_phy_pusch_create.restype = P
        L.srs_ref_phy_pusch_create.argtypes = [i, u, u, i, i, u]
        L.srs_ref_phy_pusch_destroy.argtypes = [P]
        L.srs_ref_phy_pusch_sibling.restype = P
        L.srs_ref_phy_pusch_sibling.argtypes = [P]
        L.srs_ref_phy_grid_create.restype = P
        L.srs_ref_phy_grid_create.argtypes = [P, u, u]
        L.srs_ref_phy_grid_destroy.argtypes = [P]
        L.srs_ref_phy_pusch_process.restype = i
        L.srs_ref_phy_pusch_process.argtypes = [P, P, P, P, P, u]
        L.srs_ref_phy_pusch_flush.argtypes = [P]
        L.srs_ref_phy_pusch_wait.argtypes = [P]
        L.srs_ref_phy_pusch_result.restype = i
        L.srs_ref_phy_pusch_result.argtypes = [P, i, P, P, P, P, P, P]
        L.srs_ref_phy_pusch_stats.argtypes = [P, P]
        L.srs_ref_phy_pusch_bench.restype = d
        L.srs_ref_phy_pusch_bench.argtypes = [P, P, u, u, P, u, u, P, u, P]
        L.srs_ref_phy_hgrid_create.restype = P
        L.srs_ref_phy_hgrid_create.argtypes = [P, u, u, i]
        L.srs_ref_phy_hgrid_set_device.restype = i
        L.srs_ref_phy_hgrid_set_device.argtypes = [P, P]
        L.srs_ref_phy_hgrid_read.argtypes = [P, P, P]
        L.srs_ref_phy_hgrid_transfers.argtypes = [P, P]
        L.srs_ref_fapi_pusch_convert.restype = P
        L.srs_ref_fapi_pusch_convert.argtypes = [P, P, P]
        L.srs_ref_fapi_pusch_params.argtypes = [P, P]
        L.srs_ref_fapi_pusch_free.argtypes = [P]
        L.srs_ref_phy_pusch_process_fapi.restype = i
        L.srs_ref_phy_pusch_process_fapi.argtypes = [P, P, P, P, P, u]
        L.srs_ref_pusch_process_fapi.restype = i
        L.srs_ref_pusch_process_fapi.argtypes = [P, P, u, u, P, P, u, P, P, P, P, P]
        L.srs_ref_phy_ofdm_demodulate.restype = i
        L.srs_ref_phy_ofdm_demodulate.argtypes = [P, i, i, u, u, u, d, ctypes.c_float, u, u, P]
        L.srs_ref_phy_ofdm_symbol_bench.restype = d
        L.srs_ref_phy_ofdm_symbol_bench.argtypes = [i, i, i, u, u, u, u, u, u, P, P, P]
        L.srs_ref_phy_ofdm_modulate_twice.restype = i
        L.srs_ref_phy_ofdm_modulate_twice.argtypes = [P, i, u, u, u, d, ctypes.c_float, u, u, P, i, P, P]
        L.srs_ref_phy_ofdm_modulate.restype = i
        L.srs_ref_phy_ofdm_modulate.argtypes = [P, i, i, u, u, u, d, ctypes.c_float, u, u, P]
        _declared = True
    return L


class FapiPusch(ctypes.Structure):
    """srs_ref_fapi_pusch (phy_harness.cpp): a flat FAPI UL_TTI.request PUSCH PDU (fapi::ul_pusch_pdu subset)."""

    _fields_ = [(n, ctypes.c_uint32) for n in ("rnti", "bwp_start", "bwp_size", "numerology", "sfn", "slot")] + \
        [("qm", ctypes.c_int32)] + \
        [(n, ctypes.c_uint32) for n in (
            "target_code_rate", "transform_precoding", "nid_pusch", "num_layers", "ul_dmrs_symb_pos", "dmrs_type",
            "scrambling_id", "dmrs_identity", "nscid", "num_dmrs_cdm_grps_no_data", "rb_start", "rb_size",
            "start_symbol_index", "nr_of_symbols", "tx_direct_current_location", "has_data", "rv_index",
            "harq_process_id", "new_data", "tb_size", "ldpc_base_graph", "tb_size_lbrm_bytes", "has_uci",
            "harq_ack_bit_length", "csi_part1_bit_length", "alpha_scaling", "beta_offset_harq_ack",
            "beta_offset_csi1", "beta_offset_csi2", "num_rx_ant")]


class FapiPuschPdu:
    """A FAPI PUSCH PDU converted by the reference's convert_pusch_fapi_to_phy into the PHY's pusch_pdu
    (lib/fapi_adaptor/phy/messages/pusch.cpp).  dc_position: the converted pdu_t::dc_position (None: unset);
    tb_bytes: the transport block size; params: target_code_rate, alpha, beta HARQ-ACK / CSI1 / CSI2 as floats."""

    def __init__(self, **kw):
        L = lib()
        self.fapi = FapiPusch(**kw)
        dc, tbb = ctypes.c_int(), ctypes.c_uint()
        self.h = L.srs_ref_fapi_pusch_convert(ctypes.byref(self.fapi), ctypes.byref(dc), ctypes.byref(tbb))
        self.dc_position = None if dc.value < 0 else dc.value
        self.tb_bytes = tbb.value
        out = np.zeros(5, np.float32)
        L.srs_ref_fapi_pusch_params(self.h, out.ctypes.data)
        self.params = dict(target_code_rate=float(out[0]), alpha_scaling=float(out[1]),
                           beta_offset_harq_ack=float(out[2]), beta_offset_csi_part1=float(out[3]),
                           beta_offset_csi_part2=float(out[4]))

    def __del__(self):
        if getattr(self, "h", None):
            lib().srs_ref_fapi_pusch_free(self.h)
            self.h = None


def ref_pusch_process_fapi(grid, fpdu, nof_prb=273, iterations=6, rx_buffer=None):
    """The reference's pusch_processor_impl on a converted FAPI PDU: (tb, result dict as PuschProcessorPlugin.result).
    A PDU with data gets a fresh HARQ buffer when none is given (the reference's decoder needs a valid rx_buffer)."""
    if rx_buffer is None and fpdu.tb_bytes:
        from . import RefRxBuffer

        b = 8 * fpdu.tb_bytes + (24 if 8 * fpdu.tb_bytes > 3824 else 16)
        m = 8448 if fpdu.fapi.ldpc_base_graph == 1 else 3840
        rx_buffer = RefRxBuffer(1 if b <= m else -(-b // (m - 24)))
    tb = np.zeros(max(fpdu.tb_bytes, 1), np.uint8)
    res, csi, uci = np.zeros(6, np.float64), np.zeros(5, np.float64), np.zeros(5, np.int32)
    ack = np.zeros(max(fpdu.fapi.harq_ack_bit_length, 1), np.uint8)
    c1 = np.zeros(max(fpdu.fapi.csi_part1_bit_length, 1), np.uint8)
    r = lib().srs_ref_pusch_process_fapi(grid.h, fpdu.h, nof_prb, iterations, None if rx_buffer is None else
                                        rx_buffer.h, tb.ctypes.data, fpdu.tb_bytes, res.ctypes.data, csi.ctypes.data,
                                        uci.ctypes.data, ack.ctypes.data, c1.ctypes.data)
    if r != 0:
        raise RuntimeError("reference pusch_processor_impl did not notify")
    return tb[:fpdu.tb_bytes], _result_dict(res, csi, uci, ack[:fpdu.fapi.harq_ack_bit_length],
                                            c1[:fpdu.fapi.csi_part1_bit_length], np.zeros(0, np.uint8))


def _result_dict(res, csi, uci, ack, c1, c2):
    obs = int(res[2])  # an empty statistic (a failed or UCI-only transmission) has a NaN mean
    return dict(tb_crc_ok=bool(res[0]), nof_codeblocks_total=int(res[1]), nof_observations=obs,
                iterations_sum=int(round(res[3])) if obs else 0, iterations_min=int(res[4]) if obs else 0,
                iterations_max=int(res[5]) if obs else 0,
                sinr_db=csi[0], epre_db=csi[1], rsrp_db=csi[2], time_alignment_s=csi[3], cfo_hz=csi[4],
                nof_uci=int(uci[0]), harq_ack_status=int(uci[1]), csi_part1_status=int(uci[2]),
                csi_part2_status=int(uci[3]), harq_ack=ack, csi_part1=c1, csi_part2=c2)


class DeviceGrid:
    """A device-resident grid (integration/hip_resource_grid: hip_resource_grid over the reference's
    resource_grid_impl) of uint32 [P][14][nsubc]; usable wherever Grid / WriterGrid are.  grid: initial contents
    through the host writer; device=True: written into the DEVICE copy instead (as the OFDM demodulator plug-in
    would), leaving the host mirror stale."""

    def __init__(self, grid=None, shape=None, device=False, hip_device=0):
        L = lib()
        if grid is not None:
            g = np.ascontiguousarray(grid, np.uint32)
            shape = g.shape
        self.shape = tuple(shape)
        self.h = L.srs_ref_phy_hgrid_create(None if (grid is None or device) else g.ctypes.data, self.shape[0],
                                            self.shape[2], hip_device)
        if grid is not None and device and L.srs_ref_phy_hgrid_set_device(self.h, g.ctypes.data) != 0:
            raise RuntimeError("device grid write failed")

    def read(self):
        out = np.zeros(self.shape, np.uint32)
        lib().srs_ref_phy_hgrid_read(self.h, out.ctypes.data, None)
        return out

    def transfers(self):
        t = np.zeros(2, np.uint64)
        lib().srs_ref_phy_hgrid_transfers(self.h, t.ctypes.data)
        return dict(downloads=int(t[0]), uploads=int(t[1]))

    def __del__(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_grid_destroy(self.h)
            self.h = None


class Grid:
    """A received grid uint32 [P][14][nsubc] behind the reference's resource_grid_reader_impl."""

    def __init__(self, grid):
        g = np.ascontiguousarray(grid, np.uint32)
        self.shape = g.shape
        self.h = lib().srs_ref_phy_grid_create(g.ctypes.data, g.shape[0], g.shape[2])

    def __del__(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_grid_destroy(self.h)
            self.h = None


class PuschProcessorPlugin:
    """pusch_processor_factory_hip + one of its pusch_processors (sibling=True: another processor of the same
    factory, i.e. another cell sharing the slot collector)."""

    def __init__(self, device=0, nof_prb=273, iterations=6, mmse=False, generic=False, max_wait_us=0, sibling_of=None):
        if sibling_of is not None:
            self.h = lib().srs_ref_phy_pusch_sibling(sibling_of.h)
            self._base = sibling_of
        else:
            self.h = lib().srs_ref_phy_pusch_create(device, nof_prb, iterations, int(mmse), int(generic), max_wait_us)
        if not self.h:
            raise RuntimeError("pusch_processor_factory_hip creation failed")
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_pusch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdu, tb_bytes, rx_buffer=None):
        """pusch_processor::process (asynchronous): returns (ticket, transport-block buffer)."""
        tb = np.zeros(tb_bytes, np.uint8)
        self._keep.append((tb, pdu, grid))
        t = lib().srs_ref_phy_pusch_process(self.h, grid.h, ctypes.byref(pdu), None if rx_buffer is None
                                            else rx_buffer.h, tb.ctypes.data, tb_bytes)
        return t, tb

    def flush(self):
        lib().srs_ref_phy_pusch_flush(self.h)

    def wait(self):
        lib().srs_ref_phy_pusch_wait(self.h)

    def result(self, ticket, nof_harq_ack=0, nof_csi_part1=0, max_csi2=4096):
        """None until notified; then a dict shaped as oracle.pusch_proc.ref_pusch_process's."""
        res = np.zeros(6, np.float64)
        csi = np.zeros(5, np.float64)
        uci = np.zeros(5, np.int32)
        ack = np.zeros(max(nof_harq_ack, 1), np.uint8)
        c1 = np.zeros(max(nof_csi_part1, 1), np.uint8)
        c2 = np.zeros(max_csi2, np.uint8)
        r = lib().srs_ref_phy_pusch_result(self.h, ticket, res.ctypes.data, csi.ctypes.data, uci.ctypes.data,
                                           ack.ctypes.data, c1.ctypes.data, c2.ctypes.data)
        if r <= 0:
            return None
        return _result_dict(res, csi, uci, ack[:nof_harq_ack], c1[:nof_csi_part1], c2[:int(uci[4])])

    def process_fapi(self, grid, fpdu, rx_buffer=None):
        """pusch_processor::process of a converted FAPI PDU (FapiPuschPdu): (ticket, transport-block buffer)."""
        tb = np.zeros(max(fpdu.tb_bytes, 1), np.uint8)
        self._keep.append((tb, fpdu, grid))
        t = lib().srs_ref_phy_pusch_process_fapi(self.h, grid.h, fpdu.h, None if rx_buffer is None else rx_buffer.h,
                                                 tb.ctypes.data, fpdu.tb_bytes)
        return t, tb[:fpdu.tb_bytes]

    def stats(self):
        s = np.zeros(14, np.uint64)
        lib().srs_ref_phy_pusch_stats(self.h, s.ctypes.data)
        return dict(zip(("pdus", "batches", "errors", "harq_redecodes", "retransmissions", "device_grids",
                         "harq_soft_downloads", "stage_us", "set_wait_us", "wait_us", "notify_us", "stage_reads_us",
                         "stage_call_us", "stage_download_us"),
                        (int(v) for v in s)))

    def bench(self, grids, pdu, tb_bytes, warmup, steps, depth=1):
        """Seconds per step with one PDU per cell grid (process per PDU, flush; depth 1: wait for every notification
        each step; depth d: d slots in flight, grids = d sets of the cells' grids) and the TB CRC-OK count."""
        cells = len(grids) // depth
        arr = (ctypes.c_void_p * len(grids))(*[g.h for g in grids])
        tbs = np.zeros(cells * tb_bytes, np.uint8)
        ok = ctypes.c_uint()
        dt = lib().srs_ref_phy_pusch_bench(self.h, arr, cells, depth, ctypes.byref(pdu), warmup, steps,
                                           tbs.ctypes.data, tb_bytes, ctypes.byref(ok))
        return dt, ok.value, tbs.reshape(cells, tb_bytes)


# ---- OFDM demodulator plug-ins on a device-resident grid ----

def ofdm_demodulate(grid, samples, slot, numerology, bw_rb, dft_size, fc, scale=1.0, form=1, device=0):
    """The uplink lower-PHY step (puxch_processor_impl.cpp:73-82) through the MI355X OFDM demodulator plug-in:
    samples complex64 [P][slot size] of slot `slot` of the subframe demodulated into grid (DeviceGrid: written in
    place on the device) port by port, symbol by symbol (form 1, ofdm_symbol_demodulator) or slot by slot (form 0)."""
    x = np.ascontiguousarray(samples, np.complex64)
    if lib().srs_ref_phy_ofdm_demodulate(grid.h, device, form, numerology, bw_rb, dft_size, fc, scale, slot, x.shape[0],
                                         x.ctypes.data) != 0:
        raise RuntimeError("OFDM demodulator plug-in refused the configuration")


def ofdm_modulate(grid, nports, slot, numerology, bw_rb, dft_size, fc, scale, n, form=1, device=0):
    """The downlink lower-PHY step through the MI355X OFDM modulator plug-in: every port of slot `slot` of grid
    (DeviceGrid: read in place on the device) modulated symbol by symbol (form 1) or slot by slot (form 0); returns
    complex64 [nports][n] (n: the slot size)."""
    y = np.zeros((nports, n), np.complex64)
    if lib().srs_ref_phy_ofdm_modulate(grid.h, device, form, numerology, bw_rb, dft_size, fc, scale, slot, nports,
                                       y.ctypes.data) != 0:
        raise RuntimeError("OFDM modulator plug-in refused the configuration")
    return y


def ofdm_modulate_twice(grid, nports, slot, numerology, bw_rb, dft_size, fc, scale, n, nxt, next_on_host, device=0):
    """srs_ref_phy_ofdm_modulate_twice: one symbol modulator plug-in over `grid`, then over `nxt` (uint32 [P][14][nsubc]
    written on the device or through the host writer); returns the two complex64 [nports][n] outputs."""
    y0, y1 = np.zeros((nports, n), np.complex64), np.zeros((nports, n), np.complex64)
    g = np.ascontiguousarray(nxt, np.uint32)
    if lib().srs_ref_phy_ofdm_modulate_twice(grid.h, device, numerology, bw_rb, dft_size, fc, scale, slot, nports,
                                             g.ctypes.data, int(next_on_host), y0.ctypes.data, y1.ctypes.data) != 0:
        raise RuntimeError("OFDM modulator plug-in refused the configuration")
    return y0, y1


def ofdm_symbol_bench(plugin, threads, numerology, bw_rb, dft_size, samples, slots, modulate=False, grid=None,
                      device=0):
    """Symbol-form demodulation (modulate=True: modulation of `grid` uint32 [P][14][nsubc]) from `threads` sector
    threads (srs_ref_phy_ofdm_symbol_bench): plugin 1 the MI355X plug-in on device-resident grids, 0 the reference's
    ofdm_symbol_(de)modulator_impl.  samples complex64 [P][slot size] (slot 0).  Returns (seconds, mean host us per
    call, grid transfers)."""
    x = np.ascontiguousarray(samples, np.complex64)
    g = None if grid is None else np.ascontiguousarray(grid, np.uint32)
    out = np.zeros(2, np.float64)
    dt = lib().srs_ref_phy_ofdm_symbol_bench(device, plugin, int(modulate), threads, numerology, bw_rb, dft_size,
                                             x.shape[0], slots, x.ctypes.data, None if g is None else g.ctypes.data,
                                             out.ctypes.data)
    if dt < 0:
        raise RuntimeError("OFDM symbol bench failed")
    return dt, float(out[0]), int(out[1])


# ---- PDSCH ----

class PdschPdu(ctypes.Structure):
    """srs_ref_pdsch_pdu (phy_harness.cpp): a flat pdsch_processor::pdu_t."""

    _fields_ = [(n, ctypes.c_uint32) for n in ("numerology", "slot_index", "rnti", "bwp_start_rb", "bwp_size_rb")] + \
        [("qm", ctypes.c_int32)] + \
        [(n, ctypes.c_uint32) for n in ("rv", "n_id", "ref_point", "dmrs_symbol_mask", "dmrs_type", "scrambling_id",
                                        "n_scid", "nof_cdm_groups_without_data")] + \
        [("vrb_mask", ctypes.c_uint8 * 35), ("pad", ctypes.c_uint8)] + \
        [(n, ctypes.c_uint32) for n in ("start_symbol_index", "nof_symbols", "base_graph", "tbs_lbrm_bytes")] + \
        [("ratio_pdsch_dmrs_to_sss_dB", ctypes.c_float), ("ratio_pdsch_data_to_sss_dB", ctypes.c_float),
         ("nof_layers", ctypes.c_uint32), ("nof_ports", ctypes.c_uint32), ("weights", ctypes.c_float * 32),
         ("nof_reserved", ctypes.c_uint32), ("reserved", RePattern * 8)] + \
        [(n, ctypes.c_uint32) for n in ("has_ptrs", "ptrs_freq_density", "ptrs_time_density", "ptrs_re_offset")] + \
        [("ratio_ptrs_to_pdsch_data_dB", ctypes.c_float), ("nof_prg", ctypes.c_uint32), ("prg_size", ctypes.c_uint32),
         ("prg_weights", ctypes.c_float * (7 * 32))]


def make_pdsch_pdu(vrbs, weights, reserved=(), ptrs=None, prg=None, **kw):
    """vrbs: the BWP-relative VRB indices; weights complex [L][P] (PRG 0); reserved: [(crb bool mask, re_mask,
    symbols)]; ptrs: (frequency density, time density, RE offset, PT-RS to data ratio dB); prg: (PRG size in PRBs,
    [weights complex [L][P] of PRG 1, 2, ..])."""
    p = PdschPdu()
    d = dict(numerology=1, slot_index=0, rnti=1, bwp_start_rb=0, bwp_size_rb=273, qm=2, rv=0, n_id=0, ref_point=0,
             dmrs_symbol_mask=(1 << 2) | (1 << 11), dmrs_type=1, scrambling_id=0, n_scid=0,
             nof_cdm_groups_without_data=2, start_symbol_index=0, nof_symbols=14, base_graph=1, tbs_lbrm_bytes=0,
             ratio_pdsch_dmrs_to_sss_dB=0.0, ratio_pdsch_data_to_sss_dB=0.0)
    d.update(kw)
    for k, v in d.items():
        setattr(p, k, v)
    for i in vrbs:
        p.vrb_mask[int(i) // 8] |= 1 << (int(i) % 8)
    W = np.asarray(weights, np.complex64)
    p.nof_layers, p.nof_ports = W.shape
    for l in range(W.shape[0]):
        for q in range(W.shape[1]):
            p.weights[(l * 4 + q) * 2] = float(W[l, q].real)
            p.weights[(l * 4 + q) * 2 + 1] = float(W[l, q].imag)
    if ptrs is not None:
        p.has_ptrs = 1
        p.ptrs_freq_density, p.ptrs_time_density, p.ptrs_re_offset = (int(v) for v in ptrs[:3])
        p.ratio_ptrs_to_pdsch_data_dB = float(ptrs[3])
    if prg is not None:
        p.prg_size, extra = int(prg[0]), prg[1]
        p.nof_prg = 1 + len(extra)
        for g, Wg in enumerate(extra):
            Wg = np.asarray(Wg, np.complex64)
            for l in range(Wg.shape[0]):
                for q in range(Wg.shape[1]):
                    p.prg_weights[((g * 4 + l) * 4 + q) * 2] = float(Wg[l, q].real)
                    p.prg_weights[((g * 4 + l) * 4 + q) * 2 + 1] = float(Wg[l, q].imag)
    p.nof_reserved = len(reserved)
    for r, (cm, rm, sm) in enumerate(reserved):
        cm = np.asarray(cm, bool)
        for i in np.flatnonzero(cm):
            p.reserved[r].crb_mask[i // 8] |= 1 << (i % 8)
        p.reserved[r].re_mask = rm
        p.reserved[r].symbols = sm
    return p


def _declare_pdsch(L):
    P, u, i, d = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_double
    L.srs_ref_phy_wgrid_create.restype = P
    L.srs_ref_phy_wgrid_create.argtypes = [P, u, u]
    L.srs_ref_phy_wgrid_destroy.argtypes = [P]
    L.srs_ref_phy_wgrid_read.argtypes = [P, P]
    L.srs_ref_pdsch_process.restype = i
    L.srs_ref_pdsch_process.argtypes = [P, P, P, u]
    L.srs_ref_phy_pdsch_create.restype = P
    L.srs_ref_phy_pdsch_create.argtypes = [i, u, u]
    L.srs_ref_phy_pdsch_destroy.argtypes = [P]
    L.srs_ref_phy_pdsch_process.restype = i
    L.srs_ref_phy_pdsch_process.argtypes = [P, P, P, P, u]
    L.srs_ref_phy_pdsch_flush.argtypes = [P]
    L.srs_ref_phy_pdsch_wait.argtypes = [P]
    L.srs_ref_phy_pdsch_done.restype = i
    L.srs_ref_phy_pdsch_done.argtypes = [P, i]
    L.srs_ref_phy_pdsch_stats.argtypes = [P, P]
    L.srs_ref_phy_pdsch_bench.restype = d
    L.srs_ref_phy_pdsch_bench.argtypes = [P, P, u, u, P, P, u, u, u]


_pdsch_declared = False


def _L():
    global _pdsch_declared
    L = lib()
    if not _pdsch_declared:
        _declare_pdsch(L)
        _pdsch_declared = True
    return L


class WriterGrid:
    """A slot grid uint32 [P][14][nsubc] behind the reference's resource_grid_writer_impl."""

    def __init__(self, grid):
        g = np.ascontiguousarray(grid, np.uint32)
        self.shape = g.shape
        self.h = _L().srs_ref_phy_wgrid_create(g.ctypes.data, g.shape[0], g.shape[2])

    def read(self):
        out = np.zeros(self.shape, np.uint32)
        _L().srs_ref_phy_wgrid_read(self.h, out.ctypes.data)
        return out

    def __del__(self):
        if getattr(self, "h", None):
            _L().srs_ref_phy_wgrid_destroy(self.h)
            self.h = None


def ref_pdsch_process(grid, pdu, tb):
    """The reference's pdsch_processor_impl (auto components) of one PDU into the WriterGrid."""
    tb = np.ascontiguousarray(tb, np.uint8)
    if _L().srs_ref_pdsch_process(grid.h, ctypes.byref(pdu), tb.ctypes.data, tb.size) != 0:
        raise RuntimeError("pdsch_processor_impl did not notify")


class PdschProcessorPlugin:
    """pdsch_processor_factory_hip + one of its pdsch_processors."""

    def __init__(self, device=0, nof_prb=273, max_wait_us=0):
        self.h = _L().srs_ref_phy_pdsch_create(device, nof_prb, max_wait_us)
        if not self.h:
            raise RuntimeError("pdsch_processor_factory_hip creation failed")

    def close(self):
        if getattr(self, "h", None):
            _L().srs_ref_phy_pdsch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdu, tb):
        tb = np.ascontiguousarray(tb, np.uint8)
        return _L().srs_ref_phy_pdsch_process(self.h, grid.h, ctypes.byref(pdu), tb.ctypes.data, tb.size)

    def flush(self):
        _L().srs_ref_phy_pdsch_flush(self.h)

    def wait(self):
        _L().srs_ref_phy_pdsch_wait(self.h)

    def done(self, ticket):
        return bool(_L().srs_ref_phy_pdsch_done(self.h, ticket))

    def stats(self):
        s = np.zeros(4, np.uint64)
        _L().srs_ref_phy_pdsch_stats(self.h, s.ctypes.data)
        return dict(zip(("pdus", "batches", "errors", "device_grids"), (int(v) for v in s)))

    def bench(self, grids, pdu, tb, warmup, steps, depth=1):
        """Seconds per step (depth: slots in flight, grids = depth sets of the cells' grids, as PuschProcessorPlugin)."""
        arr = (ctypes.c_void_p * len(grids))(*[g.h for g in grids])
        tb = np.ascontiguousarray(tb, np.uint8)
        return _L().srs_ref_phy_pdsch_bench(self.h, arr, len(grids) // depth, depth, ctypes.byref(pdu),
                                            tb.ctypes.data, tb.size, warmup, steps)


class PdcchProcessorPlugin:
    """pdcch_processor_factory_hip + one of its pdcch_processors and its validator (integration/
    pdcch_processor_hip), driven through the reference's pdcch_processor interface."""

    def __init__(self, device=0):
        L = lib()
        P, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        L.srs_ref_phy_pdcch_create.restype = P
        L.srs_ref_phy_pdcch_create.argtypes = [i]
        L.srs_ref_phy_pdcch_destroy.argtypes = [P]
        L.srs_ref_phy_pdcch_process.argtypes = [P, P, P, u]
        L.srs_ref_phy_pdcch_validate.restype = i
        L.srs_ref_phy_pdcch_validate.argtypes = [P, P, ctypes.c_char_p, u]
        L.srs_ref_phy_pdcch_stats.argtypes = [P, P]
        self.h = L.srs_ref_phy_pdcch_create(device)
        if not self.h:
            raise RuntimeError("pdcch_processor_factory_hip creation failed")

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_pdcch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdus):
        from srsran_project_amd.pdcch import PdcchPdu

        arr = (PdcchPdu * len(pdus))(*pdus)
        lib().srs_ref_phy_pdcch_process(self.h, grid.h, ctypes.addressof(arr), len(pdus))

    def validate(self, pdu):
        """None when valid, else the validator's message."""
        msg = ctypes.create_string_buffer(512)
        return None if lib().srs_ref_phy_pdcch_validate(self.h, ctypes.byref(pdu), msg, 512) else msg.value.decode()

    def stats(self):
        s = np.zeros(3, np.uint64)
        lib().srs_ref_phy_pdcch_stats(self.h, s.ctypes.data)
        return dict(zip(("pdus", "errors", "device_grids"), (int(v) for v in s)))


class SsbProcessorPlugin:
    """ssb_processor_factory_hip + one of its ssb_processors and its validator (integration/ssb_processor_hip),
    driven through the reference's ssb_processor interface."""

    def __init__(self, device=0):
        L = lib()
        P, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        L.srs_ref_phy_ssb_create.restype = P
        L.srs_ref_phy_ssb_create.argtypes = [i]
        L.srs_ref_phy_ssb_destroy.argtypes = [P]
        L.srs_ref_phy_ssb_process.argtypes = [P, P, P, u]
        L.srs_ref_phy_ssb_validate.restype = i
        L.srs_ref_phy_ssb_validate.argtypes = [P, P, ctypes.c_char_p, u]
        L.srs_ref_phy_ssb_stats.argtypes = [P, P]
        self.h = L.srs_ref_phy_ssb_create(device)
        if not self.h:
            raise RuntimeError("ssb_processor_factory_hip creation failed")

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_ssb_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, grid, pdus):
        from srsran_project_amd.ssb import SsbPdu

        arr = (SsbPdu * len(pdus))(*pdus)
        lib().srs_ref_phy_ssb_process(self.h, grid.h, ctypes.addressof(arr), len(pdus))

    def validate(self, pdu):
        """None when valid, else the validator's message."""
        msg = ctypes.create_string_buffer(512)
        return None if lib().srs_ref_phy_ssb_validate(self.h, ctypes.byref(pdu), msg, 512) else msg.value.decode()

    def stats(self):
        s = np.zeros(3, np.uint64)
        lib().srs_ref_phy_ssb_stats(self.h, s.ctypes.data)
        return dict(zip(("pdus", "errors", "device_grids"), (int(v) for v in s)))


class PucchProcessorPlugin:
    """pucch_processor_factory_hip + one of its pucch_processors and its validator (integration/pucch_processor_hip),
    driven through the reference's pucch_processor interface."""

    def __init__(self, device=0):
        L = lib()
        P, u, i = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int
        L.srs_ref_phy_pucch_create.restype = P
        L.srs_ref_phy_pucch_create.argtypes = [i]
        L.srs_ref_phy_pucch_destroy.argtypes = [P]
        L.srs_ref_phy_pucch_f0.argtypes = [P, P, P, u, P]
        L.srs_ref_phy_pucch_f1.argtypes = [P, P, P, u, P]
        L.srs_ref_phy_pucch_f2.argtypes = [P, P, P, P, P]
        L.srs_ref_phy_pucch_f34.argtypes = [P, P, P, P, P]
        L.srs_ref_phy_pucch_latency.restype = ctypes.c_double
        L.srs_ref_phy_pucch_latency.argtypes = [P, P, P, P, u, u]
        L.srs_ref_phy_pucch_f2_validate.restype = i
        L.srs_ref_phy_pucch_f2_validate.argtypes = [P, P, ctypes.c_char_p, u]
        L.srs_ref_phy_pucch_stats.argtypes = [P, P]
        L.srs_ref_phy_pucch_mt_bench.restype = ctypes.c_double
        L.srs_ref_phy_pucch_mt_bench.argtypes = [P, P, u, P, u, P, u, P, u, P, u, u, u, u, P, P, P, P, P, P]
        self.h = L.srs_ref_phy_pucch_create(device)
        if not self.h:
            raise RuntimeError("pucch_processor_factory_hip creation failed")

    def close(self):
        if getattr(self, "h", None):
            lib().srs_ref_phy_pucch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def f0(self, grid, pdu, grid_prb):
        from srsran_project_amd.pucch import PucchResult

        r = PucchResult()
        lib().srs_ref_phy_pucch_f0(self.h, grid.h, ctypes.byref(pdu), grid_prb, ctypes.byref(r))
        return r

    def f1(self, grid, batch, grid_prb):
        from srsran_project_amd.pucch import PucchResult

        out = (PucchResult * batch.nof_entries)()
        lib().srs_ref_phy_pucch_f1(self.h, grid.h, ctypes.byref(batch), grid_prb, out)
        return list(out)

    def f2(self, grid, pdu):
        from srsran_project_amd.pucch import PucchUciResult, payload_bits

        r = PucchUciResult()
        pay = np.zeros(max(payload_bits(pdu), 1), np.uint8)
        lib().srs_ref_phy_pucch_f2(self.h, grid.h, ctypes.byref(pdu), ctypes.byref(r), pay.ctypes.data)
        return r, pay[:payload_bits(pdu)]

    def f34(self, grid, pdu):
        from srsran_project_amd.pucch import PucchUciResult, payload_bits

        r = PucchUciResult()
        pay = np.zeros(max(payload_bits(pdu), 1), np.uint8)
        lib().srs_ref_phy_pucch_f34(self.h, grid.h, ctypes.byref(pdu), ctypes.byref(r), pay.ctypes.data)
        return r, pay[:payload_bits(pdu)]

    def latency_us(self, grid, pdu0=None, pdu2=None, grid_prb=0, reps=200):
        """Mean microseconds per pucch_processor::process call (Format 0 or Format 2 PDU)."""
        t = lib().srs_ref_phy_pucch_latency(self.h, grid.h, None if pdu0 is None else ctypes.byref(pdu0),
                                            None if pdu2 is None else ctypes.byref(pdu2), grid_prb, reps)
        return t * 1e6 / reps

    def validate_f2(self, pdu):
        msg = ctypes.create_string_buffer(512)
        return None if lib().srs_ref_phy_pucch_f2_validate(self.h, ctypes.byref(pdu), msg, 512) else msg.value.decode()

    def stats(self):
        out = (ctypes.c_uint64 * 6)()
        lib().srs_ref_phy_pucch_stats(self.h, out)
        return dict(pdus=out[0], errors=out[1], device_grids=out[2], batches=out[3], batch_host_us=out[4],
                    batch_wait_us=out[5])

    def mt_bench(self, grids, f0, f1, f2, f34, threads, reps, grid_prb):
        """srs_ref_phy_pucch_mt_bench: every cell's PDUs (same lists per grid) over `threads` executor threads, `reps`
        times.  Returns (seconds, outputs of the first rep as raw byte arrays: r0, r1, r2, p2, r34, p34)."""
        from srsran_project_amd import pucch as pu

        n = len(grids)
        arr = (ctypes.c_void_p * n)(*[g.h for g in grids])
        a0, a1 = (pu.PucchF0Pdu * max(len(f0), 1))(*f0), (pu.PucchF1Batch * max(len(f1), 1))(*f1)
        a2, a34 = (pu.PucchF2Pdu * max(len(f2), 1))(*f2), (pu.PucchF34Pdu * max(len(f34), 1))(*f34)
        ne = sum(b.nof_entries for b in f1)
        rs, us = ctypes.sizeof(pu.PucchResult), ctypes.sizeof(pu.PucchUciResult)
        r0 = np.zeros(max(n * len(f0) * rs, 1), np.uint8)
        r1 = np.zeros(max(n * ne * rs, 1), np.uint8)
        r2, p2 = np.zeros(max(n * len(f2) * us, 1), np.uint8), np.zeros(max(n * len(f2) * 64, 1), np.uint8)
        r34, p34 = np.zeros(max(n * len(f34) * us, 1), np.uint8), np.zeros(max(n * len(f34) * 64, 1), np.uint8)
        dt = lib().srs_ref_phy_pucch_mt_bench(self.h, arr, n, a0, len(f0), a1, len(f1), a2, len(f2), a34, len(f34),
                                              threads, reps, grid_prb, r0.ctypes.data, r1.ctypes.data,
                                              r2.ctypes.data, p2.ctypes.data, r34.ctypes.data, p34.ctypes.data)
        if dt < 0:
            raise RuntimeError("PUCCH processor creation failed")
        return dt, (r0, r1, r2, p2, r34, p34)

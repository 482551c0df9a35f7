"""TEST INFRASTRUCTURE: the MI355X channel-processor plug-ins (integration/pusch_processor_hip, libsrsran_amd_phy.so)
driven as the reference's upper PHY drives a pusch_processor (oracle/phy_harness.cpp in
oracle/_ref/libsrsran_ref_hw.so).  Loading it initialises the GPU on first use, so only GPU tests use it."""
import ctypes

import numpy as np

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
        L.srs_ref_phy_pusch_bench.argtypes = [P, P, u, P, u, u, P, u, P]
        _declared = True
    return L


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
        obs = int(res[2])  # an empty statistic (a failed transmission) has a NaN mean
        return dict(tb_crc_ok=bool(res[0]), nof_codeblocks_total=int(res[1]), nof_observations=obs,
                    iterations_sum=int(round(res[3])) if obs else 0, iterations_min=int(res[4]) if obs else 0,
                    iterations_max=int(res[5]) if obs else 0,
                    sinr_db=csi[0], epre_db=csi[1], rsrp_db=csi[2], time_alignment_s=csi[3], cfo_hz=csi[4],
                    nof_uci=int(uci[0]), harq_ack_status=int(uci[1]), csi_part1_status=int(uci[2]),
                    csi_part2_status=int(uci[3]), harq_ack=ack[:nof_harq_ack], csi_part1=c1[:nof_csi_part1],
                    csi_part2=c2[:int(uci[4])])

    def stats(self):
        s = np.zeros(5, np.uint64)
        lib().srs_ref_phy_pusch_stats(self.h, s.ctypes.data)
        return dict(zip(("pdus", "batches", "errors", "harq_redecodes", "retransmissions"), (int(v) for v in s)))

    def bench(self, grids, pdu, tb_bytes, warmup, steps):
        """Seconds per step with one PDU per cell grid (process per PDU, flush, wait) and the TB CRC-OK count."""
        arr = (ctypes.c_void_p * len(grids))(*[g.h for g in grids])
        tbs = np.zeros(len(grids) * tb_bytes, np.uint8)
        ok = ctypes.c_uint()
        dt = lib().srs_ref_phy_pusch_bench(self.h, arr, len(grids), ctypes.byref(pdu), warmup, steps,
                                           tbs.ctypes.data, tb_bytes, ctypes.byref(ok))
        return dt, ok.value, tbs.reshape(len(grids), tb_bytes)

"""Live kernel probes (include/srsran_amd/profiling.h): per-launch device time of one kernel family inside a
caller's own launch sequence, from HIP events recorded on each launch's stream around the launch."""
import ctypes

from . import _lib

PROBE_LDPC_HR, PROBE_LDPC_FULL, PROBE_EQUALIZER, PROBE_OFDM_DEMOD, PROBE_OFDM_MOD = range(5)
NAMES = {PROBE_LDPC_HR: "ldpc_decode_hr_kernel", PROBE_LDPC_FULL: "ldpc_decode_hr_kernel (full length)",
         PROBE_EQUALIZER: "pusch_equalize_fused_kernel", PROBE_OFDM_DEMOD: "ofdm_demodulate_kernel",
         PROBE_OFDM_MOD: "ofdm_modulate_kernel"}

_declared = False


def _L():
    global _declared
    lib = _lib.lib()
    if not _declared:
        lib.srs_amd_probe_arm.restype = ctypes.c_int
        lib.srs_amd_probe_arm.argtypes = [ctypes.c_int, ctypes.c_uint32]
        lib.srs_amd_probe_read.restype = ctypes.c_int
        lib.srs_amd_probe_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)] + \
            [ctypes.POINTER(ctypes.c_double)] * 3
        _declared = True
    return lib


def arm(probe, max_launches=4096):
    _lib.check(_L().srs_amd_probe_arm(int(probe), int(max_launches)), "probe arm")


def read(probe):
    """(launches, mean ms, min ms, max ms) of the launches recorded since arm(); disarms."""
    n = ctypes.c_uint32()
    tot, lo, hi = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    _lib.check(_L().srs_amd_probe_read(int(probe), ctypes.byref(n), ctypes.byref(tot), ctypes.byref(lo),
                                       ctypes.byref(hi)), "probe read")
    return n.value, (tot.value / n.value if n.value else None), lo.value, hi.value

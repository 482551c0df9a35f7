"""ctypes binding of the C-ABI library ``lib/libsrsran_amd.so`` (include/srsran_amd/*.h).

The HIP library is the product: there is no CPU fallback.  Loading fails
loudly when the shared object has not been built (``make -C srsran_project_amd``
or ``__graft_entry__.build()``).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRSRAN_AMD_LIB") or os.path.join(_HERE, "lib", "libsrsran_amd.so")

SRS_AMD_OK = 0
SRS_AMD_EINVAL = -1
SRS_AMD_EHIP = -2
SRS_AMD_ENOMEM = -3

_lock = threading.Lock()
_lib = None


class LDPCDecoderConfig(ctypes.Structure):
    """``srs_amd_ldpc_decoder_config`` (include/srsran_amd/ldpc.h)."""

    _fields_ = [
        ("base_graph", ctypes.c_uint32),
        ("lifting_size", ctypes.c_uint32),
        ("nof_filler_bits", ctypes.c_uint32),
        ("nof_crc_bits", ctypes.c_uint32),
        ("max_iterations", ctypes.c_uint32),
    ]


class CodeblockMetadata(ctypes.Structure):
    """``srs_amd_codeblock_metadata`` (include/srsran_amd/ldpc.h)."""

    _fields_ = [
        ("base_graph", ctypes.c_uint32),
        ("lifting_size", ctypes.c_uint32),
        ("rv", ctypes.c_uint32),
        ("modulation_order", ctypes.c_uint32),
        ("Nref", ctypes.c_uint32),
        ("nof_filler_bits", ctypes.c_uint32),
    ]


class LDPCEncoderConfig(ctypes.Structure):
    """``srs_amd_ldpc_encoder_config`` (include/srsran_amd/ldpc_encoder.h)."""

    _fields_ = [
        ("base_graph", ctypes.c_uint32),
        ("lifting_size", ctypes.c_uint32),
        ("Nref", ctypes.c_uint32),
    ]


class SrsAmdError(RuntimeError):
    pass


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    sigs = {
        "srs_amd_last_error": (c.c_char_p, []),
        "srs_amd_version": (c.c_char_p, []),
        "srs_amd_ldpc_decoder_create": (c.c_int, [c.POINTER(P), c.c_int, c.c_int, c.c_int]),
        "srs_amd_ldpc_decoder_destroy": (None, [P]),
        "srs_amd_ldpc_decoder_set_max_slots": (c.c_int, [P, c.c_uint32]),
        "srs_amd_ldpc_decode": (
            c.c_int,
            [P, P, P, c.c_uint32, c.c_int, c.POINTER(LDPCDecoderConfig), c.POINTER(c.c_int32)],
        ),
        "srs_amd_ldpc_decode_batch": (
            c.c_int,
            [P, c.POINTER(LDPCDecoderConfig), c.c_int, P, c.c_uint32, P, c.c_uint32, P, c.c_uint32, P, P,
             c.c_uint32, P],
        ),
        "srs_amd_ldpc_encoder_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_ldpc_encoder_destroy": (None, [P]),
        "srs_amd_ldpc_encode": (c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.POINTER(LDPCEncoderConfig)]),
        "srs_amd_ldpc_encode_batch": (
            c.c_int, [P, c.POINTER(LDPCEncoderConfig), P, c.c_uint32, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_ldpc_rate_matcher_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_ldpc_rate_matcher_destroy": (None, [P]),
        "srs_amd_ldpc_rate_match": (c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.POINTER(CodeblockMetadata)]),
        "srs_amd_ldpc_rate_match_batch": (
            c.c_int, [P, c.POINTER(CodeblockMetadata), P, c.c_uint32, P, P, c.c_uint32, P, c.c_uint32, P]),
        "srs_amd_ldpc_rate_dematcher_create": (c.c_int, [c.POINTER(P), c.c_int]),
        "srs_amd_ldpc_rate_dematcher_destroy": (None, [P]),
        "srs_amd_ldpc_rate_dematch": (
            c.c_int, [P, P, c.c_uint32, P, c.c_uint32, c.c_int, c.POINTER(CodeblockMetadata)]),
        "srs_amd_ldpc_rate_dematch_batch": (
            c.c_int, [P, c.POINTER(CodeblockMetadata), c.c_int, P, P, P, P, c.c_uint32, c.c_uint32, P]),
        "srs_amd_ldpc_message_length": (c.c_uint32, [c.c_uint32, c.c_uint32]),
        "srs_amd_ldpc_codeblock_length": (c.c_uint32, [c.c_uint32, c.c_uint32]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def lib():
    """Returns the loaded C-ABI library, raising if it is missing."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    "srsran_project_amd HIP library not built: %s is missing "
                    "(run `make -C srsran_project_amd` or __graft_entry__.build())" % LIB_PATH
                )
            # PyTorch-ROCm ships its own libamdhip64.so.7; when torch is present,
            # load it first so that this library binds to the same (single) HIP
            # runtime instead of pulling /opt/rocm's copy in beside it.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            _lib = _declare(ctypes.CDLL(LIB_PATH))
        return _lib


def check(rc, what=""):
    if rc != SRS_AMD_OK:
        msg = lib().srs_amd_last_error().decode()
        if rc == SRS_AMD_EINVAL:
            raise ValueError("%s: %s" % (what, msg) if what else msg)
        raise SrsAmdError("%s failed (%d): %s" % (what, rc, msg))
    return rc

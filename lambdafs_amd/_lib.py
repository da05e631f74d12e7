"""ctypes binding of libhrs.so (include/hrs.h) — the product's only compute path.

There is no CPU fallback: if the HIP library is missing, or no GPU is
visible, every coding call raises. (The CPU oracle lives in oracle/ and is
test infrastructure only.)
"""
import ctypes
import os

try:  # share torch's HIP runtime when torch is present (one libamdhip64 per process)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HRS_LIB") or os.path.join(_HERE, "libhrs.so")  # HRS_LIB: A/B runs of another build
# HBM ceiling probes: a side library for bench.py and tools, not the product
PROBE_LIB_PATH = os.path.join(_HERE, "libhrs_probe.so")

HRS_OK = 0
HRS_EINVAL = 1
HRS_ETOOMANY = 2
HRS_EDEVICE = 3
HRS_ENOMEM = 4
HRS_EALIGN = 5

HRS_CODE_RS = 0
HRS_CODE_XOR = 1
HRS_CODE_NRS = 2
HRS_CODE_SRC = 3

# Every entry point declared in include/hrs.h (checked by tests/test_abi.py:
# libhrs.so exports exactly these).
EXPORTS = (
    "hrs_create", "hrs_create_code", "hrs_create_src", "hrs_src_layout", "hrs_code_kind", "hrs_destroy",
    "hrs_last_error", "hrs_version", "hrs_locations_to_read_list",
    "hrs_stripe_size", "hrs_parity_size", "hrs_symbol_size",
    "hrs_locations_to_read", "hrs_encode_matrix", "hrs_decode_matrix",
    "hrs_encode", "hrs_decode", "hrs_decode3", "hrs_encode_crc", "hrs_decode_crc",
    "hrs_encode_dev", "hrs_decode_dev", "hrs_decode_batch_dev", "hrs_apply_dev", "hrs_crc32_dev",
    "hrs_encode_crc_dev", "hrs_decode_crc_dev", "hrs_decode_batch_host", "hrs_encode_batch_host",
    "hrs_encode_submit", "hrs_decode_submit", "hrs_collect", "hrs_pending", "hrs_ticket_shape",
    "hrs_set_kernel_mode", "hrs_last_kernel", "hrs_wait", "hrs_release",
    "hrs_device_count", "hrs_codec_device", "hrs_decode_batch_host_multi", "hrs_encode_batch_host_multi",
    "hrs_set_timing", "hrs_ticket_gpu_ms", "hrs_last_host_path",
)
# include/hrs_probe.h, exported by libhrs_probe.so
PROBE_EXPORTS = ("hrs_probe_stream", "hrs_probe_rows")


class HrsError(IOError):
    """A nonzero hrs_status (the JNI shim maps this to java.io.IOException)."""

    def __init__(self, status, msg):
        super().__init__(f"hrs status {status}: {msg}")
        self.status = status


class HipOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("reserved", ctypes.c_int * 7)]


_lib = None


def lib():
    """Load libhrs.so; raise loudly if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP engine first (make, or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    I, S, P = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    IP = ctypes.POINTER(ctypes.c_int)
    PP = ctypes.POINTER(ctypes.c_void_p)
    U8P = ctypes.c_void_p
    sigs = {
        "hrs_create": ([I, I, ctypes.POINTER(HipOpts), ctypes.POINTER(P)], I),
        "hrs_create_code": ([I, I, I, ctypes.POINTER(HipOpts), ctypes.POINTER(P)], I),
        "hrs_create_src": ([I, I, I, ctypes.POINTER(HipOpts), ctypes.POINTER(P)], I),
        "hrs_src_layout": ([P, IP, IP, IP], I),
        "hrs_code_kind": ([P], I),
        "hrs_destroy": ([P], None),
        "hrs_last_error": ([P], ctypes.c_char_p),
        "hrs_version": ([], ctypes.c_char_p),
        "hrs_stripe_size": ([P], I),
        "hrs_parity_size": ([P], I),
        "hrs_symbol_size": ([P], I),
        "hrs_locations_to_read": ([P, IP, I, IP], I),
        "hrs_locations_to_read_list": ([P, IP, I, IP, IP], I),
        "hrs_encode_matrix": ([P, U8P], I),
        "hrs_decode_matrix": ([P, IP, I, IP, I, I, U8P], I),
        "hrs_encode": ([P, PP, PP, S], I),
        "hrs_decode": ([P, PP, PP, IP, I, IP, I, IP, I, S], I),
        "hrs_decode3": ([P, PP, PP, IP, I, S], I),
        "hrs_encode_crc": ([P, PP, PP, S, P, P], I),
        "hrs_decode_crc": ([P, PP, PP, IP, I, IP, I, IP, I, S, P, P], I),
        "hrs_encode_dev": ([P, PP, S, PP, S, S, S, P], I),
        "hrs_decode_dev": ([P, PP, S, PP, S, IP, I, IP, I, S, S, P], I),
        "hrs_decode_batch_dev": ([P, P, S, S, P, I, P, S, S, S, S, P], I),
        "hrs_apply_dev": ([P, U8P, I, I, PP, S, PP, S, S, S, P], I),
        "hrs_crc32_dev": ([P, PP, I, S, S, S, P, P, P], I),
        "hrs_encode_crc_dev": ([P, PP, S, PP, S, S, S, P, P, P], I),
        "hrs_decode_crc_dev": ([P, PP, S, PP, S, IP, I, IP, I, S, S, P, P, P], I),
        "hrs_decode_batch_host": ([P, P, S, S, P, I, P, S, S, S, S], I),
        "hrs_encode_batch_host": ([P, P, S, S, S, S], I),
        "hrs_decode_batch_host_multi": ([PP, I, P, S, S, P, I, P, S, S, S, S], I),
        "hrs_encode_batch_host_multi": ([PP, I, P, S, S, S, S], I),
        "hrs_device_count": ([], I),
        "hrs_set_timing": ([P, I], I),
        "hrs_ticket_gpu_ms": ([P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float)], I),
        "hrs_codec_device": ([P], I),
        "hrs_encode_submit": ([P, PP, S, I, ctypes.POINTER(ctypes.c_uint64)], I),
        "hrs_decode_submit": ([P, PP, IP, I, IP, I, IP, I, S, I, ctypes.POINTER(ctypes.c_uint64)], I),
        "hrs_collect": ([P, ctypes.c_uint64, PP, P], I),
        "hrs_pending": ([P], I),
        "hrs_wait": ([P, ctypes.c_uint64], I),
        "hrs_release": ([P, ctypes.c_uint64], I),
        "hrs_ticket_shape": ([P, ctypes.c_uint64, IP, ctypes.POINTER(ctypes.c_size_t), IP], I),
        "hrs_set_kernel_mode": ([P, I], I),
        "hrs_last_kernel": ([P], ctypes.c_char_p),
        "hrs_last_host_path": ([P], ctypes.c_char_p),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


_probe = None


def probe_lib():
    """Load libhrs_probe.so (include/hrs_probe.h: the HBM ceiling probes
    bench.py quotes beside the kernels)."""
    global _probe
    if _probe is not None:
        return _probe
    if not os.path.exists(PROBE_LIB_PATH):
        raise ImportError(f"{PROBE_LIB_PATH} is missing: build it first (make)")
    L = ctypes.CDLL(PROBE_LIB_PATH)
    I, S, P = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    L.hrs_probe_stream.argtypes = [I, P, P, S, I, I, I, I, I, P]
    L.hrs_probe_stream.restype = I
    L.hrs_probe_rows.argtypes = [P, S, I, S, I, I, I, I, P]
    L.hrs_probe_rows.restype = I
    _probe = L
    return L


def check(status, handle=None):
    if status != HRS_OK:
        msg = lib().hrs_last_error(handle).decode(errors="replace")
        if status == HRS_ETOOMANY:
            from .erasure_code import TooManyErasedLocations
            raise TooManyErasedLocations(msg)
        raise HrsError(status, msg)


def int_array(values):
    values = [int(v) for v in values]
    return (ctypes.c_int * max(1, len(values)))(*values)


def ptr_array(ptrs):
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr

"""ctypes binding of libsymphony_hip.so (the C ABI in include/symphony_hip.h).

This is the same binding a cgo shim makes.  There is no fallback:
if the HIP library has not been built, importing the codec raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SYMHIP_LIBRARY names another build of the same ABI (tools/ use the tuning library, make tuning);
# the product path, the tests and bench.py load the default.
LIB_PATH = os.environ.get("SYMHIP_LIBRARY") or os.path.join(HERE, "lib", "libsymphony_hip.so")
CSRC = os.path.join(HERE, "csrc")

SYM_OK = 0
SYM_ERR_INVALID = -1
SYM_ERR_HIP = -2
SYM_ERR_NOMEM = -3
SYM_ERR_CAPACITY = -4
SYM_ERR_DEVICE = -5

# every symbol include/symphony_hip.h declares, with its ctypes signature
_u8p = ctypes.c_void_p
_u64p = ctypes.c_void_p
_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_int = ctypes.c_int
_ctx = ctypes.c_void_p

SIGNATURES = {
    "sym_abi_version": (_int, []),
    "sym_last_error": (ctypes.c_char_p, []),
    "sym_ctx_create": (_int, [_int, ctypes.POINTER(ctypes.c_void_p)]),
    "sym_ctx_destroy": (_int, [_ctx]),
    "sym_ctx_reserve": (_int, [_ctx, _u64]),
    "sym_ctx_check": (_int, [_ctx, _vp]),
    "sym_ctx_set_decode_impl": (_int, [_ctx, _int]),
    "sym_ctx_decode_redos": (_int, [_ctx, _vp, _u64p]),
    "sym_ctx_set_encode_impl": (_int, [_ctx, _int]),
    "sym_schema_info": (_int, [_int, ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "sym_record_overhead": (_u64, [_int]),
    "sym_encoded_size": (_u64, [_int, _u64, _u64]),
    "sym_encode": (_int, [_ctx, _int, _u64, _vp, _vp, _vp, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_decode": (_int, [_ctx, _int, _u64, _u8p, _u64p, _vp, _vp, _vp, _vp, _u8p, _vp]),
    "sym_encode_kv_set": (_int, [_ctx, _u8p, _u64p, _u8p, _u64p, _u64, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_encode_kv_get": (_int, [_ctx, _u8p, _u64p, _u64, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_encode_kv_response": (_int, [_ctx, _int, _u8p, _u64p, _u64, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_encode_echo": (_int, [_ctx, _vp, _vp, _u8p, _u64p, _u8p, _u64p, _u64, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_decode_kv_set": (_int, [_ctx, _u8p, _u64p, _u64, _u8p, _u64, _u64p, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_decode_kv_get": (_int, [_ctx, _u8p, _u64p, _u64, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_decode_kv_response": (_int, [_ctx, _int, _u8p, _u64p, _u64, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_decode_echo": (_int, [_ctx, _u8p, _u64p, _u64, _vp, _vp, _u8p, _u64, _u64p, _u8p, _u64, _u64p, _u8p,
                               _vp]),
    "sym_encoded_size_kv_mixed": (_u64, [_u64, _u64, _u64, _u64]),
    "sym_encode_kv_mixed": (_int, [_ctx, _u8p, _u8p, _u64p, _u8p, _u64p, _u64, _u32, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_decode_kv_mixed": (_int, [_ctx, _u8p, _u64p, _u8p, _u64, _u8p, _u64, _u64p, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_host_alloc": (_int, [_ctx, _u64, ctypes.POINTER(ctypes.c_void_p)]),
    "sym_host_free": (_int, [_ctx, _vp]),
    "sym_encode_host": (_int, [_ctx, _int, _u64, _vp, _vp, _vp, _u32, _u32, _u8p, _u64p]),
    "sym_decode_host": (_int, [_ctx, _int, _u64, _u8p, _u64p, _vp, _vp, _vp, _vp, _u8p]),
    "sym_fragment_plan": (_int, [_ctx, _u8p, _u64p, _u64, _u32, _u64p, _u64p, _u8p, _vp]),
    "sym_fragment_write": (_int, [_ctx, _u8p, _u64p, _u64, _u32, ctypes.c_uint8, _u64p, _vp, _u64p, _u64p, _u8p,
                                  _u8p, _u64p, _vp]),
    "sym_raw_get_fixed": (_int, [_ctx, _u8p, _u64p, _u64, _int, _u32, _u32, _vp, _u8p, _vp]),
    "sym_raw_get_bytes": (_int, [_ctx, _u8p, _u64p, _u64, _int, _u32, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_firewall_filter": (_int, [_ctx, _u8p, _u64p, _u64, _u32, ctypes.c_int32, _vp, _u8p, _u8p, _u64, _u64p,
                                   _u64p, _u64p, _vp]),
    "sym_reassemble": (_int, [_ctx, _u8p, _u64p, _u64, _u8p, _u64, _u64p, _u64p, _u64p, _u64p, _u8p, _vp]),
    "sym_flat_encoded_size": (_u64, [_vp, _int, _u64, _u64]),
    "sym_flat_encode": (_int, [_ctx, _vp, _int, _u64, _vp, _vp, _u32, _u32, _u8p, _u64p, _vp]),
    "sym_flat_decode": (_int, [_ctx, _vp, _int, _u64, _u8p, _u64p, _vp, _vp, _vp, _u8p, _vp]),
    "sym_flat_encoded_size_ex": (_u64, [_vp, _int, _u64, _vp, _vp]),
    "sym_flat_encode_ex": (_int, [_ctx, _vp, _int, _u64, _vp, _vp, _vp, _vp, _u8p, _u64p, _vp]),
    "sym_flat_decode_ex": (_int, [_ctx, _vp, _int, _u64, _u64p, _u8p, _u64p, _u64p, _u64p, _u64p, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _u8p, _u8p, _vp]),
    "sym_flat_nested_status": (_int, [_ctx, _vp, _int, _int, _vp, _u64, _u64p, _vp, _vp, _u8p, _u8p, _vp]),
    "sym_flat_list_sizes": (_int, [_ctx, _int, _u64, _u64p, _vp, _vp, _vp, _u64p, _vp]),
    "sym_raw_set": (_int, [_ctx, _vp, _int, _int, _u8p, _u64p, _u64, _vp, _u64p, _u8p, _u64, _u64p, _u8p, _vp]),
    "sym_batcher_create": (_int, [_int, _int, _u32, _u64, _u32, ctypes.POINTER(ctypes.c_void_p)]),
    "sym_batcher_destroy": (_int, [_vp]),
    "sym_batcher_encode_one": (_int, [_vp, _vp, _vp, _vp, _u32, _u32, _u8p, _u64, _u64p]),
    "sym_batcher_decode_one": (_int, [_vp, _u8p, _u64, _vp, _vp, _vp, _vp, _u8p]),
    "sym_batcher_stats": (_int, [_vp, _u64p, _u64p, _u64p, _u64p]),
    "sym_batcher_quiesce": (_int, [_vp]),
    "sym_encrypt": (_int, [_ctx, _u8p, _u64p, _u64, ctypes.c_char_p, ctypes.c_char_p, _u8p, _u8p, _u64p, _u8p, _vp]),
    "sym_decrypt": (_int, [_ctx, _u8p, _u64p, _u64, ctypes.c_char_p, ctypes.c_char_p, _u8p, _u64p, _u8p, _vp]),
}

SYM_DECODE_PIPELINE = 0
SYM_DECODE_THREE_KERNEL = 1
SYM_DECODE_LOOKBACK = 2
SYM_ENCODE_PIPELINE = 0
SYM_ENCODE_THREE_KERNEL = 1
SYM_ENCODE_LOOKBACK = 2

SYM_MAX_UDP_PAYLOAD = 1400
SYM_DATA_PACKET_HEADER = 31
SYM_PACKET_REQUEST = 1
SYM_PACKET_RESPONSE = 2
SYM_FRAG_OK = 0
SYM_FRAG_TOO_SHORT = 1
SYM_FRAG_BAD_OFFSET = 2
SYM_SEGMENT_PUBLIC = 0
SYM_SEGMENT_PRIVATE = 1
SYM_PUBLIC_TABLE_START = 13
SYM_PRIVATE_TABLE_START = 1
SYM_RAW_OK = 0
SYM_RAW_INVALID_BUFFER = 1
SYM_RAW_PUBLIC_ONLY = 2
SYM_VERDICT_PASS = 1
SYM_VERDICT_DROP = 2
SYM_RX_CONSUMED = 0
SYM_RX_PENDING = 1
SYM_RX_NOT_DATA = 2
SYM_RX_TOO_SHORT = 3
SYM_RX_BAD_LENGTH = 4
SYM_CRYPT_OK = 0
SYM_CRYPT_TOO_SHORT = 1
SYM_CRYPT_BAD_OFFSET = 2
SYM_CRYPT_AUTH_PUBLIC = 3
SYM_CRYPT_AUTH_PRIVATE = 4
SYM_CRYPT_BAD_VERSION = 5
SYM_GCM_OVERHEAD = 28


SYM_SET_OK = 0
SYM_SET_COMPLETE_BUFFER = 1
SYM_SET_INVALID_BUFFER = 2
SYM_SET_PUBLIC_ONLY = 3
SYM_SET_TOO_SHORT = 4
SYM_SET_UNMARSHAL = 5
SYM_SET_BOUNDS = 6
SYM_SET_BAD_LENGTH = 7

SYM_MAX_FLAT_FIELDS = 16
SYM_FIELD_REPEATED = 0x80
SYM_FIELD_MESSAGE = 0x40
SYM_FIELD_FRAMED = 0x20
SYM_STATUS_NESTED = 5


class SymField(ctypes.Structure):
    """struct sym_field (include/symphony_hip.h)."""
    _fields_ = [("segment", ctypes.c_uint8), ("width", ctypes.c_uint8)]


SYM_FRAME_PREFIX_MAX = 24


class FlatEncodeOpts(ctypes.Structure):
    """struct sym_flat_encode_opts (include/symphony_hip.h)."""
    _fields_ = [("service_id", ctypes.c_uint32), ("method_id", ctypes.c_uint32), ("framed", ctypes.c_uint32),
                ("frame_prefix_len", ctypes.c_uint32), ("frame_prefix", ctypes.c_uint8 * SYM_FRAME_PREFIX_MAX),
                ("string_bytes", ctypes.c_uint64), ("d_gate_rec", ctypes.c_void_p), ("gate_n", ctypes.c_uint64),
                ("gate_when_all", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Endpoints(ctypes.Structure):
    """struct sym_endpoints (include/symphony_hip.h)."""
    _fields_ = [("dst_ip", ctypes.c_uint8 * 4), ("dst_port", ctypes.c_uint16),
                ("src_ip", ctypes.c_uint8 * 4), ("src_port", ctypes.c_uint16)]

_lib = None


class SymphonyHipError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with code {code}: {last_error()}")
        self.code = code


def lib() -> ctypes.CDLL:
    """Load the HIP codec library; raises if it was never built (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"HIP Symphony codec not built ({LIB_PATH} missing); run `make -C {CSRC}` "
                "or `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.sym_abi_version() != 2:
            raise ImportError(f"unexpected ABI version {L.sym_abi_version()} in {LIB_PATH}")
        _lib = L
    return _lib


def last_error() -> str:
    if _lib is None:
        return ""
    msg = _lib.sym_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, what: str) -> None:
    if rc != SYM_OK:
        raise SymphonyHipError(rc, what)


def ptr_array(values) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def u64_array(values) -> ctypes.Array:
    arr = (ctypes.c_uint64 * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr

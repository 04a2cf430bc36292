"""ctypes wrapper around the CPU Symphony oracle (oracle/symphony_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product (arpc_amd) never
imports this module.

The functions take numpy arrays in the same columnar layout as the C-ABI in
include/symphony_hip.h: per var field a packed byte column plus a u64 offset
array of n+1 entries; per fixed field an int32 column.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_symphony.so")
_lib = None

STATUS_OK = 0
STATUS_TOO_SHORT = 1
STATUS_BAD_VERSION = 2
STATUS_NO_PRIVATE = 3
STATUS_FIELD_TOO_SHORT = 4


def build() -> str:
    """Compile the oracle with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in os.listdir(_HERE) if f.endswith(".c")]
        if not os.path.exists(_LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(_LIB_PATH) for s in srcs):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, i32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
        L.sym_oracle_record_size.restype = u64
        L.sym_oracle_record_size.argtypes = [i32, i32, vp]
        L.sym_oracle_marshal.restype = u64
        L.sym_oracle_marshal.argtypes = [i32, i32, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp]
        L.sym_oracle_unmarshal.restype = i32
        L.sym_oracle_unmarshal.argtypes = [i32, i32, vp, u64, vp, vp, vp]
        L.sym_oracle_encode_batch.restype = u64
        L.sym_oracle_encode_batch.argtypes = [i32, i32, u64, vp, vp, vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp]
        L.sym_oracle_decode_batch.restype = None
        L.sym_oracle_decode_batch.argtypes = [i32, i32, u64, vp, vp, vp, vp, vp, vp]
        u32 = ctypes.c_uint32
        L.sym_oracle_encode_kv_mixed.restype = u64
        L.sym_oracle_encode_kv_mixed.argtypes = [u64, vp, vp, vp, vp, vp, u32, u32, u32, vp, vp]
        L.sym_oracle_decode_kv_mixed.restype = None
        L.sym_oracle_decode_kv_mixed.argtypes = [u64, vp, vp, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _ptr_array(arrays) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(arrays)))()
    for i, a in enumerate(arrays):
        arr[i] = _ptr(a)
    return arr


# ---------------------------------------------------------------- single record
def marshal(fixed: list[int], fields: list[bytes], service_id: int = 0, method_id: int = 0) -> bytes:
    """One record, as the generated MarshalSymphony (+ client ID patch)."""
    nf, nv = len(fixed), len(fields)
    fx = np.array(fixed, dtype=np.int32)
    bufs = [np.frombuffer(f, dtype=np.uint8) if len(f) else np.zeros(1, np.uint8) for f in fields]
    lens = np.array([len(f) for f in fields], dtype=np.uint64)
    size = lib().sym_oracle_record_size(nf, nv, _ptr(lens))
    out = np.zeros(size, dtype=np.uint8)
    lib().sym_oracle_marshal(nf, nv, _ptr(fx), _ptr_array(bufs), _ptr(lens), service_id, method_id, _ptr(out))
    return out.tobytes()


def unmarshal(nfixed: int, nvar: int, data: bytes):
    """One record into a fresh struct -> (status, fixed values, var field bytes)."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    fx = np.zeros(max(1, nfixed), dtype=np.int32)
    pos = np.zeros(max(1, nvar), dtype=np.uint64)
    ln = np.zeros(max(1, nvar), dtype=np.uint64)
    st = lib().sym_oracle_unmarshal(nfixed, nvar, _ptr(buf), len(data), _ptr(fx), _ptr(pos), _ptr(ln))
    fields = [bytes(data[int(pos[f]):int(pos[f]) + int(ln[f])]) for f in range(nvar)]
    return st, [int(v) for v in fx[:nfixed]], fields


# ---------------------------------------------------------------- batches
def encode_batch(fixed_cols, var_cols, service_id: int = 0, method_id: int = 0):
    """fixed_cols: list of int32 arrays [n]; var_cols: list of (bytes u8 array, offs u64 array [n+1]).

    Returns (out u8 array, out_off u64 array [n+1])."""
    nf, nv = len(fixed_cols), len(var_cols)
    n = len(var_cols[0][1]) - 1 if nv else len(fixed_cols[0])
    fixed_cols = [np.ascontiguousarray(c, dtype=np.int32) for c in fixed_cols]
    vb = [np.ascontiguousarray(b, dtype=np.uint8) for b, _ in var_cols]
    vo = [np.ascontiguousarray(o, dtype=np.uint64) for _, o in var_cols]
    total = n * (14 + 4 * (nf + nv) + 4 * nv) + sum(int(o[-1] - o[0]) for o in vo)
    out = np.zeros(max(1, total), dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint64)
    got = lib().sym_oracle_encode_batch(nf, nv, n, _ptr_array(fixed_cols), _ptr_array(vb), _ptr_array(vo),
                                        service_id, method_id, _ptr(out), _ptr(out_off))
    assert got == total, (got, total)
    return out[:total], out_off


def decode_batch(nfixed: int, nvar: int, data: np.ndarray, rec_off: np.ndarray):
    """Returns (fixed_cols, [(bytes, offs)], status)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = len(rec_off) - 1
    cap = max(1, int(rec_off[-1] - rec_off[0]))
    fixed = [np.zeros(max(1, n), dtype=np.int32) for _ in range(nfixed)]
    cols = [np.zeros(cap, dtype=np.uint8) for _ in range(nvar)]
    offs = [np.zeros(n + 1, dtype=np.uint64) for _ in range(nvar)]
    status = np.zeros(max(1, n), dtype=np.uint8)
    lib().sym_oracle_decode_batch(nfixed, nvar, n, _ptr(data) if data.size else 0, _ptr(rec_off),
                                  _ptr_array(fixed), _ptr_array(cols), _ptr_array(offs), _ptr(status))
    return ([f[:n] for f in fixed], [(cols[i][:int(offs[i][-1])], offs[i]) for i in range(nvar)], status[:n])


def bench_echo(iters: int) -> tuple[float, float]:
    """ns per MarshalSymphony and per UnmarshalSymphony of config 1's echo record, one record per
    call with Go's allocation semantics (oracle/bench_oracle.c; testcases/simple/main.go:248-420)."""
    L = lib()
    if not getattr(L, "_bench_ready", False):
        L.sym_oracle_bench_echo.restype = ctypes.c_uint64
        L.sym_oracle_bench_echo.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]
        L._bench_ready = True
    m, u = ctypes.c_double(), ctypes.c_double()
    L.sym_oracle_bench_echo(iters, ctypes.byref(m), ctypes.byref(u))
    return m.value, u.value


class BatchBench:
    """A batch's encode + decode on one CPU thread into buffers allocated once (oracle/bench_oracle.c
    sym_oracle_bench_batch): run(reps) -> (encode seconds, decode seconds) per round."""

    def __init__(self, fixed_cols, var_cols):
        self.nf, self.nv = len(fixed_cols), len(var_cols)
        self.n = n = len(var_cols[0][1]) - 1 if self.nv else len(fixed_cols[0])
        self.fixed = [np.ascontiguousarray(c, dtype=np.int32) for c in fixed_cols]
        self.vb = [np.ascontiguousarray(b, dtype=np.uint8) for b, _ in var_cols]
        self.vo = [np.ascontiguousarray(o, dtype=np.uint64) for _, o in var_cols]
        var = sum(int(o[-1] - o[0]) for o in self.vo)
        self.total = n * (14 + 4 * (self.nf + self.nv) + 4 * self.nv) + var
        self.out = np.zeros(max(1, self.total), dtype=np.uint8)
        self.out_off = np.zeros(n + 1, dtype=np.uint64)
        self.dfixed = [np.zeros(max(1, n), dtype=np.int32) for _ in range(self.nf)]
        self.dbytes = [np.zeros(max(1, self.total), dtype=np.uint8) for _ in range(self.nv)]
        self.doffs = [np.zeros(n + 1, dtype=np.uint64) for _ in range(self.nv)]
        self.status = np.zeros(max(1, n), dtype=np.uint8)
        for a in [self.out, self.out_off, self.status] + self.dbytes + self.doffs:
            a.fill(0)  # first touch here, not in the timed rounds
        L = lib()
        if not getattr(L, "_bench_batch_ready", False):
            vp, pa = ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)
            dp = ctypes.POINTER(ctypes.c_double)
            L.sym_oracle_bench_batch.restype = ctypes.c_uint64
            L.sym_oracle_bench_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, pa, pa, pa, vp, vp, pa,
                                                 pa, pa, vp, ctypes.c_int, dp, dp]
            L._bench_batch_ready = True

    def run(self, reps: int):
        enc, dec = (ctypes.c_double * reps)(), (ctypes.c_double * reps)()
        size = lib().sym_oracle_bench_batch(
            self.nf, self.nv, self.n, _ptr_array(self.fixed), _ptr_array(self.vb), _ptr_array(self.vo),
            _ptr(self.out), _ptr(self.out_off), _ptr_array(self.dfixed), _ptr_array(self.dbytes),
            _ptr_array(self.doffs), _ptr(self.status), reps, enc, dec)
        assert size == self.total and not self.status[:self.n].any()
        return list(enc), list(dec)


# ---------------------------------------------------------------- mixed Get/Set batches
def encode_kv_mixed(rtype, key, val, service_id: int = 0, get_method_id: int = 0, set_method_id: int = 0):
    """rtype: u8 [n] (0 GetRequest, else SetRequest); key / val: (u8 bytes, u64 offs [n+1]).
    Returns (stream u8, rec_off u64 [n+1])."""
    rtype = np.ascontiguousarray(rtype, dtype=np.uint8)
    kb, ko = np.ascontiguousarray(key[0], dtype=np.uint8), np.ascontiguousarray(key[1], dtype=np.uint64)
    vb, vo = np.ascontiguousarray(val[0], dtype=np.uint8), np.ascontiguousarray(val[1], dtype=np.uint64)
    n = len(ko) - 1
    is_set = rtype[:n] != 0
    total = 22 * n + int(ko[-1] - ko[0]) + int((8 + np.diff(vo).astype(np.int64))[is_set].sum()) if n else 0
    out = np.zeros(max(1, total), dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint64)
    got = lib().sym_oracle_encode_kv_mixed(n, _ptr(rtype), _ptr(kb), _ptr(ko), _ptr(vb), _ptr(vo), service_id,
                                           get_method_id, set_method_id, _ptr(out), _ptr(off))
    assert got == total, (got, total)
    return out[:total], off


def decode_kv_mixed(data: np.ndarray, rec_off: np.ndarray, rtype: np.ndarray):
    """Returns ([(key bytes, key offs), (val bytes, val offs)], status)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    rtype = np.ascontiguousarray(rtype, dtype=np.uint8)
    n = len(rec_off) - 1
    cap = max(1, int(rec_off[-1] - rec_off[0]))
    cols = [np.zeros(cap, dtype=np.uint8) for _ in range(2)]
    offs = [np.zeros(n + 1, dtype=np.uint64) for _ in range(2)]
    status = np.zeros(max(1, n), dtype=np.uint8)
    lib().sym_oracle_decode_kv_mixed(n, _ptr(data) if data.size else 0, _ptr(rec_off), _ptr(rtype), _ptr(cols[0]),
                                     _ptr(offs[0]), _ptr(cols[1]), _ptr(offs[1]), _ptr(status))
    return [(cols[i][:int(offs[i][-1])], offs[i]) for i in range(2)], status[:n]


# ---------------------------------------------------------------- packetization (fragment_oracle.c)
FRAG_OK = 0
FRAG_TOO_SHORT = 1   # "data too short for offset header" (pkg/transport/symphony_fragmentation.go:33-35)
FRAG_BAD_OFFSET = 2  # "invalid offset" (:37-39)


def _frag_lib():
    L = lib()
    if not getattr(L, "_frag_ready", False):
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.sym_oracle_fragment_plan.restype = None
        L.sym_oracle_fragment_plan.argtypes = [u64, vp, vp, ctypes.c_uint32, vp, vp, vp]
        L.sym_oracle_fragment_write.restype = None
        L.sym_oracle_fragment_write.argtypes = [u64, vp, vp, ctypes.c_uint32, ctypes.c_uint8, vp, vp,
                                                ctypes.c_uint16, vp, ctypes.c_uint16, vp, vp, vp]
        L._frag_ready = True
    return L


def fragment_batch(data: np.ndarray, rec_off: np.ndarray, rpc_id: np.ndarray, packet_type: int = 1,
                   dst=(b"\x7f\x00\x00\x01", 9000), src=(b"\x7f\x00\x00\x01", 9001), max_udp_payload: int = 1400):
    """FragmentPackets + DataPacket serialization of every record, as aRPC's Send loop.

    Returns (wire u8 array, dg_off u64 [total_dg+1], first u64 [n+1], out_off u64 [n+1], status u8 [n])."""
    L = _frag_lib()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    rpc_id = np.ascontiguousarray(rpc_id, dtype=np.uint64)
    n = len(rec_off) - 1
    first = np.zeros(n + 1, np.uint64)
    out_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(max(1, n), np.uint8)
    dp = _ptr(data) if data.size else 0
    L.sym_oracle_fragment_plan(n, dp, _ptr(rec_off), max_udp_payload, _ptr(first), _ptr(out_off), _ptr(status))
    total_dg, total = int(first[n]), int(out_off[n])
    out = np.zeros(max(1, total), np.uint8)
    dg_off = np.zeros(total_dg + 1, np.uint64)
    longest = int(np.max(np.diff(rec_off))) if n else 0
    scratch = np.zeros(longest // max(1, max_udp_payload - 31) + 4, np.uint64)
    dip = np.frombuffer(bytes(dst[0]), np.uint8).copy()
    sip = np.frombuffer(bytes(src[0]), np.uint8).copy()
    L.sym_oracle_fragment_write(n, dp, _ptr(rec_off), max_udp_payload, packet_type, _ptr(rpc_id) if n else 0,
                                _ptr(dip), dst[1], _ptr(sip), src[1], _ptr(out), _ptr(dg_off), _ptr(scratch))
    return out[:total], dg_off, first, out_off, status[:n]


# ---------------------------------------------------------------- Raw getters / firewall (raw_oracle.c)
RAW_OK = 0
RAW_INVALID_BUFFER = 1  # private getter panic: "called on invalid buffer" (main.go:1003-1006)
RAW_PUBLIC_ONLY = 2     # private getter panic: "called on public-only buffer" (main.go:1007-1013)
VERDICT_PASS = 1        # cmd/proxy/util/packet.go:57-58
VERDICT_DROP = 2


def _raw_lib():
    L = lib()
    if not getattr(L, "_raw_ready", False):
        u64, u32, i32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        L.sym_oracle_raw_fixed.restype = None
        L.sym_oracle_raw_fixed.argtypes = [u64, vp, vp, i32, u32, u32, vp, vp]
        L.sym_oracle_raw_bytes.restype = None
        L.sym_oracle_raw_bytes.argtypes = [u64, vp, vp, i32, u32, vp, vp, vp]
        L.sym_oracle_firewall.restype = u64
        L.sym_oracle_firewall.argtypes = [u64, vp, vp, u32, ctypes.c_int32, vp, vp, vp, vp, vp]
        L.sym_oracle_marshal_element_batch.restype = u64
        L.sym_oracle_marshal_element_batch.argtypes = [u64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.sym_oracle_element_size.restype = u64
        L.sym_oracle_element_size.argtypes = [i32, u64, u64, u64]
        L._raw_ready = True
    return L


def _batch_args(data, rec_off):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    return data, rec_off, len(rec_off) - 1, (_ptr(data) if data.size else 0)


def raw_fixed(data, rec_off, table_off: int, width: int = 4, private: bool = False):
    """-> (values as uint8/uint32/uint64 [n], status u8 [n])."""
    data, rec_off, n, dp = _batch_args(data, rec_off)
    out = np.zeros(max(1, n), {1: np.uint8, 4: np.uint32, 8: np.uint64}[width])
    st = np.zeros(max(1, n), np.uint8)
    _raw_lib().sym_oracle_raw_fixed(n, dp, _ptr(rec_off), int(private), table_off, width, _ptr(out), _ptr(st))
    return out[:n], st[:n]


def raw_bytes(data, rec_off, table_off: int, private: bool = False):
    """-> (values u8, offsets u64 [n+1], status u8 [n])."""
    data, rec_off, n, dp = _batch_args(data, rec_off)
    out = np.zeros(max(1, data.size), np.uint8)
    offs = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(1, n), np.uint8)
    _raw_lib().sym_oracle_raw_bytes(n, dp, _ptr(rec_off), int(private), table_off, _ptr(out), _ptr(offs), _ptr(st))
    return out[:int(offs[n])], offs, st[:n]


def firewall(data, rec_off, block_threshold: int, score_table_off: int = 13):
    """-> (score i32 [n], verdict u8 [n], kept u8, kept_off u64 [nkept+1], kept_index u64 [nkept])."""
    data, rec_off, n, dp = _batch_args(data, rec_off)
    score = np.zeros(max(1, n), np.int32)
    verdict = np.zeros(max(1, n), np.uint8)
    kept = np.zeros(max(1, data.size), np.uint8)
    kept_off = np.zeros(n + 1, np.uint64)
    kept_index = np.zeros(max(1, n), np.uint64)
    k = _raw_lib().sym_oracle_firewall(n, dp, _ptr(rec_off), score_table_off, block_threshold, _ptr(score),
                                       _ptr(verdict), _ptr(kept), _ptr(kept_off), _ptr(kept_index))
    return score[:n], verdict[:n], kept[:int(kept_off[k])], kept_off[:k + 1], kept_index[:k]


def marshal_element_batch(score, strings):
    """Element-schema {Get,Set}Request records; strings = [(bytes, offs)] for Username, Key[, Value]."""
    L = _raw_lib()
    score = np.ascontiguousarray(score, dtype=np.int32)
    n, npriv = len(score), len(strings) - 1
    cols = [(np.ascontiguousarray(b, np.uint8), np.ascontiguousarray(o, np.uint64)) for b, o in strings]
    total = int(L.sym_oracle_element_size(npriv, 0, 0, 0)) * n + sum(int(o[-1] - o[0]) for _, o in cols)
    out = np.zeros(max(1, total), np.uint8)
    out_off = np.zeros(n + 1, np.uint64)
    val = cols[2] if npriv == 2 else (np.zeros(1, np.uint8), np.zeros(n + 1, np.uint64))
    got = L.sym_oracle_marshal_element_batch(n, npriv, _ptr(score), _ptr(cols[0][0]) or 0, _ptr(cols[0][1]),
                                             _ptr(cols[1][0]), _ptr(cols[1][1]), _ptr(val[0]), _ptr(val[1]),
                                             _ptr(out), _ptr(out_off))
    assert got == total, (got, total)
    return out[:total], out_off


# ---------------------------------------------------------------- reassembly (reassembly_oracle.c)
RX_CONSUMED = 0   # part of a returned message
RX_PENDING = 1    # still held by the reassembler after the batch
RX_NOT_DATA = 2   # not a Request / Response DataPacket
RX_TOO_SHORT = 3  # empty or shorter than the 31-byte header
RX_BAD_LENGTH = 4  # "data too short for declared payload length"


def reassemble(wire, dg_off):
    """DataReassembler over datagrams in arrival order ->
    (msg u8, msg_off u64 [nmsg+1], msg_rpc u64 [nmsg], msg_dg u64 [nmsg], status u8 [n])."""
    L = lib()
    if not getattr(L, "_rx_ready", False):
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.sym_oracle_reassemble.restype = u64
        L.sym_oracle_reassemble.argtypes = [u64, vp, vp, vp, vp, vp, vp, vp]
        L._rx_ready = True
    wire = np.ascontiguousarray(wire, dtype=np.uint8)
    dg_off = np.ascontiguousarray(dg_off, dtype=np.uint64)
    n = len(dg_off) - 1
    msg = np.zeros(max(1, wire.size), np.uint8)
    msg_off = np.zeros(n + 1, np.uint64)
    rpc = np.zeros(max(1, n), np.uint64)
    dg = np.zeros(max(1, n), np.uint64)
    st = np.zeros(max(1, n), np.uint8)
    k = L.sym_oracle_reassemble(n, _ptr(wire) if wire.size else 0, _ptr(dg_off), _ptr(msg), _ptr(msg_off), _ptr(rpc),
                                _ptr(dg), _ptr(st))
    return msg[:int(msg_off[k])], msg_off[:k + 1], rpc[:k], dg[:k], st[:n]


# ---------------------------------------------------------------- segment encryption (crypto_oracle.c)
CRYPT_OK = 0
CRYPT_TOO_SHORT = 1
CRYPT_BAD_OFFSET = 2
CRYPT_AUTH_PUBLIC = 3
CRYPT_AUTH_PRIVATE = 4
CRYPT_BAD_VERSION = 5
# pkg/transport/encryption.go:17-19
DEFAULT_PUBLIC_KEY = bytes.fromhex("27e1fa17d72b1faf722362deb1974a7675058db98843705124a074c61172f796")
DEFAULT_PRIVATE_KEY = bytes.fromhex("9b5300678420678a3157a4bcacdc3e864693971f8a3fab05b06913fb43c7ebf9")


def _crypto_lib():
    L = lib()
    if not getattr(L, "_crypto_ready", False):
        u64, vp = ctypes.c_uint64, ctypes.c_void_p
        L.sym_oracle_gcm_seal.restype = None
        L.sym_oracle_gcm_seal.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, u64, vp, vp]
        L.sym_oracle_encrypt_batch.restype = u64
        L.sym_oracle_encrypt_batch.argtypes = [u64, vp, vp, ctypes.c_char_p, ctypes.c_char_p, vp, vp, vp, vp]
        L.sym_oracle_decrypt_batch.restype = u64
        L.sym_oracle_decrypt_batch.argtypes = [u64, vp, vp, ctypes.c_char_p, ctypes.c_char_p, vp, vp, vp]
        L._crypto_ready = True
    return L


def gcm_seal(key: bytes, nonce: bytes, plaintext: bytes) -> tuple[bytes, bytes]:
    """AES-256-GCM seal with empty AAD -> (ciphertext, tag)."""
    p = np.frombuffer(plaintext, np.uint8).copy() if plaintext else np.zeros(1, np.uint8)
    c = np.zeros(max(1, len(plaintext)), np.uint8)
    t = np.zeros(16, np.uint8)
    _crypto_lib().sym_oracle_gcm_seal(key, nonce, _ptr(p), len(plaintext), _ptr(c), _ptr(t))
    return c[:len(plaintext)].tobytes(), t.tobytes()


def encrypt_batch(data, rec_off, nonces, pub_key=DEFAULT_PUBLIC_KEY, priv_key=DEFAULT_PRIVATE_KEY):
    """EncryptSymphonyData per record -> (out u8, out_off u64 [n+1], status u8 [n]); nonces: u8 [n, 24]."""
    data, rec_off, n, dp = _batch_args(data, rec_off)
    nonces = np.ascontiguousarray(nonces, dtype=np.uint8).reshape(-1)
    out = np.zeros(max(1, data.size + 56 * n), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(1, n), np.uint8)
    _crypto_lib().sym_oracle_encrypt_batch(n, dp, _ptr(rec_off), pub_key, priv_key, _ptr(nonces) if nonces.size else 0,
                                           _ptr(out), _ptr(off), _ptr(st))
    return out[:int(off[n])], off, st[:n]


def decrypt_batch(data, rec_off, pub_key=DEFAULT_PUBLIC_KEY, priv_key=DEFAULT_PRIVATE_KEY):
    """DecryptSymphonyData per record -> (out u8, out_off u64 [n+1], status u8 [n])."""
    data, rec_off, n, dp = _batch_args(data, rec_off)
    out = np.zeros(max(1, data.size), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(1, n), np.uint8)
    _crypto_lib().sym_oracle_decrypt_batch(n, dp, _ptr(rec_off), pub_key, priv_key, _ptr(out), _ptr(off), _ptr(st))
    return out[:int(off[n])], off, st[:n]


# ---------------------------------------------------------------- flat schemas (flat_oracle.c)
class _Field(ctypes.Structure):
    _fields_ = [("segment", ctypes.c_uint8), ("width", ctypes.c_uint8)]


REPEATED = 0x80  # or'ed into a field's width: repeated fixed-width field (payload: u32 count + elements)


def _flat_lib():
    L = lib()
    if not getattr(L, "_flat_ready", False):
        u64, u32, i32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        L.sym_oracle_flat_encode.restype = u64
        L.sym_oracle_flat_encode.argtypes = [i32, vp, u64, vp, vp, vp, u32, u32, vp, vp]
        L.sym_oracle_flat_decode.restype = None
        L.sym_oracle_flat_decode.argtypes = [i32, vp, u64, vp, vp, vp, vp, vp, vp]
        L._flat_ready = True
    return L


def _fields(fields):
    arr = (_Field * max(1, len(fields)))()
    for k, (seg, w) in enumerate(fields):
        arr[k].segment, arr[k].width = seg, w
    return arr


def flat_encode(fields, cols, n: int, service_id: int = 0, method_id: int = 0):
    """fields: [(segment 0/1, width 1/4/8 or 0 = string)]; cols[k]: numpy array of n values (fixed,
    any dtype of that width) or (bytes u8, offs u64 [n+1]) (string).  -> (out u8, out_off u64)."""
    L = _flat_lib()
    fx, vb, vo, keep = [], [], [], []
    total = (14 if not fields else 0) * n
    for (seg, w), c in zip(fields, cols):
        if w and not w & REPEATED:
            a = np.ascontiguousarray(c).view(np.uint8)
            keep.append(a)
            fx.append(_ptr(a)), vb.append(0), vo.append(0)
        else:
            b, o = np.ascontiguousarray(c[0], np.uint8), np.ascontiguousarray(c[1], np.uint64)
            keep += [b, o]
            fx.append(0), vb.append(_ptr(b)), vo.append(_ptr(o))
            total += int(o[-1] - o[0]) + 4 * n
    if fields:
        total += n * (13 + sum(4 if (not w or w & REPEATED) else w for _, w in fields) + 1)
    out = np.zeros(max(1, total), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    arr = lambda v: (ctypes.c_void_p * max(1, len(v)))(*v)
    f = _fields(fields)  # kept alive across the call
    got = L.sym_oracle_flat_encode(len(fields), ctypes.addressof(f), n, arr(fx), arr(vb), arr(vo), service_id,
                                   method_id, _ptr(out), _ptr(off))
    assert got == total, (got, total)
    return out[:total], off


def flat_decode(fields, data, rec_off):
    """-> (cols, status): cols[k] = u8 array [n, width] (fixed) or (bytes, offs [n+1]) (string)."""
    L = _flat_lib()
    data, rec_off, n, dp = _batch_args(data, rec_off)
    cap = max(1, data.size)
    outs, fx, vb, vo = [], [], [], []
    for seg, w in fields:
        if w and not w & REPEATED:
            a = np.zeros((max(1, n), w), np.uint8)
            outs.append(a)
            fx.append(_ptr(a)), vb.append(0), vo.append(0)
        else:
            b, o = np.zeros(cap, np.uint8), np.zeros(n + 1, np.uint64)
            outs.append((b, o))
            fx.append(0), vb.append(_ptr(b)), vo.append(_ptr(o))
    st = np.zeros(max(1, n), np.uint8)
    arr = lambda v: (ctypes.c_void_p * max(1, len(v)))(*v)
    f = _fields(fields)
    L.sym_oracle_flat_decode(len(fields), ctypes.addressof(f), n, dp, _ptr(rec_off), arr(fx), arr(vb), arr(vo),
                             _ptr(st))
    cols = [o[:n] if isinstance(o, np.ndarray) else (o[0][:int(o[1][n])], o[1]) for o in outs]
    return cols, st[:n]


(SET_OK, SET_COMPLETE_BUFFER, SET_INVALID_BUFFER, SET_PUBLIC_ONLY, SET_TOO_SHORT, SET_UNMARSHAL, SET_BOUNDS,
 SET_BAD_LENGTH) = range(8)


def raw_set_bound(fields, rec_off, val_bytes: int) -> int:
    """Output bytes that always suffice for a batched setter: (nv + 1) len + G per record + new bytes."""
    nv = sum(1 for _, w in fields if not w or w & REPEATED)
    g = 14 + sum(4 if (not w or w & REPEATED) else w for _, w in fields) + 4 * nv
    lens = np.diff(np.asarray(rec_off, np.uint64)).astype(np.int64)
    return int(((nv + 1) * lens + g).sum()) + int(val_bytes) + 16


def raw_set(fields, k: int, data, rec_off, values):
    """XxxRaw.Set<field k>(value i) on buffer i (flat_oracle.c sym_oracle_raw_set).  values: u8 array
    [n, width] (fixed field) or (bytes, offs [n+1]) (string / repeated: element bytes).
    -> (out u8, out_off u64 [n+1], status u8 [n])."""
    L = lib()
    if not getattr(L, "_set_ready", False):
        u64, i32, vp = ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p
        L.sym_oracle_raw_set.restype = u64
        L.sym_oracle_raw_set.argtypes = [i32, vp, i32, u64, vp, vp, vp, vp, vp, vp, vp]
        L._set_ready = True
    data, rec_off, n, dp = _batch_args(data, rec_off)
    seg, w = fields[k]
    if w and not w & REPEATED:
        vb = np.ascontiguousarray(values, np.uint8).reshape(-1)
        vo = None
        nbytes = vb.size
    else:
        vb, vo = np.ascontiguousarray(values[0], np.uint8), np.ascontiguousarray(values[1], np.uint64)
        nbytes = int(vo[-1] - vo[0])
    cap = raw_set_bound(fields, rec_off, nbytes)
    out = np.zeros(cap, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    st = np.zeros(max(1, n), np.uint8)
    f = _fields(fields)
    total = L.sym_oracle_raw_set(len(fields), ctypes.addressof(f), k, n, dp, _ptr(rec_off), _ptr(vb) if vb.size else 0,
                                 _ptr(vo) if vo is not None else 0, _ptr(out), _ptr(off), _ptr(st))
    return out[:total], off, st[:n]

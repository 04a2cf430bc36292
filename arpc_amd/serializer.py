"""Host-side mirror of aRPC's serializer plugin interface, backed by the HIP codec.

Reference (Go):
  type Serializer interface {                       pkg/serializer/serializer.go:3-6
      Marshal(msg any) ([]byte, error)
      Unmarshal(data []byte, out any) error
  }
  type SymphonyMessage interface {                  pkg/serializer/symphony.go:3-6
      MarshalSymphony() ([]byte, error)
      UnmarshalSymphony([]byte) error
  }
  SymphonySerializer.Marshal / Unmarshal            pkg/serializer/symphony.go:10-16

Same names, argument meaning and error behaviour:
  * marshal(msg) -> bytes; a message type the codec does not know raises TypeError
    (Go panics on the failed type assertion, symphony.go:11).
  * unmarshal(data, out) fills `out` in place like UnmarshalSymphony into a FRESH
    struct (every aRPC call site passes one: server.go:152's `dec` target and the
    client's resp), and raises SymphonyError carrying Go's exact error text.  As in
    Go, int32 fields read before the error keep their values (echo.syn.go:223-231);
    fields Go skips or never reaches come back zero / empty.
  * The serializer is stateless from the caller's view and safe to share across
    threads (one codec context per thread; pkg/serializer/symphony.go:8).

The reference is one record per call.  `marshal_batch` / `unmarshal_batch` are the
batched extension that the GPU is built for; the per-record methods run the same
kernels on a batch of one (through the C ABI's host entry points).
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass, fields

import numpy as np

from . import _native, schemas

ERROR_TEXT = {
    1: "invalid data: too short",
    2: "invalid data: wrong public version",
    3: "missing private segment",
    4: "invalid data: too short for field",
}


class SymphonyError(ValueError):
    """An UnmarshalSymphony error (Go `error` value) with its status code."""

    def __init__(self, status: int):
        super().__init__(ERROR_TEXT.get(status, f"status {status}"))
        self.status = status


def _b(v) -> bytes:
    return v.encode() if isinstance(v, str) else bytes(v)


# ----------------------------------------------------------------- message types
# Go structs of the generated code (string fields hold arbitrary bytes; Symphony does
# no UTF-8 check, kv.syn.go:725).  Field names follow the Go identifiers.
@dataclass
class GetRequest:
    Key: bytes = b""
    SCHEMA = schemas.KV_GET_REQUEST


@dataclass
class SetRequest:
    Key: bytes = b""
    Value: bytes = b""
    SCHEMA = schemas.KV_SET_REQUEST


@dataclass
class GetResponse:
    Value: bytes = b""
    SCHEMA = schemas.KV_GET_RESPONSE


@dataclass
class SetResponse:
    Value: bytes = b""
    SCHEMA = schemas.KV_SET_RESPONSE


@dataclass
class EchoRequest:
    Id: int = 0
    Score: int = 0
    Username: bytes = b""
    Content: bytes = b""
    SCHEMA = schemas.ECHO_REQUEST


@dataclass
class EchoResponse:
    Id: int = 0
    Score: int = 0
    Username: bytes = b""
    Content: bytes = b""
    SCHEMA = schemas.ECHO_RESPONSE


MESSAGE_TYPES = (GetRequest, SetRequest, GetResponse, SetResponse, EchoRequest, EchoResponse)


def _schema_of(msg) -> schemas.Schema:
    s = getattr(type(msg), "SCHEMA", None)
    if s is None:
        # Go: msg.(SymphonyMessage) panics for a non-Symphony type (symphony.go:11)
        raise TypeError(f"{type(msg).__name__} is not a SymphonyMessage")
    return s


def _i32(v: int) -> int:
    v = int(v) & 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


# ----------------------------------------------------------------- host staging
class _HostCodec(threading.local):
    """Per-thread C-ABI context for the host entry points (sym_encode_host / sym_decode_host)."""

    def __init__(self):
        self.ctx = None
        self.device = None

    def get(self, device: int):
        if self.ctx is None or self.device != device:
            L = _native.lib()
            h = ctypes.c_void_p()
            _native.check(L.sym_ctx_create(device, ctypes.byref(h)), "sym_ctx_create")
            self.ctx, self.device = h, device
        return self.ctx


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def encode_columns_host(ctx, s: schemas.Schema, fixed_cols, var_cols, service_id=0, method_id=0):
    """numpy columns -> (stream u8, offsets u64) via the HIP codec (H2D, kernel, D2H)."""
    L = _native.lib()
    n = len(var_cols[0][1]) - 1 if s.nvar else len(fixed_cols[0])
    fixed_cols = [np.ascontiguousarray(c, dtype=np.int32) for c in fixed_cols]
    vb = [np.ascontiguousarray(b, dtype=np.uint8) if len(b) else np.zeros(1, np.uint8) for b, _ in var_cols]
    vo = [np.ascontiguousarray(o, dtype=np.uint64) for _, o in var_cols]
    total = int(L.sym_encoded_size(s.schema_id, n, sum(int(o[-1] - o[0]) for o in vo)))
    out = np.empty(max(1, total), dtype=np.uint8)
    out_off = np.empty(n + 1, dtype=np.uint64)
    rc = L.sym_encode_host(ctx, s.schema_id, n, _native.ptr_array([_np_ptr(c) for c in fixed_cols]),
                           _native.ptr_array([_np_ptr(b) for b in vb]), _native.ptr_array([_np_ptr(o) for o in vo]),
                           service_id, method_id, _np_ptr(out), _np_ptr(out_off))
    _native.check(rc, f"sym_encode_host({s.name})")
    return out[:total], out_off


def decode_columns_host(ctx, s: schemas.Schema, data: np.ndarray, rec_off: np.ndarray):
    L = _native.lib()
    data = np.ascontiguousarray(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    rec_off = np.ascontiguousarray(rec_off, dtype=np.uint64)
    n = len(rec_off) - 1
    cap = int(rec_off[-1] - rec_off[0]) if n else 0
    fixed = [np.zeros(max(1, n), dtype=np.int32) for _ in range(s.nfixed)]
    cols = [np.empty(max(1, cap), dtype=np.uint8) for _ in range(s.nvar)]
    offs = [np.empty(n + 1, dtype=np.uint64) for _ in range(s.nvar)]
    status = np.empty(max(1, n), dtype=np.uint8)
    rc = L.sym_decode_host(ctx, s.schema_id, n, _np_ptr(data), _np_ptr(rec_off),
                           _native.ptr_array([_np_ptr(c) for c in fixed]), _native.ptr_array([_np_ptr(c) for c in cols]),
                           _native.u64_array([cap] * s.nvar), _native.ptr_array([_np_ptr(o) for o in offs]),
                           _np_ptr(status))
    _native.check(rc, f"sym_decode_host({s.name})")
    return [f[:n] for f in fixed], [(cols[i], offs[i]) for i in range(s.nvar)], status[:n]


# ----------------------------------------------------------------- the plugin
class SymphonySerializer:
    """GPU-backed drop-in for pkg/serializer.SymphonySerializer."""

    def __init__(self, device: int = 0, service_id: int = 0, method_id: int = 0):
        self.device = device
        # MarshalSymphony writes zeros into [5:13]; the client patches IDs afterwards
        # (client.go:267-271).  Nonzero IDs here produce the patched bytes directly.
        self.service_id = service_id
        self.method_id = method_id
        self._tls = _HostCodec()

    # --- pkg/serializer.Serializer -------------------------------------------------
    def marshal(self, msg) -> bytes:
        return self.marshal_batch([msg])[0]

    def unmarshal(self, data: bytes, out) -> None:
        err = self.unmarshal_batch([data], [out])[0]
        if err is not None:
            raise err

    # --- batched extension ---------------------------------------------------------
    def marshal_batch(self, msgs) -> list[bytes]:
        msgs = list(msgs)
        out: list = [None] * len(msgs)
        for s, idx in _group_by_schema(msgs).items():
            group = [msgs[i] for i in idx]
            fixed = [np.array([_i32(getattr(m, f)) for m in group], dtype=np.int32) for f in s.fixed_fields]
            var = []
            for f in s.var_fields:
                vals = [_b(getattr(m, f)) for m in group]
                offs = np.zeros(len(vals) + 1, dtype=np.uint64)
                np.cumsum([len(v) for v in vals], out=offs[1:])
                var.append((np.frombuffer(b"".join(vals), dtype=np.uint8), offs))
            data, off = encode_columns_host(self._tls.get(self.device), s, fixed, var, self.service_id,
                                            self.method_id)
            raw = data.tobytes()
            for k, i in enumerate(idx):
                out[i] = raw[int(off[k]):int(off[k + 1])]
        return out

    def unmarshal_batch(self, datas, outs) -> list:
        """Fills each out in place; returns per record None or the SymphonyError Go would return."""
        datas, outs = list(datas), list(outs)
        if len(datas) != len(outs):
            raise ValueError("datas and outs differ in length")
        errs: list = [None] * len(outs)
        for s, idx in _group_by_schema(outs).items():
            blobs = [bytes(datas[i]) for i in idx]
            rec_off = np.zeros(len(blobs) + 1, dtype=np.uint64)
            np.cumsum([len(b) for b in blobs], out=rec_off[1:])
            stream = np.frombuffer(b"".join(blobs), dtype=np.uint8)
            fixed, var, status = decode_columns_host(self._tls.get(self.device), s, stream, rec_off)
            for k, i in enumerate(idx):
                m = outs[i]
                for f, name in enumerate(s.fixed_fields):
                    setattr(m, name, int(fixed[f][k]))
                for f, name in enumerate(s.var_fields):
                    col, off = var[f]
                    setattr(m, name, col[int(off[k]):int(off[k + 1])].tobytes())
                if status[k]:
                    errs[i] = SymphonyError(int(status[k]))
        return errs


class BatchingSerializer:
    """The per-record drop-in for pkg/serializer.SymphonySerializer under concurrency: every
    marshal / unmarshal call is one record (as Go's Call goroutines make them, pkg/rpc/client.go:233-310,
    server.go:152 / :173), coalesced with the calls other threads make meanwhile into one device
    batch by the C ABI's batcher (sym_batcher_*, arpc_amd/csrc/batcher.cpp).  Same results and
    errors as SymphonySerializer, for records of any size: a record larger than the batcher's slot
    (max_bytes) goes through a SymphonySerializer of its own, as the reference's Serializer has no
    size limit.  Safe to share across threads (ctypes releases the GIL while a call waits for its
    batch)."""

    def __init__(self, device: int = 0, service_id: int = 0, method_id: int = 0, max_records: int = 4096,
                 max_bytes: int = 8 << 20, max_wait_us: int = 0):
        self.device, self.service_id, self.method_id = device, service_id, method_id
        self._cfg = (max_records, max_bytes, max_wait_us)
        self._batchers: dict = {}
        self._lock = threading.Lock()
        self._direct = SymphonySerializer(device, service_id, method_id)  # records over max_bytes

    def _batcher(self, s: schemas.Schema):
        b = self._batchers.get(s.schema_id)
        if b is None:
            with self._lock:
                b = self._batchers.get(s.schema_id)
                if b is None:
                    h = ctypes.c_void_p()
                    _native.check(_native.lib().sym_batcher_create(self.device, s.schema_id, *self._cfg,
                                                                   ctypes.byref(h)), "sym_batcher_create")
                    b = self._batchers[s.schema_id] = h
        return b

    def marshal(self, msg) -> bytes:
        s = _schema_of(msg)
        vals = [_b(getattr(msg, f)) for f in s.var_fields]
        fixed = (ctypes.c_int32 * max(1, s.nfixed))(*[_i32(getattr(msg, f)) for f in s.fixed_fields])
        bufs = [ctypes.create_string_buffer(v, max(1, len(v))) for v in vals]
        ptrs = (ctypes.c_void_p * max(1, s.nvar))(*[ctypes.addressof(b) for b in bufs])
        lens = (ctypes.c_uint64 * max(1, s.nvar))(*[len(v) for v in vals])
        size = s.overhead + sum(len(v) for v in vals)
        if size > self._cfg[1]:
            return self._direct.marshal(msg)
        out = ctypes.create_string_buffer(max(1, size))
        n = ctypes.c_uint64()
        _native.check(_native.lib().sym_batcher_encode_one(self._batcher(s), fixed, ptrs, lens, self.service_id,
                                                           self.method_id, out, size, ctypes.byref(n)),
                      "sym_batcher_encode_one")
        return out.raw[:n.value]

    def unmarshal(self, data: bytes, out) -> None:
        s = _schema_of(out)
        data = bytes(data)
        if len(data) > self._cfg[1]:
            return self._direct.unmarshal(data, out)
        cap = max(1, len(data))
        fixed = (ctypes.c_int32 * max(1, s.nfixed))()
        bufs = [ctypes.create_string_buffer(cap) for _ in range(s.nvar)]
        ptrs = (ctypes.c_void_p * max(1, s.nvar))(*[ctypes.addressof(b) for b in bufs])
        caps = (ctypes.c_uint64 * max(1, s.nvar))(*([cap] * s.nvar))
        lens = (ctypes.c_uint64 * max(1, s.nvar))()
        st = ctypes.c_uint8()
        _native.check(_native.lib().sym_batcher_decode_one(self._batcher(s), data, len(data), fixed, ptrs, caps, lens,
                                                           ctypes.byref(st)), "sym_batcher_decode_one")
        for f, name in enumerate(s.fixed_fields):
            setattr(out, name, int(fixed[f]))
        for f, name in enumerate(s.var_fields):
            setattr(out, name, bufs[f].raw[:lens[f]])
        if st.value:
            raise SymphonyError(int(st.value))

    def stats(self) -> dict:
        """Batches flushed and records carried per schema and direction (sym_batcher_stats)."""
        out = {}
        for sid, b in list(self._batchers.items()):
            v = [ctypes.c_uint64() for _ in range(4)]
            _native.check(_native.lib().sym_batcher_stats(b, *[ctypes.byref(x) for x in v]), "sym_batcher_stats")
            out[sid] = {"encode_batches": v[0].value, "encode_records": v[1].value,
                        "decode_batches": v[2].value, "decode_records": v[3].value}
        return out

    def quiesce(self) -> None:
        """Stop the device's ring workers now (sym_batcher_quiesce; the next call restarts them): before
        a device-wide synchronisation that should not wait for their idle timeout."""
        for b in list(self._batchers.values()):
            _native.check(_native.lib().sym_batcher_quiesce(b), "sym_batcher_quiesce")
            break  # the rings are the device's, shared by every batcher

    def close(self) -> None:
        with self._lock:
            for b in self._batchers.values():
                _native.lib().sym_batcher_destroy(b)
            self._batchers.clear()


def _group_by_schema(msgs) -> dict:
    groups: dict = {}
    for i, m in enumerate(msgs):
        groups.setdefault(_schema_of(m), []).append(i)
    return groups


def message_fields(msg) -> dict:
    return {f.name: getattr(msg, f.name) for f in fields(msg)}


__all__ = ["SymphonySerializer", "BatchingSerializer", "SymphonyError", "ERROR_TEXT", "GetRequest", "SetRequest", "GetResponse",
           "SetResponse", "EchoRequest", "EchoResponse", "MESSAGE_TYPES", "encode_columns_host",
           "decode_columns_host", "message_fields"]

"""Any Symphony schema on the GPU: flat, repeated and nested.

Reference: the protoc-gen-symphony generator emits, per message, MarshalSymphony / UnmarshalSymphony
whose layout follows the fields' kinds and `is_public` flags
(cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-368 marshal, :622-800 unmarshal, :493-620 and
:843-947 repeated / nested; field classification :1172-1239).  Here the message is described at run
time -- `FlatSchema` lists the fields in declaration order -- and one set of kernels serves every
schema (arpc_amd/csrc/flat.hip, `sym_flat_encode_ex` / `sym_flat_decode_ex`).  A message-typed
field is one level of that codec: `encode` / `decode` below walk the message tree, encoding inner
messages first (their bytes become the outer field's items) and decoding outer records first (their
items become the inner records), folding inner statuses back with `sym_flat_nested_status`.

Kinds (protobuf scalar -> table width): bool 1; int32, uint32, float, enum 4; int64, uint64,
double 8; string, bytes 0 (a 4-byte payload offset in the table, then length + bytes); message
(a 4-byte offset, then length + the inner message, or a 0 offset when nil).

Columns (per field, n records):
  scalar                  tensor of n values
  string / bytes          (uint8 bytes, int64 offsets [n+1])
  repeated scalar         (uint8 element bytes, int64 byte offsets [n+1])
  repeated string / bytes ListColumn(bytes, item_off [m+1], rec [n+1]: record i has items rec[i]..rec[i+1])
  message                 MessageColumn(cols of the inner schema over m present messages, rec [n+1], at
                          most one per record; none = nil)
  repeated message        MessageColumn(cols over m items, rec [n+1])
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field as dc_field

import numpy as np
import torch

from . import _native
from .codec import Codec, _check_col, _dptr, _stream_handle

WIDTH = {"bool": 1, "int32": 4, "uint32": 4, "float": 4, "enum": 4, "int64": 8, "uint64": 8, "double": 8,
         "string": 0, "bytes": 0}
DTYPE = {"bool": torch.uint8, "int32": torch.int32, "uint32": torch.int32, "float": torch.float32,
         "enum": torch.int32, "int64": torch.int64, "uint64": torch.int64, "double": torch.float64}


@dataclass(frozen=True)
class FlatField:
    """One field; `repeated` with a fixed-width kind is `repeated int32 xs` etc. (payload: u32
    count + elements, main.go:493-535, :795-841), carried like a string column: (element bytes,
    int64 byte offsets [n+1]).  kind "message" takes the inner schema in `message`."""
    name: str
    kind: str
    public: bool = False
    repeated: bool = False
    message: "FlatSchema | None" = None

    def __post_init__(self):
        if (self.kind == "message") != (self.message is not None):
            raise ValueError(f"{self.name}: a message field names its schema (and only it does)")
        if self.kind != "message" and self.kind not in WIDTH:
            raise ValueError(f"{self.name}: unknown kind {self.kind}")

    @property
    def list_like(self) -> bool:
        """Repeated string / bytes, nested and repeated messages: item lists on the C-ABI."""
        return self.kind == "message" or (self.repeated and not WIDTH[self.kind])

    @property
    def width(self) -> int:
        """Scalar width of a fixed field's value column; 0 for payload fields."""
        return 0 if self.repeated or self.kind == "message" else WIDTH[self.kind]

    @property
    def c_width(self) -> int:
        if self.kind == "message":
            return _native.SYM_FIELD_MESSAGE | (_native.SYM_FIELD_REPEATED if self.repeated else 0)
        return (_native.SYM_FIELD_REPEATED | WIDTH[self.kind]) if self.repeated else WIDTH[self.kind]


@dataclass
class ListColumn:
    """Items of a list-like field: bytes, item byte offsets [m+1], record item ranges [n+1]."""
    bytes: torch.Tensor
    item_off: torch.Tensor
    rec: torch.Tensor


@dataclass
class MessageColumn:
    """Inner messages of a message field: the inner schema's columns over its m items, the record
    item ranges [n+1], and (decode) the items' statuses."""
    cols: list
    rec: torch.Tensor
    status: torch.Tensor | None = None
    n_items: int = 0


_C_FIELDS: dict = {}


@dataclass(frozen=True)
class FlatSchema:
    name: str
    fields: tuple

    def c_fields(self, framed: bool = False):
        """The C field list; framed: message fields flagged SYM_FIELD_FRAMED (encode, their items
        being the inner level's frames)."""
        arr = _C_FIELDS.get((self, framed))
        if arr is None:  # built once per schema (a tree walk asks for it at every level)
            arr = (_native.SymField * max(1, len(self.fields)))()
            for k, f in enumerate(self.fields):
                arr[k].segment = _native.SYM_SEGMENT_PUBLIC if f.public else _native.SYM_SEGMENT_PRIVATE
                arr[k].width = f.c_width | (_native.SYM_FIELD_FRAMED if framed and f.kind == "message" else 0)
            _C_FIELDS[(self, framed)] = arr
        return arr

    @property
    def has_lists(self) -> bool:
        return any(f.list_like for f in self.fields)


# benchmark/kv-store-symphony-element/symphony/kv.proto:18-41 (score and username public)
ELEMENT_SET_REQUEST = FlatSchema("SetRequest(element)", (FlatField("Score", "int32", True),
                                                         FlatField("Username", "string", True),
                                                         FlatField("Key", "string"), FlatField("Value", "string")))
ELEMENT_GET_REQUEST = FlatSchema("GetRequest(element)", (FlatField("Score", "int32", True),
                                                         FlatField("Username", "string", True),
                                                         FlatField("Key", "string")))
# cmd/symphony-gen-arpc/test/test.proto:13-22 (message Fixed)
TEST_FIXED = FlatSchema("Fixed", (FlatField("FInt32", "int32", True), FlatField("FInt64", "int64"),
                                  FlatField("FUint32", "uint32", True), FlatField("FUint64", "uint64"),
                                  FlatField("FBool", "bool", True), FlatField("FFloat", "float"),
                                  FlatField("FDouble", "double", True)))


def encode(codec: Codec, schema: FlatSchema, cols: list, service_id: int = 0, method_id: int = 0,
           stream=None, n: int | None = None, out=None):
    """cols[k] per the module docstring.  -> (stream uint8, offsets int64 [n+1]).  `n` is needed
    only for a schema without fields (n empty messages).  out=(uint8 buffer, int64 [n+1]): the
    buffer must hold the encoded size; it is returned whole.  Message fields are encoded first
    (their own message fields first), with service / method ids 0 as MarshalSymphony writes for
    nested messages.  The whole tree is launched without a host sync; only the returned stream's
    length (offsets[n]) is read back at the end.  A level's message fields are independent
    subtrees: with two or more, each runs on a branch of the codec (Codec.branch: its own stream)
    and the level waits for them all."""
    cur = stream if stream is not None else torch.cuda.current_stream(codec.device)
    keep: list = []  # every level's temporaries, alive until the tree is queued (see _encode)
    fork_min = _fork_min(cur)
    if out is None and fork_min == _NO_BRANCH:
        raise ValueError("encode under a graph capture needs out=(buffer, offsets): the returned stream's length "
                         "is a host read (or use EncodeGraph)")
    buf, off = _encode(codec, codec._ctx, schema, cols, service_id, method_id, cur, n, out, False, keep,
                       [0, fork_min])
    if out is not None:
        return buf, off
    size = int(off[-1].item()) if off.numel() > 1 else 0
    return buf[:size], off


_BRANCH_MIN = 1 << 16  # records of a level below which its subtrees stay on its stream (forks cost host time)
_NO_BRANCH = 1 << 62  # graph captures: every subtree on the capturing stream (see _capture)


def _capturing(stream) -> bool:
    """Is `stream` being captured into a HIP graph (a caller's torch.cuda.graph or
    hipStreamBeginCapture)?  torch asks hipStreamIsCapturing of the current stream."""
    with torch.cuda.stream(stream):
        return torch.cuda.is_current_stream_capturing()


def _fork_min(stream) -> int:
    """The walk's branch threshold on `stream`: no branches at all while it is captured.  This ROCm's
    hipStreamEndCapture segfaults on a capture in which a stream forked from the capturing stream
    forks again (DESIGN.md section 4 "Graph capture and branch streams": profiles/r04_graph_fork.txt,
    r04_graph_stages.txt), and a tree of three message levels with two message fields each does exactly
    that; one stream costs a captured walk nothing (a graph's launches are queued by the device)."""
    return _NO_BRANCH if _capturing(stream) else _BRANCH_MIN


def _rows(cols: list, schema: FlatSchema) -> int:
    """A level's record count as far as the host knows it (column sizes, no device read)."""
    for f, c in zip(schema.fields, cols):
        if isinstance(c, MessageColumn) or isinstance(c, ListColumn):
            return c.rec.numel() - 1
        if isinstance(c, tuple):
            return c[1].numel() - 1
        if isinstance(c, torch.Tensor):
            return c.numel()
    return 0


def _wrapper(schema: FlatSchema) -> bool:
    """A wrapper: one field, a private non-repeated message of a schema with fields (online-boutique's
    PlaceOrderResponse{Order}, GetQuoteResponse{CostUsd}).  Its record is 18 constant bytes before
    the item's frame when the item is present (generator main.go:196-330, :565-590): header
    (version, offset_to_private 13, service, method), the private marker, the table entry 5."""
    return len(schema.fields) == 1 and schema.fields[0].kind == "message" and not schema.fields[0].repeated \
        and not schema.fields[0].public and bool(schema.fields[0].message.fields)


def _wrapper_prefix(service_id: int, method_id: int) -> bytes:
    le = lambda v: int(v).to_bytes(4, "little")  # noqa: E731
    return b"\x01" + le(13) + le(service_id) + le(method_id) + b"\x01" + le(5)


def _encode(codec: Codec, ctx, schema: FlatSchema, cols: list, service_id: int, method_id: int, stream, n, out,
            framed: bool, keep: list, fork: list, wrap: dict | None = None):
    """encode() without the final read-back: the output buffer is sized from the columns' tensor
    sizes (an upper bound of the encoded size: sym_flat_encoded_size_ex of every byte / item column
    taken whole), so no level needs a device value on the host.  Inner levels are encoded framed
    (sym_flat_encode_opts.framed: [u32 size] before each record), so an outer body is one window of
    them.  A wrapper level that is not itself framed (_wrapper; the tree's root) is written by its
    inner level's kernel when every record has its item -- the 18 wrapper bytes as that kernel's
    frame prefix, straight into the wrapper's output (`wrap`) -- and by its own kernel otherwise;
    both alternatives are queued, gated on the device by the item ranges (d_gate_rec), so the walk
    still reads nothing back.  The wrapper's own kernel would copy every inner byte again (the
    boutique root level: ~90 us for 150 MB).
    Subtrees on other branches free nothing before the whole tree is queued (`keep`): a block freed
    while a kernel of another branch may still read it could be handed to a concurrent branch;
    after the walk, later work on any branch is ordered after this tree (branches start by waiting
    on the caller's stream)."""
    if len(cols) != len(schema.fields):
        raise ValueError(f"{schema.name}: {len(schema.fields)} columns expected")
    if not schema.fields and n is None:
        raise ValueError(f"{schema.name}: a schema without fields needs the record count n")
    ptrs, offs, items, nbytes, nitems, n_arg = [], [], [], [], [], n
    string_bytes = 0
    n = None if schema.fields else n
    msg = [k for k, f in enumerate(schema.fields) if f.kind == "message"]
    for k in msg:
        if not isinstance(cols[k], MessageColumn):
            raise ValueError(f"{schema.fields[k].name}: a MessageColumn expected")
    # independent subtrees: the first on this stream, the others on branches that start after this
    # stream's work so far and are joined back before this level's kernel
    runs = [(ctx, stream)]
    for _ in (msg[1:] if _rows(cols, schema) >= fork[1] else []):
        b_ctx, b_st = codec.branch(fork[0])
        fork[0] += 1
        b_st.wait_stream(stream)
        runs.append((b_ctx, b_st))
    inner = {}
    gate = None  # a wrapper level written by its inner level's kernel: the item ranges its own launch is gated on
    runs += [(ctx, stream)] * (len(msg) - len(runs))  # small levels: every subtree on this stream
    for (r_ctx, r_st), k in zip(runs, msg):
        c = cols[k]
        # a fieldless inner schema needs its record count: the one host read of a level, which a
        # graph capture cannot hold
        m_in = None
        if not c.cols:
            if c.rec.numel() > 1 and _capturing(r_st):
                raise ValueError(f"{schema.fields[k].name}: a nested message without fields needs a host read "
                                 "of its item count, which a graph capture cannot hold; encode it eagerly")
            m_in = int(c.rec[-1].item() - c.rec[0].item()) if c.rec.numel() > 1 else 0
        w = None
        if not framed and _wrapper(schema) and c.rec.numel() > 1:
            w = {"prefix": _wrapper_prefix(service_id, method_id), "out": out, "n": c.rec.numel() - 1, "rec": c.rec}
        ib, io = _encode(codec, r_ctx, schema.fields[k].message, c.cols, 0, 0, r_st, m_in, None, True, keep, fork, w)
        if w is not None and w.get("fused"):
            out, gate = w["out"], w["rec"]  # this level's output: the buffers the fused launch wrote
        inner[k] = ListColumn(ib, io, c.rec)
        keep.append(inner[k])
    for _, r_st in runs[1:]:
        stream.wait_stream(r_st)
    for k, (f, c) in enumerate(zip(schema.fields, cols)):
        if k in inner:
            c = inner[k]
        if f.list_like:
            _check_col(c.bytes, torch.uint8, f.name, codec.device)
            _check_col(c.item_off, torch.int64, f.name + " item offsets", codec.device)
            _check_col(c.rec, torch.int64, f.name + " record items", codec.device)
            m = c.rec.numel() - 1
            ptrs.append(_dptr(c.bytes) or 1)
            offs.append(_dptr(c.rec))
            items.append(_dptr(c.item_off))
            nbytes.append(c.bytes.numel())
            nitems.append(max(0, c.item_off.numel() - 1))
        elif f.width:
            if c.element_size() != f.width or c.device != codec.device or not c.is_contiguous():
                raise ValueError(f"{f.name}: a contiguous {f.width}-byte column on {codec.device} expected")
            m = c.numel()
            ptrs.append(_dptr(c) or 1)
            offs.append(0)
            items.append(0)
            nbytes.append(0)
            nitems.append(0)
        else:
            b, o = c
            _check_col(b, torch.uint8, f.name, codec.device)
            _check_col(o, torch.int64, f.name + " offsets", codec.device)
            m = o.numel() - 1
            nbytes.append(b.numel())
            string_bytes += b.numel()  # (the kernel's choice of windows per chunk: a size hint)
            nitems.append(0)
            ptrs.append(_dptr(b) or 1)
            offs.append(_dptr(o))
            items.append(0)
        if n is not None and m != n:
            raise ValueError("columns disagree on the record count")
        n = m
    if n_arg is not None and n is not None and n != n_arg:
        raise ValueError("columns disagree with n")
    n = n or 0
    cf = schema.c_fields(framed=True)  # (the flag only matters for message fields, whose items are frames)
    if out is None:
        size = codec._lib.sym_flat_encoded_size_ex(cf, len(schema.fields), n, _native.u64_array(nbytes or [0]),
                                                   _native.u64_array(nitems or [0])) + (4 * n if framed else 0)
        out = torch.empty(max(1, size), dtype=torch.uint8, device=codec.device)
        off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    else:
        out, off = out
        _check_col(out, torch.uint8, "out", codec.device)
        _check_col(off, torch.int64, "out offsets", codec.device)
        if off.numel() != n + 1:
            raise ValueError("out offsets: n + 1 entries expected")
    lists = schema.has_lists

    def launch(o, buf, boff):
        _native.check(codec._lib.sym_flat_encode_ex(ctx, cf, len(schema.fields), n, _native.ptr_array(ptrs),
                                                    _native.ptr_array(offs), _native.ptr_array(items) if lists else None,
                                                    ctypes.byref(o), _dptr(buf), _dptr(boff), stream.cuda_stream),
                      "sym_flat_encode_ex")

    opts = _native.FlatEncodeOpts(service_id=service_id, method_id=method_id, framed=1 if framed else 0,
                                  string_bytes=string_bytes)
    if wrap is not None and n and n == wrap["n"]:  # the wrapper above, written here when every record has its item
        wn = wrap["n"]
        if wrap["out"] is None:  # its output, sized as its own launch would size it (and for the prefixes)
            wsize = 18 * max(wn, n) + out.numel() + 16
            wrap["out"] = (torch.empty(wsize, dtype=torch.uint8, device=codec.device),
                           torch.empty(wn + 1, dtype=torch.int64, device=codec.device))
        wbuf, woff = wrap["out"]
        _check_col(wbuf, torch.uint8, "out", codec.device)
        _check_col(woff, torch.int64, "out offsets", codec.device)
        if woff.numel() != wn + 1:
            raise ValueError("out offsets: n + 1 entries expected")
        fused = _native.FlatEncodeOpts(framed=1, frame_prefix_len=len(wrap["prefix"]), string_bytes=string_bytes,
                                       d_gate_rec=_dptr(wrap["rec"]), gate_n=wn, gate_when_all=1)
        fused.frame_prefix[:len(wrap["prefix"])] = list(wrap["prefix"])
        launch(fused, wbuf, woff)
        wrap["fused"] = True
        opts.d_gate_rec, opts.gate_n, opts.gate_when_all = _dptr(wrap["rec"]), wn, 0
    if gate is not None and n:  # this (wrapper) level's own launch: only when an item is missing
        opts.d_gate_rec, opts.gate_n, opts.gate_when_all = _dptr(gate), n, 0
    launch(opts, out, off)
    return out, off


def decode(codec: Codec, schema: FlatSchema, data: torch.Tensor, rec_off: torch.Tensor, stream=None,
           span: int | None = None, with_fail: bool = False, rec_len: torch.Tensor | None = None,
           extent: tuple | None = None):
    """UnmarshalSymphony into fresh structs -> (cols, status) (with_fail: (cols, status, fail)); cols
    per the module docstring, message fields decoded recursively with their items' statuses folded
    into `status` (SYM_STATUS_NESTED).  span = rec_off[n] - rec_off[0] when the caller knows it
    (skips a device sync).  Inner levels are decoded in place (sym_flat_decode_ex): a message
    field's items stay where they are in `data` -- rec_off holds their offsets, rec_len their
    lengths, extent the device pointers bounding data's readable bytes, span an upper bound of their
    bytes -- so no level copies its inner messages out.  The whole tree is queued without a host
    sync: an inner level's record count stays on the device (the outer level's item count, from
    sym_flat_list_sizes) and its columns are sized for a capacity; every level's list sizes are
    read back once, at the end, and the columns cut to them.  A level's message fields are
    independent subtrees: with two or more, each runs on a branch of the codec (Codec.branch: its
    own stream and context, the decode workspace being per context)."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    if rec_len is not None:
        _check_col(rec_len, torch.int64, "rec_len", codec.device)
        if rec_len.numel() and (extent is None or span is None):
            raise ValueError("records in place need extent and span")
    n = rec_off.numel() - 1 if rec_len is None else rec_len.numel()
    cur = stream if stream is not None else torch.cuda.current_stream(codec.device)
    if _capturing(cur):
        raise ValueError("decode cuts its columns to sizes read back from the device, which a graph capture "
                         "cannot hold: capture it with DecodeGraph")
    if span is None:
        span = int(rec_off[-1].item() - rec_off[0].item()) if n else 0
    pend: list = []  # every level's device list sizes, read back together
    lvl = _decode_level(codec, codec._ctx, schema, data, rec_off, rec_len, n, None, span, extent, cur, pend,
                        [0, _fork_min(cur)])
    sizes = torch.cat(pend).tolist() if pend else []  # the tree's one host read
    out, st, fail = _finish_level(lvl, n, sizes)
    return (out, st, fail) if with_fail else (out, st)


@dataclass
class _Level:
    """A decode level queued on the device (_decode_level), to be cut to its sizes (_finish_level)."""
    schema: FlatSchema
    cols: list
    st: torch.Tensor
    fail: torch.Tensor
    lk: list        # list-like field indices
    at: int         # their (items, item bytes) pairs' position in the tree's size list
    inner: dict     # message field index -> _Level


def _decode_level(codec: Codec, ctx, schema: FlatSchema, data, rec_src, rec_len, ncap: int, n_dev, span: int, extent,
                  stream, pend: list, fork: list) -> _Level:
    """Queues one level over `ncap` records (n_dev: a device u64 address holding the real count,
    <= ncap; None: ncap is the count) on `stream` with context `ctx` and, recursively, its message
    fields' levels (two or more on branches, joined back before the statuses are folded in)."""
    hs = stream.cuda_stream
    in_place = rec_len is not None and ncap > 0
    if extent is None and ncap:  # data's readable extent: rec_off[0], rec_off[n] (device values)
        extent = (_dptr(rec_src), _dptr(rec_src) + 8 * ncap)
    cols, ptrs, caps, offs, items, ilens, icaps = [], [], [], [], [], [], []
    for f in schema.fields:
        if f.width:
            c = torch.empty(max(1, ncap), dtype=DTYPE[f.kind], device=codec.device)
            cols.append(c)
            ptrs.append(_dptr(c))
            caps.append(0)
            offs.append(0)
            items.append(0)
            ilens.append(0)
            icaps.append(0)
        elif f.list_like:
            icap = ncap if (f.kind == "message" and not f.repeated) else span // 4 + 1  # items hold a [u32 len] each
            msg = f.kind == "message"  # items left in place: (offset into data, length)
            b = torch.empty(1 if msg else max(1, span), dtype=torch.uint8, device=codec.device)
            io = torch.empty(icap + 1, dtype=torch.int64, device=codec.device)
            il = torch.empty(max(1, icap), dtype=torch.int64, device=codec.device) if msg else None
            rec = torch.empty(ncap + 1, dtype=torch.int64, device=codec.device)
            lc = ListColumn(b, io, rec)
            lc.item_len = il
            cols.append(lc)
            ptrs.append(_dptr(b))
            caps.append(0 if msg else span)
            offs.append(_dptr(rec))
            items.append(_dptr(io))
            ilens.append(_dptr(il) if msg else 0)
            icaps.append(icap)
        else:
            b = torch.empty(max(1, span), dtype=torch.uint8, device=codec.device)
            o = torch.empty(ncap + 1, dtype=torch.int64, device=codec.device)
            cols.append((b, o))
            ptrs.append(_dptr(b))
            caps.append(span)
            offs.append(_dptr(o))
            items.append(0)
            ilens.append(0)
            icaps.append(0)
    st = torch.empty(max(1, ncap), dtype=torch.uint8, device=codec.device)
    fail = torch.empty(max(1, ncap), dtype=torch.uint8, device=codec.device)
    cf = schema.c_fields()
    lists = schema.has_lists
    lo, hi = extent if in_place else (0, 0)
    _native.check(codec._lib.sym_flat_decode_ex(ctx, cf, len(schema.fields), ncap, n_dev, _dptr(data) or 1,
                                                _dptr(rec_src) or 1, _dptr(rec_len) if in_place else 0, lo, hi,
                                                _native.ptr_array(ptrs), _native.u64_array(caps),
                                                _native.ptr_array(offs), _native.ptr_array(items) if lists else None,
                                                _native.ptr_array(ilens) if lists else None,
                                                _native.u64_array(icaps) if lists else None, _dptr(st), _dptr(fail),
                                                hs), "sym_flat_decode_ex")
    lk = [k for k, f in enumerate(schema.fields) if f.list_like]
    lvl = _Level(schema, cols, st, fail, lk, sum(t.numel() for t in pend), {})
    if not ncap:  # no records: empty inner levels
        for k in lk:
            if schema.fields[k].kind == "message":
                lc = cols[k]
                lvl.inner[k] = _decode_level(codec, ctx, schema.fields[k].message, data, lc.item_off[:0],
                                             lc.item_len[:0], 0, None, span, extent, stream, pend, fork)
        return lvl
    if not lk:
        return lvl
    # every list field's item count and item bytes, on the device (read back with the whole tree's)
    sz = torch.empty(2 * len(lk), dtype=torch.int64, device=codec.device)
    _native.check(codec._lib.sym_flat_list_sizes(ctx, len(lk), ncap, n_dev,
                                                  _native.ptr_array([_dptr(cols[k].rec) for k in lk]),
                                                  _native.ptr_array([_dptr(cols[k].item_off) for k in lk]),
                                                  _native.u64_array([icaps[k] for k in lk]), _dptr(sz), hs),
                  "sym_flat_list_sizes")
    pend.append(sz)
    msg = [(i, k) for i, k in enumerate(lk) if schema.fields[k].kind == "message"]
    runs = [(ctx, stream)]
    for _ in (msg[1:] if ncap >= fork[1] else []):  # branches start after this level's kernels
        b_ctx, b_st = codec.branch(fork[0])
        fork[0] += 1
        b_st.wait_stream(stream)
        runs.append((b_ctx, b_st))
    runs += [(ctx, stream)] * (len(msg) - len(runs))  # small levels: every subtree on this stream
    for (r_ctx, r_st), (i, k) in zip(runs, msg):
        lc = cols[k]
        # the items are the inner records, in place in `data`: their count is sz[2i] on the device
        lvl.inner[k] = _decode_level(codec, r_ctx, schema.fields[k].message, data, lc.item_off, lc.item_len, icaps[k],
                                     _dptr(sz) + 16 * i, span, extent, r_st, pend, fork)
    for _, r_st in runs[1:]:
        stream.wait_stream(r_st)
    if lvl.inner:  # the inner statuses folded into this level's, every message field in one launch
        ks = sorted(lvl.inner)
        _native.check(codec._lib.sym_flat_nested_status(
            ctx, cf, len(schema.fields), len(ks), (ctypes.c_int * len(ks))(*ks), ncap, n_dev,
            _native.ptr_array([_dptr(cols[k].rec) for k in ks]),
            _native.ptr_array([_dptr(lvl.inner[k].st) or 1 for k in ks]), _dptr(st), _dptr(fail), hs),
            "sym_flat_nested_status")
    return lvl


def _finish_level(lvl: _Level, n: int, sizes: list):
    """The level's columns cut to its n records and its lists' sizes -> (cols, status, fail); the
    level itself is left whole (a DecodeGraph cuts the same level after every replay)."""
    cols = list(lvl.cols)
    for i, k in enumerate(lvl.lk):
        m, nb = (int(sizes[lvl.at + 2 * i]), int(sizes[lvl.at + 2 * i + 1])) if n else (0, 0)
        lc = cols[k]
        if k in lvl.inner:
            inner_cols, inner_st, _ = _finish_level(lvl.inner[k], m, sizes)
            cols[k] = MessageColumn(inner_cols, lc.rec[:n + 1], inner_st, m)
            continue
        cols[k] = ListColumn(lc.bytes[:nb if m else 0], lc.item_off[:m + 1], lc.rec[:n + 1])
    for k, c in enumerate(cols):
        if isinstance(c, torch.Tensor):
            cols[k] = c[:n]
        elif isinstance(c, tuple):
            cols[k] = (c[0], c[1][:n + 1])
    return cols, lvl.st[:n], lvl.fail[:n]


_GRAPH_TRACE = bool(int(__import__("os").environ.get("SYMHIP_GRAPH_TRACE", "0")))


def _capture(codec: Codec, run):
    """run(stream) queued once on a side stream (its workspaces, branch contexts and streams
    created), then captured as a HIP graph on that stream (torch.cuda.CUDAGraph: stream capture,
    torch's graph pool holding every buffer the walk allocates) -> (graph, stream, run's result of
    the capture).  Nothing in a tree walk syncs the host, so the whole walk is one graph.  The walk
    is captured on one stream: with branch streams forked and joined inside the capture this ROCm's
    hipStreamEndCapture crashes -- the tree walk's forks (tools/graph_stages.py, stage 5), a fork of
    a fork with torch ops alone (tools/graph_fork.py, stage 2; `profiles/r04_graph_fork.txt`), and
    the walk with forks from the capturing stream only, one fork point open at a time."""
    s = torch.cuda.Stream(codec.device)
    s.wait_stream(torch.cuda.current_stream(codec.device))
    run(s)
    codec.check(s)
    if _GRAPH_TRACE:
        print("graph: warm-up run done", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        res = run(s)
    if _GRAPH_TRACE:
        print("graph: captured", flush=True)
    return g, s, res


class _Replayed:
    """A captured walk's replay, split in two so that many graphs can be queued before any result
    is read: launch() queues the graph on `stream` (the current one by default) and the copy of its
    sizes into pinned host memory; result() waits for that copy alone."""

    def _bind_sizes(self, sizes):
        self._dev_sizes = sizes
        self._host = torch.empty(sizes.numel(), dtype=torch.int64, pin_memory=True) if sizes is not None else None
        self._done = torch.cuda.Event()

    def launch(self, stream=None):
        cur = stream if stream is not None else torch.cuda.current_stream(self.codec.device)
        with torch.cuda.stream(cur):  # a graph replays on the current stream, not the one it was captured on
            self.graph.replay()
            if self._host is not None:
                self._host.copy_(self._dev_sizes, non_blocking=True)
            self._done.record(cur)

    def _sizes_read(self) -> list:
        self._done.synchronize()
        return self._host.tolist() if self._host is not None else []


class EncodeGraph(_Replayed):
    """encode() of one schema over bound input columns, captured once as a HIP graph and replayed:
    one graph launch instead of the walk's kernel launches and its host work (the walk's Python,
    the C-ABI calls and ~5 us of launch cost per kernel).  The caller refills
    the bound columns in place between calls (same shapes: the walk's grids and the output's
    capacity follow the column sizes, as in encode()); every replay encodes their current contents.
    The returned stream and offsets are the graph's own buffers, overwritten by the next replay.
    The graph has its own Codec (contexts whose workspaces stay where the graph saw them)."""

    def __init__(self, device, schema: FlatSchema, cols: list, service_id: int = 0, method_id: int = 0,
                 n: int | None = None):
        self.codec = Codec(device)
        self.cols = cols

        def run(s):
            keep: list = []
            res = _encode(self.codec, self.codec._ctx, schema, cols, service_id, method_id, s, n, None, False,
                          keep, [0, _NO_BRANCH])
            return res, keep
        self.graph, self.stream, ((self.buf, self.off), self._keep) = _capture(self.codec, run)
        self._bind_sizes(self.off[-1:] if self.off.numel() > 1 else None)

    def result(self):
        """-> (stream uint8, offsets int64 [n+1]) of the last launch()."""
        sz = self._sizes_read()
        return self.buf[:int(sz[0]) if sz else 0], self.off

    def replay(self, stream=None):
        """launch() then result(): the bound columns' current contents encoded."""
        self.launch(stream)
        return self.result()


class DecodeGraph(_Replayed):
    """decode() of one schema over bound input buffers (data, rec_off), captured once as a HIP graph
    and replayed (see EncodeGraph).  Every level's columns are sized from n and `span` alone (inner
    record counts stay on the device), so one graph decodes any batch of n records whose bytes fit
    in `span`: the caller refills data and rec_off in place between calls.  Results are views of the
    graph's own buffers, cut to the replay's sizes (one host read), overwritten by the next replay."""

    def __init__(self, device, schema: FlatSchema, data: torch.Tensor, rec_off: torch.Tensor, span: int | None = None):
        self.codec = Codec(device)
        _check_col(data, torch.uint8, "data", self.codec.device)
        _check_col(rec_off, torch.int64, "rec_off", self.codec.device)
        self.n = n = rec_off.numel() - 1
        self.data, self.rec_off = data, rec_off
        span = data.numel() if span is None else span

        def run(s):
            pend: list = []
            lvl = _decode_level(self.codec, self.codec._ctx, schema, data, rec_off, None, n, None, span, None, s,
                                pend, [0, _NO_BRANCH])
            return lvl, (torch.cat(pend) if pend else None)
        self.graph, self.stream, (self._lvl, sizes) = _capture(self.codec, run)
        self._bind_sizes(sizes)

    def result(self, with_fail: bool = False):
        """-> (cols, status) (with_fail: (cols, status, fail)) of the last launch().  The column views
        are cut again only when the replay's sizes differ from the previous replay's (the cutting is
        ~45 us of Python for the online-boutique tree; the views of equal sizes are the same)."""
        sizes = self._sizes_read()
        key = tuple(sizes)
        if getattr(self, "_cut_key", None) != key:
            self._cut = _finish_level(self._lvl, self.n, sizes)
            self._cut_key = key
        out, st, fail = self._cut
        out = list(out)  # (the caller's own list)
        return (out, st, fail) if with_fail else (out, st)

    def replay(self, stream=None, with_fail: bool = False):
        """launch() then result(): the bound buffers' current contents decoded."""
        self.launch(stream)
        return self.result(with_fail)


def _c_fields(fields):
    """A FlatSchema, or [(segment 0 public / 1 private, width | SYM_FIELD_REPEATED)] pairs."""
    if isinstance(fields, FlatSchema):
        return fields.c_fields(), [(0 if f.public else 1, f.c_width) for f in fields.fields]
    arr = (_native.SymField * max(1, len(fields)))()
    for k, (seg, w) in enumerate(fields):
        arr[k].segment, arr[k].width = seg, w
    return arr, list(fields)


def raw_set(codec: Codec, fields, k: int, data: torch.Tensor, rec_off: torch.Tensor, values, n: int | None = None,
            out_cap: int | None = None, stream=None):
    """XxxRaw.Set<field k>(values[i]) on buffer i (sym_raw_set; generator main.go:1038-1093, 1296-1336,
    1567-1620, 1685-1740, 371-437).  values: a tensor of n values of the field's width (fixed field)
    or (uint8 bytes, int64 offsets [n+1]) (string / bytes / repeated).  -> (out uint8, out_off int64
    [n+1], status uint8 [n], SYM_SET_*).  out_cap defaults to the bound that always suffices (one
    device sync to read the input span)."""
    cf, pairs = _c_fields(fields)
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    n = rec_off.numel() - 1 if n is None else n
    seg, w = pairs[k]
    scalar = w != 0 and not (w & _native.SYM_FIELD_REPEATED)
    if scalar:
        vb, vo = values, None
        _check_col(vb, vb.dtype, "values", codec.device)
        vbytes = vb.numel() * vb.element_size()
    else:
        vb, vo = values
        _check_col(vb, torch.uint8, "values", codec.device)
        _check_col(vo, torch.int64, "value offsets", codec.device)
        vbytes = int(vo[-1].item() - vo[0].item()) if n else 0
    if out_cap is None:
        nv = sum(1 for _, wd in pairs if wd == 0 or wd & _native.SYM_FIELD_REPEATED)
        g = 14 + sum(4 if (wd == 0 or wd & _native.SYM_FIELD_REPEATED) else wd for _, wd in pairs) + 4 * nv
        span = int(rec_off[-1].item() - rec_off[0].item()) if n else 0
        out_cap = (nv + 1) * span + n * g + vbytes + 16
    out = torch.empty(max(1, out_cap), dtype=torch.uint8, device=codec.device)
    off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    st = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    _native.check(codec._lib.sym_raw_set(codec._ctx, cf, len(pairs), k, _dptr(data) or 1, _dptr(rec_off), n,
                                         _dptr(vb) or 1, _dptr(vo) if vo is not None else 0, _dptr(out), out_cap,
                                         _dptr(off), _dptr(st), _stream_handle(codec.device, stream)), "sym_raw_set")
    return out, off, st[:n]


# benchmark/serialization/online-boutique/proto/onlineboutique.proto (every field private: the
# file sets no is_public option); the messages of the PlaceOrder and ListProducts responses
OB_MONEY = FlatSchema("Money", (FlatField("CurrencyCode", "string"), FlatField("Units", "int64"),
                                FlatField("Nanos", "int32")))
OB_CART_ITEM = FlatSchema("CartItem", (FlatField("ProductId", "string"), FlatField("Quantity", "int32")))
OB_ADDRESS = FlatSchema("Address", (FlatField("StreetAddress", "string"), FlatField("City", "string"),
                                    FlatField("State", "string"), FlatField("Country", "string"),
                                    FlatField("ZipCode", "int32")))
OB_ORDER_ITEM = FlatSchema("OrderItem", (FlatField("Item", "message", message=OB_CART_ITEM),
                                         FlatField("Cost", "message", message=OB_MONEY)))
OB_ORDER_RESULT = FlatSchema("OrderResult", (FlatField("OrderId", "string"), FlatField("ShippingTrackingId", "string"),
                                             FlatField("ShippingCost", "message", message=OB_MONEY),
                                             FlatField("ShippingAddress", "message", message=OB_ADDRESS),
                                             FlatField("Items", "message", repeated=True, message=OB_ORDER_ITEM)))
OB_PLACE_ORDER_RESPONSE = FlatSchema("PlaceOrderResponse", (FlatField("Order", "message", message=OB_ORDER_RESULT),))
OB_PRODUCT = FlatSchema("Product", (FlatField("Id", "string"), FlatField("Name", "string"),
                                    FlatField("Description", "string"), FlatField("Picture", "string"),
                                    FlatField("PriceUsd", "message", message=OB_MONEY),
                                    FlatField("Categories", "string", repeated=True)))
OB_LIST_PRODUCTS_RESPONSE = FlatSchema("ListProductsResponse",
                                       (FlatField("Products", "message", repeated=True, message=OB_PRODUCT),))


def columns_from_tree(schema: FlatSchema, nodes: list, device) -> list:
    """Host column trees (arpc_amd.datagen.ob_place_order) -> device columns for `encode`."""
    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device)
    cols = []
    for f, nd in zip(schema.fields, nodes):
        if f.kind == "message":
            _, children, rec = nd
            cols.append(MessageColumn(columns_from_tree(f.message, children, device), dev(rec)))
        elif f.list_like:
            _, b, io, rec = nd
            cols.append(ListColumn(dev(b), dev(io), dev(rec)))
        elif f.width:
            cols.append(dev(nd))
        else:
            b, o = nd
            cols.append((dev(b), dev(o)))
    return cols

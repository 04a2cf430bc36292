"""Any flat Symphony schema on the GPU (the flat part).

Reference: the protoc-gen-symphony generator emits, per message, MarshalSymphony / UnmarshalSymphony
whose layout follows the fields' kinds and `is_public` flags
(cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:196-368 marshal, :622-800 unmarshal; field
classification :1172-1239).  Here the message is described at run time -- `FlatSchema` lists the
fields in declaration order -- and one pair of kernels serves every flat schema (arpc_amd/csrc/
flat.hip, `sym_flat_encode` / `sym_flat_decode`).  Repeated fixed-width fields are covered;
repeated string and nested fields are not.

Kinds (protobuf scalar -> table width): bool 1; int32, uint32, float, enum 4; int64, uint64,
double 8; string, bytes 0 (a 4-byte payload offset in the table, then length + bytes).
"""
from __future__ import annotations

from dataclasses import dataclass

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
    int64 byte offsets [n+1])."""
    name: str
    kind: str
    public: bool = False
    repeated: bool = False

    def __post_init__(self):
        if self.repeated and not WIDTH[self.kind]:
            raise ValueError(f"{self.name}: repeated {self.kind} fields are not covered")

    @property
    def width(self) -> int:
        """Scalar width of a fixed field's value column; 0 for string and repeated fields."""
        return 0 if self.repeated else WIDTH[self.kind]

    @property
    def c_width(self) -> int:
        return (_native.SYM_FIELD_REPEATED | WIDTH[self.kind]) if self.repeated else WIDTH[self.kind]


@dataclass(frozen=True)
class FlatSchema:
    name: str
    fields: tuple

    def c_fields(self):
        arr = (_native.SymField * max(1, len(self.fields)))()
        for k, f in enumerate(self.fields):
            arr[k].segment = _native.SYM_SEGMENT_PUBLIC if f.public else _native.SYM_SEGMENT_PRIVATE
            arr[k].width = f.c_width
        return arr


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
    """cols[k]: tensor of n values (fixed field; any dtype of the field's width) or (uint8 bytes,
    int64 offsets [n+1]) (string field).  -> (stream uint8, offsets int64 [n+1]).  `n` is needed
    only for a schema without fields (n empty messages).  out=(uint8 buffer, int64 [n+1]) skips
    the size query (a device sync): the buffer must hold encoded_size bytes."""
    if len(cols) != len(schema.fields):
        raise ValueError(f"{schema.name}: {len(schema.fields)} columns expected")
    if not schema.fields and n is None:
        raise ValueError(f"{schema.name}: a schema without fields needs the record count n")
    var_total, ptrs, offs, n_arg = 0, [], [], n
    n = None if schema.fields else n
    for f, c in zip(schema.fields, cols):
        if f.width:
            if c.element_size() != f.width or c.device != codec.device or not c.is_contiguous():
                raise ValueError(f"{f.name}: a contiguous {f.width}-byte column on {codec.device} expected")
            m = c.numel()
            ptrs.append(_dptr(c) or 1)
            offs.append(0)
        else:
            b, o = c
            _check_col(b, torch.uint8, f.name, codec.device)
            _check_col(o, torch.int64, f.name + " offsets", codec.device)
            m = o.numel() - 1
            if out is None:
                var_total += int(o[-1].item() - o[0].item()) if m else 0
            ptrs.append(_dptr(b) or 1)
            offs.append(_dptr(o))
        if n is not None and m != n:
            raise ValueError("columns disagree on the record count")
        n = m
    if n_arg is not None and n is not None and n != n_arg:
        raise ValueError("columns disagree with n")
    n = n or 0
    cf = schema.c_fields()
    if out is None:
        size = codec._lib.sym_flat_encoded_size(cf, len(schema.fields), n, var_total)
        out = torch.empty(max(1, size), dtype=torch.uint8, device=codec.device)
        off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    else:
        out, off = out
        _check_col(out, torch.uint8, "out", codec.device)
        _check_col(off, torch.int64, "out offsets", codec.device)
        if off.numel() != n + 1:
            raise ValueError("out offsets: n + 1 entries expected")
        size = out.numel()
    _native.check(codec._lib.sym_flat_encode(codec._ctx, cf, len(schema.fields), n, _native.ptr_array(ptrs),
                                            _native.ptr_array(offs), service_id, method_id, _dptr(out), _dptr(off),
                                            _stream_handle(codec.device, stream)), "sym_flat_encode")
    return out[:size], off


def decode(codec: Codec, schema: FlatSchema, data: torch.Tensor, rec_off: torch.Tensor, stream=None,
           span: int | None = None):
    """UnmarshalSymphony into fresh structs -> (cols, status); cols[k] a tensor of n values (fixed,
    dtype of its kind) or (uint8 bytes, int64 offsets [n+1]) (string).  span = rec_off[n] -
    rec_off[0] when the caller knows it (skips a device sync)."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    n = rec_off.numel() - 1
    if span is None:
        span = int(rec_off[-1].item() - rec_off[0].item()) if n else 0
    cols, ptrs, caps, offs = [], [], [], []
    for f in schema.fields:
        if f.width:
            c = torch.empty(max(1, n), dtype=DTYPE[f.kind], device=codec.device)
            cols.append(c)
            ptrs.append(_dptr(c))
            caps.append(0)
            offs.append(0)
        else:
            b = torch.empty(max(1, span), dtype=torch.uint8, device=codec.device)
            o = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
            cols.append((b, o))
            ptrs.append(_dptr(b))
            caps.append(span)
            offs.append(_dptr(o))
    st = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    cf = schema.c_fields()
    _native.check(codec._lib.sym_flat_decode(codec._ctx, cf, len(schema.fields), n, _dptr(data) or 1, _dptr(rec_off),
                                            _native.ptr_array(ptrs), _native.u64_array(caps),
                                            _native.ptr_array(offs), _dptr(st), _stream_handle(codec.device, stream)),
                  "sym_flat_decode")
    return [c[:n] if isinstance(c, torch.Tensor) else c for c in cols], st[:n]


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

"""Device-resident batched Symphony codec over torch tensors.

PyTorch is plumbing here: it owns device memory and the current HIP stream; every
byte is produced by the gfx950 kernels behind the C ABI (arpc_amd/csrc).

Layout (matches include/symphony_hip.h): a string field is a uint8 column plus an
int64 offset tensor of n+1 entries (uint64 on the C side); an int32 field is an
int32 column; the encoded stream is a uint8 tensor plus its n+1 record offsets.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _native, schemas


def _stream_handle(device: torch.device, stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream


def _dptr(t: torch.Tensor | None) -> int:
    return 0 if t is None or t.numel() == 0 else t.data_ptr()


def _check_col(t: torch.Tensor, dtype, what: str, device: torch.device):
    if t.dtype != dtype:
        raise TypeError(f"{what}: expected {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{what}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")


@dataclass
class EncodedBatch:
    data: torch.Tensor     # uint8 [total]
    offsets: torch.Tensor  # int64 [n+1]


@dataclass
class DecodedBatch:
    fixed: list            # int32 [n] per fixed field
    var: list              # (uint8 column, int64 offsets [n+1]) per string field
    status: torch.Tensor   # uint8 [n], SYM_STATUS_*


class Codec:
    """One C-ABI context (decode workspace + device error word) bound to one GPU.

    Not safe for concurrent calls from several threads: use one Codec per thread/stream.
    """

    def __init__(self, device: int | torch.device = 0):
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("Codec needs a GPU device")
        self._lib = _native.lib()
        h = ctypes.c_void_p()
        _native.check(self._lib.sym_ctx_create(self.device.index or 0, ctypes.byref(h)), "sym_ctx_create")
        self._ctx = h

    def branch(self, i: int):
        """(ctx, stream) of concurrent branch i (created on first use): a context of its own (decode
        workspace, error word) and a stream, for a tree walk's independent subtrees (arpc_amd/flat.py).
        check() covers the branches' error words too."""
        br = self.__dict__.setdefault("_branches", [])
        while len(br) <= i:
            h = ctypes.c_void_p()
            _native.check(self._lib.sym_ctx_create(self.device.index or 0, ctypes.byref(h)), "sym_ctx_create")
            br.append((h, torch.cuda.Stream(self.device)))
        return br[i]

    def close(self):
        for h, _ in self.__dict__.get("_branches", []):
            self._lib.sym_ctx_destroy(h)
        self.__dict__["_branches"] = []
        if getattr(self, "_ctx", None):
            self._lib.sym_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, max_records: int):
        _native.check(self._lib.sym_ctx_reserve(self._ctx, max_records), "sym_ctx_reserve")

    def check(self, stream=None):
        """Synchronize and raise if a call reported a device-side error (capacity, unplaceable batch)."""
        _native.check(self._lib.sym_ctx_check(self._ctx, _stream_handle(self.device, stream)), "sym_ctx_check")
        for h, st in self.__dict__.get("_branches", []):
            _native.check(self._lib.sym_ctx_check(h, st.cuda_stream), "sym_ctx_check")

    def set_decode_impl(self, impl: int):
        """SYM_DECODE_PIPELINE (default), SYM_DECODE_THREE_KERNEL or SYM_DECODE_LOOKBACK (same results)."""
        _native.check(self._lib.sym_ctx_set_decode_impl(self._ctx, impl), "sym_ctx_set_decode_impl")

    def decode_redos(self, stream=None) -> int:
        """Re-decodes the speculative decode's gate has run on this ctx so far (synchronizes `stream`)."""
        import ctypes
        v = ctypes.c_uint64(0)
        _native.check(self._lib.sym_ctx_decode_redos(self._ctx, _stream_handle(self.device, stream), ctypes.byref(v)),
                      "sym_ctx_decode_redos")
        return int(v.value)

    def set_encode_impl(self, impl: int):
        """Mixed Get/Set encodes' size scan: SYM_ENCODE_PIPELINE (default), SYM_ENCODE_THREE_KERNEL or
        SYM_ENCODE_LOOKBACK (same results)."""
        _native.check(self._lib.sym_ctx_set_encode_impl(self._ctx, impl), "sym_ctx_set_encode_impl")

    # ------------------------------------------------------------------ encode
    def encode(self, schema: schemas.Schema | str, fixed, var, service_id: int = 0, method_id: int = 0,
               out: torch.Tensor | None = None, out_off: torch.Tensor | None = None,
               var_total: int | None = None, stream=None) -> EncodedBatch:
        """Marshal n records (n = len(offsets) - 1).  `var_total` (sum of string bytes) avoids a sync
        when `out` is not given."""
        s = schemas.BY_NAME[schema] if isinstance(schema, str) else schema
        if len(fixed) != s.nfixed or len(var) != s.nvar:
            raise ValueError(f"{s.name}: expected {s.nfixed} int32 and {s.nvar} string columns")
        n = (var[0][1].numel() - 1) if s.nvar else fixed[0].numel()
        for i, c in enumerate(fixed):
            _check_col(c, torch.int32, f"fixed[{i}]", self.device)
            if c.numel() < n:
                raise ValueError(f"fixed[{i}] has {c.numel()} < {n} values")
        for i, (b, o) in enumerate(var):
            _check_col(b, torch.uint8, f"var[{i}] bytes", self.device)
            _check_col(o, torch.int64, f"var[{i}] offsets", self.device)
            if o.numel() != n + 1:
                raise ValueError(f"var[{i}] offsets must have n+1={n + 1} entries")
        if out is None:
            if var_total is None:
                var_total = sum(int(o[-1].item() - o[0].item()) for _, o in var) if n else 0
            out = torch.empty(max(1, n * s.overhead + var_total), dtype=torch.uint8, device=self.device)
        if out_off is None:
            out_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        rc = self._lib.sym_encode(
            self._ctx, s.schema_id, n, _native.ptr_array([_dptr(c) for c in fixed]),
            _native.ptr_array([_dptr(b) if b.numel() else 1 for b, _ in var]),
            _native.ptr_array([_dptr(o) for _, o in var]), service_id, method_id, _dptr(out), _dptr(out_off),
            _stream_handle(self.device, stream))
        _native.check(rc, f"sym_encode({s.name})")
        return EncodedBatch(out, out_off)

    # ------------------------------------------------------------------ decode
    def decode(self, schema: schemas.Schema | str, data: torch.Tensor, rec_off: torch.Tensor,
               caps: list | None = None, outputs: DecodedBatch | None = None, stream=None) -> DecodedBatch:
        """Unmarshal n records (n = len(rec_off) - 1) into packed columns.  Default column capacity is
        rec_off[n] - rec_off[0] (always sufficient; costs one sync to read)."""
        s = schemas.BY_NAME[schema] if isinstance(schema, str) else schema
        _check_col(data, torch.uint8, "data", self.device)
        _check_col(rec_off, torch.int64, "rec_off", self.device)
        n = rec_off.numel() - 1
        if outputs is None:
            if caps is None:
                span = int(rec_off[-1].item() - rec_off[0].item()) if n else 0
                caps = [span] * s.nvar
            outputs = DecodedBatch(
                fixed=[torch.empty(max(1, n), dtype=torch.int32, device=self.device) for _ in range(s.nfixed)],
                var=[(torch.empty(max(1, caps[f]), dtype=torch.uint8, device=self.device),
                      torch.empty(n + 1, dtype=torch.int64, device=self.device)) for f in range(s.nvar)],
                status=torch.empty(max(1, n), dtype=torch.uint8, device=self.device))
        elif caps is None:
            caps = [b.numel() for b, _ in outputs.var]
        rc = self._lib.sym_decode(
            self._ctx, s.schema_id, n, _dptr(data) if data.numel() else 1, _dptr(rec_off),
            _native.ptr_array([_dptr(c) for c in outputs.fixed]),
            _native.ptr_array([_dptr(b) for b, _ in outputs.var]), _native.u64_array(caps),
            _native.ptr_array([_dptr(o) for _, o in outputs.var]), _dptr(outputs.status),
            _stream_handle(self.device, stream))
        _native.check(rc, f"sym_decode({s.name})")
        return outputs


# ------------------------------------------------------------------ mixed Get/Set batches
def _encode_kv_mixed(codec: "Codec", rtype: torch.Tensor, key, val, service_id: int = 0, get_method_id: int = 0,
                     set_method_id: int = 0, out: torch.Tensor | None = None, out_off: torch.Tensor | None = None,
                     out_bytes: int | None = None, stream=None) -> EncodedBatch:
    """A batch of GetRequests (rtype == 0) and SetRequests (else) in one call (sym_encode_kv_mixed).
    key / val: (uint8 column, int64 offsets [n+1]); a GetRequest's value slice is not encoded.
    `out_bytes` (sym_encoded_size_kv_mixed) avoids a host sync when `out` is not given."""
    _check_col(rtype, torch.uint8, "type", codec.device)
    for what, (b, o) in (("key", key), ("val", val)):
        _check_col(b, torch.uint8, f"{what} bytes", codec.device)
        _check_col(o, torch.int64, f"{what} offsets", codec.device)
    n = key[1].numel() - 1
    if val[1].numel() != n + 1 or rtype.numel() < n:
        raise ValueError("type / key / val columns disagree on the record count")
    if out is None:
        if out_bytes is None:
            is_set = (rtype[:n] != 0).to(torch.int64)
            vlen = (val[1][1:] - val[1][:-1]) * is_set
            out_bytes = 22 * n + int((8 * is_set + vlen).sum().item()) + int((key[1][-1] - key[1][0]).item()) if n else 0
        out = torch.empty(max(1, out_bytes), dtype=torch.uint8, device=codec.device)
    if out_off is None:
        out_off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    _native.check(codec._lib.sym_encode_kv_mixed(
        codec._ctx, _dptr(rtype) if n else 1, _dptr(key[0]) if key[0].numel() else 1, _dptr(key[1]),
        _dptr(val[0]) if val[0].numel() else 1, _dptr(val[1]), n, service_id, get_method_id, set_method_id,
        _dptr(out), _dptr(out_off), _stream_handle(codec.device, stream)), "sym_encode_kv_mixed")
    return EncodedBatch(out, out_off)


def _decode_kv_mixed(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, rtype: torch.Tensor,
                     caps: list | None = None, outputs: DecodedBatch | None = None, stream=None) -> DecodedBatch:
    """Unmarshal each record as its type (0 GetRequest, else SetRequest) into a key and a value column
    (empty values for GetRequests), sym_decode_kv_mixed."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    _check_col(rtype, torch.uint8, "type", codec.device)
    n = rec_off.numel() - 1
    if rtype.numel() < n:  # the kernels read type[r] for every record
        raise ValueError(f"type column has {rtype.numel()} entries for {n} records")
    if outputs is None:
        if caps is None:
            span = int(rec_off[-1].item() - rec_off[0].item()) if n else 0
            caps = [span, span]
        outputs = DecodedBatch(fixed=[], var=[(torch.empty(max(1, c), dtype=torch.uint8, device=codec.device),
                                               torch.empty(n + 1, dtype=torch.int64, device=codec.device)) for c in caps],
                               status=torch.empty(max(1, n), dtype=torch.uint8, device=codec.device))
    elif caps is None:
        caps = [b.numel() for b, _ in outputs.var]
    (kb, ko), (vb, vo) = outputs.var
    _native.check(codec._lib.sym_decode_kv_mixed(
        codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), _dptr(rtype) if n else 1, n, _dptr(kb),
        caps[0], _dptr(ko), _dptr(vb), caps[1], _dptr(vo), _dptr(outputs.status), _stream_handle(codec.device, stream)),
        "sym_decode_kv_mixed")
    return outputs


Codec.encode_kv_mixed = _encode_kv_mixed
Codec.decode_kv_mixed = _decode_kv_mixed


@dataclass
class Datagrams:
    wire: torch.Tensor     # uint8 [total bytes]: every serialized DataPacket back to back
    dg_off: torch.Tensor   # int64 [datagrams+1]: datagram j is wire[dg_off[j]:dg_off[j+1]]
    first: torch.Tensor    # int64 [n+1]: record i's first datagram
    wire_off: torch.Tensor  # int64 [n+1]: record i's first wire byte
    status: torch.Tensor   # uint8 [n]: SYM_FRAG_*


def _fragment(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, rpc_id: torch.Tensor,
              packet_type: int = _native.SYM_PACKET_REQUEST, dst=((127, 0, 0, 1), 9000), src=((127, 0, 0, 1), 9001),
              max_udp_payload: int = _native.SYM_MAX_UDP_PAYLOAD, stream=None) -> Datagrams:
    """aRPC's send side (FragmentPackets + DataPacket framing, pkg/transport/transport.go:146-201) for n
    marshalled records; one sync between the plan and the write (the output size depends on the data)."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    _check_col(rpc_id, torch.int64, "rpc_id", codec.device)
    n = rec_off.numel() - 1
    if rpc_id.numel() < n:
        raise ValueError(f"rpc_id has {rpc_id.numel()} < {n} entries")
    dev, sh = codec.device, _stream_handle(codec.device, stream)
    first = torch.empty(n + 1, dtype=torch.int64, device=dev)
    wire_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    status = torch.empty(max(1, n), dtype=torch.uint8, device=dev)
    _native.check(codec._lib.sym_fragment_plan(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                              max_udp_payload, _dptr(first), _dptr(wire_off), _dptr(status), sh),
                  "sym_fragment_plan")
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    s.synchronize()
    total_dg, total = int(first[n].item()), int(wire_off[n].item())
    wire = torch.empty(max(1, total), dtype=torch.uint8, device=dev)
    dg_off = torch.empty(total_dg + 1, dtype=torch.int64, device=dev)
    ep = _native.Endpoints((ctypes.c_uint8 * 4)(*dst[0]), dst[1], (ctypes.c_uint8 * 4)(*src[0]), src[1])
    _native.check(codec._lib.sym_fragment_write(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                               max_udp_payload, packet_type, _dptr(rpc_id), ctypes.byref(ep),
                                               _dptr(first), _dptr(wire_off), _dptr(status), _dptr(wire),
                                               _dptr(dg_off), sh), "sym_fragment_write")
    return Datagrams(wire[:total] if total else wire[:0], dg_off, first, wire_off, status[:n])


Codec.fragment = _fragment


_FIXED_DTYPE = {1: torch.uint8, 4: torch.int32, 8: torch.int64}


def _raw_get_fixed(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, table_off: int, width: int = 4,
                   segment: int = _native.SYM_SEGMENT_PUBLIC, stream=None):
    """One fixed-width Raw getter over n buffers (main.go:1260-1294).  Returns (values, status):
    uint8 / int32 / int64 [n] for width 1 / 4 / 8 (reinterpret for uint32, float, double), and uint8
    [n] SYM_RAW_* (private fields: the complete-buffer assertion Go panics on)."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    if width not in _FIXED_DTYPE:
        raise ValueError(f"width {width}: fixed fields are 1, 4 or 8 bytes")
    n = rec_off.numel() - 1
    out = torch.empty(max(1, n), dtype=_FIXED_DTYPE[width], device=codec.device)
    status = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    _native.check(codec._lib.sym_raw_get_fixed(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                              segment, table_off, width, _dptr(out), _dptr(status),
                                              _stream_handle(codec.device, stream)), "sym_raw_get_fixed")
    return out[:n], status[:n]


def _raw_get_bytes(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, table_off: int,
                   segment: int = _native.SYM_SEGMENT_PUBLIC, cap: int | None = None, stream=None):
    """One string / bytes Raw getter over n buffers (main.go:1517-1565).  Returns (values uint8,
    offsets int64 [n+1], status uint8 [n]).  `cap` bounds the value bytes (default: the input's
    size, which always suffices; no host sync).  The values tensor has `cap` bytes: its first
    offsets[n] are the values."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    n = rec_off.numel() - 1
    if cap is None:
        cap = data.numel()
    out = torch.empty(max(1, cap), dtype=torch.uint8, device=codec.device)
    offs = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    status = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    _native.check(codec._lib.sym_raw_get_bytes(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                              segment, table_off, _dptr(out), cap, _dptr(offs), _dptr(status),
                                              _stream_handle(codec.device, stream)), "sym_raw_get_bytes")
    return out, offs, status[:n]


@dataclass
class Filtered:
    score: torch.Tensor       # int32 [n]: GetScore of every buffer
    verdict: torch.Tensor     # uint8 [n]: SYM_VERDICT_PASS / SYM_VERDICT_DROP
    kept: torch.Tensor        # uint8 [>= kept bytes]: the passing buffers back to back
    kept_off: torch.Tensor    # int64 [n+1]: the first nkept+1 entries are the kept buffers' offsets
    kept_index: torch.Tensor  # int64 [n]: the first nkept entries are their input positions
    nkept: torch.Tensor       # int64 [1] (device)


def _firewall(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, block_threshold: int,
              score_table_off: int = _native.SYM_PUBLIC_TABLE_START, stream=None) -> Filtered:
    """FirewallElement.ProcessRequest (cmd/proxy/element/firewall.go:39-52) over n buffered requests,
    device-resident and without a host sync."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    n = rec_off.numel() - 1
    dev = codec.device
    score = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    verdict = torch.empty(max(1, n), dtype=torch.uint8, device=dev)
    kept = torch.empty(max(1, data.numel()), dtype=torch.uint8, device=dev)
    kept_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    kept_index = torch.empty(max(1, n), dtype=torch.int64, device=dev)
    nkept = torch.empty(1, dtype=torch.int64, device=dev)
    _native.check(codec._lib.sym_firewall_filter(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                                score_table_off, block_threshold, _dptr(score), _dptr(verdict),
                                                _dptr(kept), data.numel(), _dptr(kept_off), _dptr(kept_index),
                                                _dptr(nkept), _stream_handle(dev, stream)), "sym_firewall_filter")
    return Filtered(score[:n], verdict[:n], kept, kept_off, kept_index[:n], nkept)


@dataclass
class Messages:
    data: torch.Tensor     # uint8 [>= message bytes]: completed messages back to back
    offsets: torch.Tensor  # int64 [n+1]: the first nmsg+1 entries are the message offsets
    rpc_id: torch.Tensor   # int64 [n]: the first nmsg entries are their RPCIDs
    dgram: torch.Tensor    # int64 [n]: ... and the arrival index of each one's completing datagram
    nmsg: torch.Tensor     # int64 [1] (device)
    status: torch.Tensor   # uint8 [n]: SYM_RX_* per datagram


def _reassemble(codec: "Codec", wire: torch.Tensor, dg_off: torch.Tensor, cap: int | None = None,
                stream=None) -> Messages:
    """UDPTransport.Receive + DataReassembler.ProcessFragment (pkg/transport/transport.go:253-317,
    fragmentation.go:49-183) over n datagrams in arrival order, device-resident, no host sync.
    `cap` bounds the message bytes (default: the wire size, which always suffices)."""
    _check_col(wire, torch.uint8, "wire", codec.device)
    _check_col(dg_off, torch.int64, "dg_off", codec.device)
    n = dg_off.numel() - 1
    dev = codec.device
    cap = wire.numel() if cap is None else cap
    data = torch.empty(max(1, cap), dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    rpc = torch.empty(max(1, n), dtype=torch.int64, device=dev)
    dg = torch.empty(max(1, n), dtype=torch.int64, device=dev)
    nmsg = torch.empty(1, dtype=torch.int64, device=dev)
    status = torch.empty(max(1, n), dtype=torch.uint8, device=dev)
    _native.check(codec._lib.sym_reassemble(codec._ctx, _dptr(wire) if wire.numel() else 1, _dptr(dg_off), n,
                                           _dptr(data), cap, _dptr(offs), _dptr(rpc), _dptr(dg), _dptr(nmsg),
                                           _dptr(status), _stream_handle(dev, stream)), "sym_reassemble")
    return Messages(data, offs, rpc[:n], dg[:n], nmsg, status[:n])


Codec.reassemble = _reassemble


@dataclass
class Sealed:
    data: torch.Tensor     # uint8 [>= offsets[n]]
    offsets: torch.Tensor  # int64 [n+1]
    status: torch.Tensor   # uint8 [n]: SYM_CRYPT_*


def _check_key(k: bytes, what: str) -> bytes:
    k = bytes(k)
    if len(k) != 32:
        raise ValueError(f"{what}: AES-256 keys are 32 bytes, got {len(k)}")
    return k


def _encrypt(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, nonces: torch.Tensor, public_key: bytes,
             private_key: bytes, stream=None) -> Sealed:
    """EncryptSymphonyData (pkg/transport/encryption.go:82-171) over n records; nonces: uint8 [n, 24]
    (public, then private), the random draw of encryption.go:115-121 made an input.  No host sync."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    _check_col(nonces, torch.uint8, "nonces", codec.device)
    n = rec_off.numel() - 1
    if nonces.numel() < 24 * n:
        raise ValueError(f"nonces: need 24 bytes per record ({24 * n}), got {nonces.numel()}")
    out = torch.empty(max(1, data.numel() + 2 * _native.SYM_GCM_OVERHEAD * n), dtype=torch.uint8, device=codec.device)
    off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    st = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    _native.check(codec._lib.sym_encrypt(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                        _check_key(public_key, "public_key"), _check_key(private_key, "private_key"),
                                        _dptr(nonces) if n else 1, _dptr(out), _dptr(off), _dptr(st),
                                        _stream_handle(codec.device, stream)), "sym_encrypt")
    return Sealed(out, off, st[:n])


def _decrypt(codec: "Codec", data: torch.Tensor, rec_off: torch.Tensor, public_key: bytes, private_key: bytes,
             stream=None) -> Sealed:
    """DecryptSymphonyData (pkg/transport/encryption.go:183-256) over n records.  A record that fails
    authentication keeps its size and is zero-filled; status says why.  No host sync."""
    _check_col(data, torch.uint8, "data", codec.device)
    _check_col(rec_off, torch.int64, "rec_off", codec.device)
    n = rec_off.numel() - 1
    out = torch.empty(max(1, data.numel()), dtype=torch.uint8, device=codec.device)
    off = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    st = torch.empty(max(1, n), dtype=torch.uint8, device=codec.device)
    _native.check(codec._lib.sym_decrypt(codec._ctx, _dptr(data) if data.numel() else 1, _dptr(rec_off), n,
                                        _check_key(public_key, "public_key"), _check_key(private_key, "private_key"),
                                        _dptr(out), _dptr(off), _dptr(st), _stream_handle(codec.device, stream)),
                  "sym_decrypt")
    return Sealed(out, off, st[:n])


Codec.encrypt = _encrypt
Codec.decrypt = _decrypt
Codec.raw_get_fixed = _raw_get_fixed
Codec.raw_get_bytes = _raw_get_bytes
Codec.firewall = _firewall


def to_device(batch, device) -> tuple[list, list]:
    """datagen.Batch (numpy) -> (fixed int32 tensors, [(uint8 tensor, int64 offsets tensor)]) on device."""
    fixed = [torch.from_numpy(c).to(device) for c in batch.fixed]
    var = []
    for b, o in batch.var:
        bt = torch.from_numpy(b) if b.size else torch.zeros(1, dtype=torch.uint8)
        var.append((bt.to(device), torch.from_numpy(o.view("int64")).to(device)))
    return fixed, var

"""Host-side mirror of aRPC's proxy element interface for batches of buffered packets.

Reference (Go):
  type RPCElement interface {                                   cmd/proxy/element.go:9-19
      ProcessRequest(ctx, *BufferedPacket) (*BufferedPacket, PacketVerdict, ctx, error)
      ProcessResponse(ctx, *BufferedPacket) (*BufferedPacket, PacketVerdict, ctx, error)
      Name() string
  }
  FirewallElement{blockThreshold}; ProcessRequest drops a request whose
  kv.GetRequestRaw(payload).GetScore() >= blockThreshold        cmd/proxy/element/firewall.go:20-52
  PacketVerdictPass = 1, PacketVerdictDrop = 2                  cmd/proxy/util/packet.go:51-62
  XxxRaw getters (zero-copy field reads)                        kv-store-symphony-element kv.syn.go:285-335,
                                                                generator main.go:984-1099

Here a call handles n buffered packets at once on the GPU: `Packets` is the batch (payload bytes
back to back + n+1 offsets, device-resident), ProcessRequest returns the passing packets as a new
batch (unchanged bytes, input order) plus one verdict per input packet.  Go's per-packet
ErrPacketBlocked is the DROP verdict.  Getters return device columns; a private getter on a
public-only buffer, where Go panics, reports SYM_RAW_PUBLIC_ONLY / SYM_RAW_INVALID_BUFFER in the
status column and reads zero / empty.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _native
from .codec import Codec, Filtered

PUBLIC, PRIVATE = _native.SYM_SEGMENT_PUBLIC, _native.SYM_SEGMENT_PRIVATE
PASS, DROP = _native.SYM_VERDICT_PASS, _native.SYM_VERDICT_DROP


@dataclass(frozen=True)
class RawField:
    """A field as the generated Raw getter addresses it: its segment, its table offset (absolute
    from 13 for public fields, relative to the private segment from 1 for private ones) and its
    width (1, 4, 8; 0 = string / bytes).  main.go:986-989, 1243-1257."""
    name: str
    segment: int
    table_off: int
    width: int


def _element_fields(private_strings):
    return (RawField("Score", PUBLIC, 13, 4), RawField("Username", PUBLIC, 17, 0),
            *(RawField(nm, PRIVATE, 1 + 4 * k, 0) for k, nm in enumerate(private_strings)))


# benchmark/kv-store-symphony-element/symphony/kv.proto:18-41 (score, username public)
ELEMENT_SCHEMAS = {
    "GetRequest": _element_fields(["Key"]),
    "GetResponse": _element_fields(["Value"]),
    "SetRequest": _element_fields(["Key", "Value"]),
    "SetResponse": _element_fields(["Value"]),
}


@dataclass
class Packets:
    """n buffered packets (util.BufferedPacket.Payload each) on one device."""
    payload: torch.Tensor  # uint8
    offsets: torch.Tensor  # int64 [n+1]

    @property
    def n(self) -> int:
        return self.offsets.numel() - 1


def field(schema: str, name: str) -> RawField:
    for f in ELEMENT_SCHEMAS[schema]:
        if f.name == name:
            return f
    raise KeyError(f"{schema} has no field {name}")


def get(codec: Codec, packets: Packets, f: RawField, stream=None):
    """XxxRaw.GetF over the batch -> (values, status) for fixed fields, (bytes, offsets, status) for
    string / bytes fields."""
    if f.width:
        return codec.raw_get_fixed(packets.payload, packets.offsets, f.table_off, f.width, f.segment, stream=stream)
    return codec.raw_get_bytes(packets.payload, packets.offsets, f.table_off, f.segment, stream=stream)


class FirewallElement:
    """cmd/proxy/element/firewall.go: blocks requests whose public Score >= block_threshold."""

    def __init__(self, block_threshold: int, codec: Codec, score_field: RawField = ELEMENT_SCHEMAS["GetRequest"][0]):
        if score_field.segment != PUBLIC or score_field.width != 4:
            raise ValueError("the firewall reads a public int32 score")
        self.block_threshold = int(block_threshold)
        self.codec = codec
        self.score_field = score_field

    def should_block(self, score: torch.Tensor) -> torch.Tensor:
        """shouldBlock (firewall.go:34-36), elementwise."""
        return score >= self.block_threshold

    def process_request_filtered(self, packets: Packets, stream=None) -> Filtered:
        """Scores, verdicts and the compacted passing batch, all device-resident, no host sync."""
        return self.codec.firewall(packets.payload, packets.offsets, self.block_threshold,
                                   self.score_field.table_off, stream=stream)

    def process_request(self, packets: Packets, stream=None) -> tuple[Packets, torch.Tensor]:
        """ProcessRequest (firewall.go:39-52) over the batch -> (passing packets, verdict per input).
        Syncs once to size the returned batch."""
        r = self.process_request_filtered(packets, stream)
        k = int(r.nkept.item())
        return Packets(r.kept[:int(r.kept_off[k].item())] if k else r.kept[:0], r.kept_off[:k + 1]), r.verdict

    def process_response(self, packets: Packets, stream=None) -> tuple[Packets, torch.Tensor]:
        """ProcessResponse (firewall.go:54-58): every response passes unchanged."""
        return packets, torch.full((packets.n,), PASS, dtype=torch.uint8, device=packets.payload.device)

    def name(self) -> str:
        return "FirewallElement"

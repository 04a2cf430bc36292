"""Flat Symphony schemas served by the HIP codec.

A schema here is `nfixed` int32 fields followed by `nvar` string/bytes fields, in
declaration order -- the shape of every message on the hot path:

  kv_get_request   GetRequest{Key}           benchmark/kv-store-symphony/symphony/kv.syn.go:74-185
  kv_get_response  GetResponse{Value}        kv.syn.go:333-444
  kv_set_request   SetRequest{Key, Value}    kv.syn.go:611-745
  kv_set_response  SetResponse{Value}        kv.syn.go:963-1074
  echo_request     EchoRequest{Id, Score, Username, Content}
                                             examples/echo_symphony/symphony/echo.syn.go:111-263
  echo_response    EchoResponse (same fields as EchoRequest, echo.proto)

Fixed overhead per record (header 13 + private version 1 + table + length prefixes):
  14 + 4*(nfixed + nvar) + 4*nvar bytes.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Schema:
    name: str
    go_type: str
    fixed_fields: tuple
    var_fields: tuple
    schema_id: int  # matches SYM_SCHEMA_* in include/symphony_hip.h

    @property
    def nfixed(self) -> int:
        return len(self.fixed_fields)

    @property
    def nvar(self) -> int:
        return len(self.var_fields)

    @property
    def fields(self) -> tuple:
        return self.fixed_fields + self.var_fields

    @property
    def overhead(self) -> int:
        return 14 + 4 * (self.nfixed + self.nvar) + 4 * self.nvar

    def record_size(self, var_lens) -> int:
        return self.overhead + sum(var_lens)


KV_GET_REQUEST = Schema("kv_get_request", "GetRequest", (), ("Key",), 0)
KV_SET_REQUEST = Schema("kv_set_request", "SetRequest", (), ("Key", "Value"), 1)
KV_GET_RESPONSE = Schema("kv_get_response", "GetResponse", (), ("Value",), 2)
KV_SET_RESPONSE = Schema("kv_set_response", "SetResponse", (), ("Value",), 3)
ECHO_REQUEST = Schema("echo_request", "EchoRequest", ("Id", "Score"), ("Username", "Content"), 4)
ECHO_RESPONSE = Schema("echo_response", "EchoResponse", ("Id", "Score"), ("Username", "Content"), 5)

ALL = (KV_GET_REQUEST, KV_SET_REQUEST, KV_GET_RESPONSE, KV_SET_RESPONSE, ECHO_REQUEST, ECHO_RESPONSE)
BY_NAME = {s.name: s for s in ALL}
BY_GO_TYPE = {s.go_type: s for s in ALL}

"""Writes tests/golden/kats.json and tests/golden/corpora.json.

Two kinds of fixture, kept apart on purpose:

1. kats.json -- known-answer vectors HAND-DERIVED from the generated Go source of the
   reference (no Go toolchain exists here, so nothing can be produced by running it).
   Every expected value below is a literal written from reading the Go code, NOT
   computed by the oracle:
     encode: benchmark/kv-store-symphony/symphony/kv.syn.go:611-678 (SetRequest),
             :74-132 (GetRequest), examples/echo_symphony/symphony/echo.syn.go:111-184;
             IDs patched as pkg/rpc/client.go:267-271 does.
     decode: kv.syn.go:680-745 and echo.syn.go:186-263 -- each adversarial case notes
             which Go branch it takes.
   The encode KATs are the ones listed in SURVEY.md section 8c.

2. corpora.json -- SHA-256 digests of seeded synthetic batches encoded by the CPU
   oracle (regression pins so GPU tests can check full-size batches without
   re-running the oracle).  These are self-consistency pins, not reference pins.

Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

HDR = "010d000000" + "00000000" + "00000000" + "01"  # [0]=1, off2p=13, sid=0, mid=0, [13]=1


def hx(s: str) -> str:
    return s.replace(" ", "")


# ------------------------------------------------------------------ encode KATs
ENCODE_KATS = [
    # name, schema, fixed, fields, sid, mid, expected hex
    ("set_ab_xyz", "kv_set_request", [], ["ab", "xyz"], 0, 0,
     HDR + "09000000 0f000000 02000000 6162 03000000 78797a"),
    ("get_ab", "kv_get_request", [], ["ab"], 0, 0,
     HDR + "05000000 02000000 6162"),
    ("set_empty", "kv_set_request", [], ["", ""], 0, 0,
     HDR + "09000000 0d000000 00000000 00000000"),
    ("echo_alice_bob", "echo_request", [42, 100], ["alice", "Bob"], 0, 0,
     HDR + "2a000000 64000000 11000000 1a000000 05000000 616c696365 03000000 426f62"),
    ("echo_config1", "echo_request", [42, 300], ["alice", "hello world"], 0, 0,
     HDR + "2a000000 2c010000 11000000 1a000000 05000000 616c696365 0b000000 68656c6c6f20776f726c64"),
    # client.go:267-271 patch: KV service 1, Set = method 2, Get = method 1 (kv_arpc.syn.go:11-28)
    ("set_ab_xyz_ids", "kv_set_request", [], ["ab", "xyz"], 1, 2,
     "010d000000" + "01000000" + "02000000" + "01" + "09000000 0f000000 02000000 6162 03000000 78797a"),
    ("get_ab_ids", "kv_get_request", [], ["ab"], 1, 1,
     "010d000000" + "01000000" + "01000000" + "01" + "05000000 02000000 6162"),
    # GetResponse/SetResponse share GetRequest's layout with field Value (kv.syn.go:333-391, :963-1021)
    ("get_response_v", "kv_get_response", [], ["v"], 0, 0, HDR + "05000000 01000000 76"),
    ("set_response_empty", "kv_set_response", [], [""], 0, 0, HDR + "05000000 00000000"),
    # int32 fields are written as uint32(m.Id) two's complement (echo.syn.go:164-167)
    ("echo_negative", "echo_request", [-1, -2147483648], ["", ""], 0, 0,
     HDR + "ffffffff 00000080 11000000 15000000 00000000 00000000"),
]

SET_AB_XYZ = hx(HDR + "09000000 0f000000 02000000 6162 03000000 78797a")


def patch(h: str, byte_off: int, new_hex: str) -> str:
    return h[:2 * byte_off] + new_hex + h[2 * byte_off + len(new_hex):]


# ------------------------------------------------------------------ decode KATs
# (name, schema, input hex, expected status, expected fixed, expected fields)
DECODE_KATS = [
    ("empty", "kv_set_request", "", 1, [], ["", ""]),                       # len < 13 (kv.syn.go:681)
    ("len12", "kv_set_request", "01" * 12, 1, [], ["", ""]),                 # len < 13
    ("bad_version", "kv_set_request", "02" + "00" * 12, 2, [], ["", ""]),    # data[0] != 1 (:686)
    ("off2p_eq_len", "kv_set_request", hx(HDR)[:26], 3, [], ["", ""]),       # 13 >= len 13 (:696)
    ("private_version_2", "kv_set_request", hx(HDR)[:26] + "02", 3, [], ["", ""]),  # data[13] != 1
    ("header_only", "kv_set_request", hx(HDR), 0, [], ["", ""]),             # table entries out of range: skip
    # off2p = 0: data[0] == 1 passes; table at [1:5] reads 0 -> payloadOffset 0 -> skip
    ("off2p_zero", "kv_set_request", "01" + "00000000" + "00" * 8, 0, [], ["", ""]),
    ("valid", "kv_set_request", SET_AB_XYZ, 0, [], ["ab", "xyz"]),
    # value length 4 > the 3 bytes left: len >= po+4+n fails -> Value skipped
    ("value_len_overflow", "kv_set_request", patch(SET_AB_XYZ, 28, "04000000"), 0, [], ["ab", ""]),
    # key offset 0xffffffff: po+4 > len -> Key skipped
    ("key_off_huge", "kv_set_request", patch(SET_AB_XYZ, 14, "ffffffff"), 0, [], ["", "xyz"]),
    # key offset 0 -> payloadOffset stays 0 -> skipped
    ("key_off_zero", "kv_set_request", patch(SET_AB_XYZ, 14, "00000000"), 0, [], ["", "xyz"]),
    # truncated to 25 B: key needs 26+2, value table entry present but payload gone
    ("truncated_25", "kv_set_request", SET_AB_XYZ[:50], 0, [], ["", ""]),
    ("truncated_28", "kv_set_request", SET_AB_XYZ[:56], 0, [], ["ab", ""]),
    # key offset 1 -> po = 14: length = u32(data[14:18]) = 1 (the patched entry itself),
    # key = data[18:19] = 0x0f (low byte of the value's table entry)
    ("key_into_table", "kv_set_request", patch(SET_AB_XYZ, 14, "01000000"), 0, [], ["0f", "xyz"]),
    # key length 0xffffffff: len >= po+4+n fails in 64-bit Go int arithmetic -> skipped
    ("key_len_huge", "kv_set_request", patch(SET_AB_XYZ, 22, "ffffffff"), 0, [], ["", "xyz"]),
    # service/method IDs are ignored by UnmarshalSymphony (kv.syn.go:692-693)
    ("with_ids", "kv_set_request", patch(SET_AB_XYZ, 5, "0100000002000000"), 0, [], ["ab", "xyz"]),
    # trailing garbage after a valid record is ignored
    ("trailing", "kv_set_request", SET_AB_XYZ + "deadbeef", 0, [], ["ab", "xyz"]),
    # off2p = 1 pointing at a 0x01 byte inside offset_to_private itself: [1:5] = 01 00 00 00
    # -> pts = 2, key entry = u32(data[2:6]) = 0 -> skipped; value entry u32(data[6:10])
    ("off2p_one", "kv_set_request", "01" + "01000000" + "00" * 8 + "01", 0, [], ["", ""]),
    # GetRequest: a SetRequest's bytes decode as Key only
    ("get_from_set", "kv_get_request", SET_AB_XYZ, 0, [], ["ab"]),
    # echo: fixed-field bounds return an ERROR (echo.syn.go:223-231), Id kept if already read
    ("echo_header_only", "echo_request", hx(HDR), 4, [0, 0], ["", ""]),
    ("echo_id_only", "echo_request", hx(HDR) + "2a000000", 4, [42, 0], ["", ""]),
    ("echo_ids_no_table", "echo_request", hx(HDR) + "2a000000" + "2c010000", 0, [42, 300], ["", ""]),
]


def as_field_hex(s: str, name: str) -> str:
    # key_into_table stores raw hex; everything else is ASCII text
    return s if name == "key_into_table" and s == "0f" else s.encode().hex()


def make_kats() -> dict:
    enc = [dict(name=n, schema=s, fixed=fx, fields=[f.encode().hex() for f in flds], service_id=sid,
                method_id=mid, expected=hx(e)) for n, s, fx, flds, sid, mid, e in ENCODE_KATS]
    dec = []
    for n, s, inp, st, fx, flds in DECODE_KATS:
        dec.append(dict(name=n, schema=s, input=hx(inp), status=st, fixed=fx,
                        fields=[as_field_hex(f, n) for f in flds]))
    return {"source": "hand-derived from the reference's generated Go code; see make_golden.py",
            "encode": enc, "decode": dec}


def make_corpora() -> dict:
    sys.path.insert(0, ROOT)
    from arpc_amd import datagen  # noqa: E402
    from oracle import oracle  # noqa: E402
    out = {}
    for name, kw in datagen.CORPORA.items():
        batch = datagen.make_batch(**kw)
        data, off = oracle.encode_batch(batch.fixed, batch.var, kw.get("service_id", 0), kw.get("method_id", 0))
        out[name] = dict(params=kw, n=int(len(off) - 1), bytes=int(off[-1]),
                         sha256_stream=hashlib.sha256(data.tobytes()).hexdigest(),
                         sha256_offsets=hashlib.sha256(off.tobytes()).hexdigest())
    return out


def main():
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(make_kats(), f, indent=1)
    with open(os.path.join(HERE, "corpora.json"), "w") as f:
        json.dump(make_corpora(), f, indent=1)


if __name__ == "__main__":
    main()

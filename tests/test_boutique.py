"""The online-boutique workload on the reference's own payloads.

The reference's serialization benchmark (benchmark/serialization/online-boutique/bench_test.go:282-351)
marshals and unmarshals 93,275 JSON payloads of 30 message types with the generated Symphony code
(proto/onlineboutique.syn.go).  tests/golden/boutique_payloads.json.xz holds those payloads as data
(made by tests/golden/make_boutique_payloads.py).  Here:
* CPU: known-answer vectors written out by hand from onlineboutique.syn.go -- CartItem (a string
  before an int32 in the private table, :83-144), Money (int64 units, :Money.MarshalSymphony),
  Cart (repeated nested message, :1361-1457), ListRecommendationsResponse (repeated string),
  Address (four strings then an int32), Empty (:1742-1751) -- reproduced by the restatement
  oracle/nested_ref.py; the fixture's type and message counts;
* GPU: every payload of every type encoded by arpc_amd.flat through arpc_amd.boutique's schemas,
  each record byte-equal to nested_ref.marshal, and decoded back to the same field values
  (nested_ref's fresh-struct defaults), plus the KAT records themselves.
Byte parity with Go stays unpinned beyond these hand-derived vectors (no Go toolchain here).
"""
import json
import lzma
import os
import struct

import numpy as np
import pytest

from arpc_amd import boutique as B
from oracle import nested_ref as ref

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "boutique_payloads.json.xz")
_PACK = {"bool": "<B", "int32": "<i", "uint32": "<I", "float": "<f", "enum": "<i", "int64": "<q", "uint64": "<Q",
         "double": "<d"}


def payloads() -> dict:
    with lzma.open(FIXTURE, "rt", encoding="utf-8") as fh:
        return json.load(fh)["types"]


def ref_rec(schema, obj: dict) -> dict:
    """A payload object (protojson names and rules, loader.go) -> nested_ref's record form."""
    rec = {}
    for f in schema.fields:
        v = obj.get(B.json_name(f.name))
        if f.kind == "message":
            rec[f.name] = [ref_rec(f.message, x) for x in (v or [])] if f.repeated else \
                (None if v is None else ref_rec(f.message, v))
        elif f.repeated and f.kind in ("string", "bytes"):
            rec[f.name] = [s.encode() for s in (v or [])]
        elif f.kind in ("string", "bytes"):
            rec[f.name] = (v or "").encode()
        else:
            rec[f.name] = struct.pack(_PACK[f.kind], B._scalar(f.kind, v))
    return rec


# ------------------------------------------------------------------ hand-derived vectors (CPU)
H = bytes.fromhex
HDR = "01" "0d000000" "00000000" "00000000" "01"  # public version, off2p 13, ids 0, private version
KATS = [
    # CartItem{ProductId "p1", Quantity 7}: table [ProductId @+9][Quantity], then len + "p1"
    ("CartItem", {"product_id": "p1", "quantity": 7}, H(HDR + "09000000" "07000000" "02000000" "7031")),
    # Money{"USD", Units -2, Nanos 750000000}: table [CurrencyCode @+17][Units u64][Nanos u32]
    ("Money", {"currency_code": "USD", "units": "-2", "nanos": 750000000},
     H(HDR + "11000000" "feffffffffffffff" "8017b42c" "03000000" "555344")),
    # Cart{"u", [{a, 2}, {}]}: [UserId @+9][Items @+14]; count 2, then [len][CartItem] per item
    ("Cart", {"user_id": "u", "items": [{"product_id": "a", "quantity": 2}, {}]},
     H(HDR + "09000000" "0e000000" "01000000" "75" "02000000"
       "1b000000" + HDR + "09000000" "02000000" "01000000" "61"
       "1a000000" + HDR + "09000000" "00000000" "00000000")),
    # ListRecommendationsResponse{["p1", "", "xyz"]}: [ProductIds @+5]; count, then [len][bytes] each
    ("ListRecommendationsResponse", {"product_ids": ["p1", "", "xyz"]},
     H(HDR + "05000000" "03000000" "02000000" "7031" "00000000" "03000000" "78797a")),
    # Address{"1 Main", "X", "", "US", 94043}: four string entries, then ZipCode inline at +16
    ("Address", {"street_address": "1 Main", "city": "X", "state": "", "country": "US", "zip_code": 94043},
     H(HDR + "15000000" "1f000000" "24000000" "28000000" "5b6f0100"
       "06000000" "31204d61696e" "01000000" "58" "00000000" "02000000" "5553")),
    # Empty{}: the 14-byte empty message
    ("Empty", {}, H(HDR)),
    # GetQuoteResponse{CostUsd nil}: a nil nested message is a 0 table entry and no payload
    ("GetQuoteResponse", {}, H(HDR + "00000000")),
]


@pytest.mark.parametrize("name,obj,want", KATS, ids=[k[0] for k in KATS])
def test_hand_kats_reproduced_by_the_restatement(name, obj, want):
    s = B.SCHEMAS[name]
    assert ref.marshal(s, ref_rec(s, obj)) == want
    st, rec, _ = ref.unmarshal(s, want)
    assert st == ref.OK and rec == ref_rec(s, obj) | {}


def test_fixture_holds_the_reference_payloads():
    p = payloads()
    assert len(p) == 30 and sum(len(v) for v in p.values()) == 93275
    assert all(name in B.SCHEMAS for name in p)
    assert p["Empty"] == [{}]


def test_payload_fields_are_schema_fields():
    """Every key of every payload object names a field of its schema (no value would be dropped)."""
    def check(schema, obj):
        names = {B.json_name(f.name): f for f in schema.fields}
        assert set(obj) <= set(names), (schema.name, set(obj) - set(names))
        for k, v in obj.items():
            f = names[k]
            if f.kind == "message":
                for x in (v if f.repeated else [v]):
                    check(f.message, x)
    for name, objs in payloads().items():
        for o in objs[:200]:
            check(B.SCHEMAS[name], o)


# ------------------------------------------------------------------ GPU
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def codec(dev):
    from arpc_amd.codec import Codec
    c = Codec(dev)
    yield c
    c.close()


@pytest.fixture(scope="module")
def all_payloads():
    return payloads()


def _gpu_check(codec, dev, schema, objs):
    from arpc_amd import flat
    from test_nested import from_columns, full
    n = len(objs)
    recs = [ref_rec(schema, o) for o in objs]
    data, off = flat.encode(codec, schema, B.columns_from_json(schema, objs, dev), n=n)
    codec.check()
    got = data.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    for i in range(n):
        want = ref.marshal(schema, recs[i])
        assert got[o[i]:o[i + 1]] == want, (schema.name, i, objs[i])
    cols, st = flat.decode(codec, schema, data, off)
    codec.check()
    assert (st.cpu().numpy() == 0).all()
    assert from_columns(schema, cols, n) == [full(schema, r) for r in recs]


@pytest.mark.gpu
def test_gpu_hand_kats(codec, dev):
    for name, obj, want in KATS:
        s = B.SCHEMAS[name]
        from arpc_amd import flat
        data, off = flat.encode(codec, s, B.columns_from_json(s, [obj, obj], dev), n=2)
        codec.check()
        assert data.cpu().numpy().tobytes() == want + want, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(B.SCHEMAS))
def test_gpu_every_reference_payload(codec, dev, all_payloads, name):
    """All payloads of one type (the whole file): GPU bytes == the restatement's per message, and
    Marshal -> Unmarshal returns the payload's values.  Types without payloads in the reference
    (ListProductsResponse, SearchProductsResponse, AdResponse) get messages built from the
    Product / Ad payloads."""
    s = B.SCHEMAS[name]
    objs = all_payloads.get(name)
    if objs is None:
        inner = {"ListProductsResponse": ("Product", "products"), "SearchProductsResponse": ("Product", "results"),
                 "AdResponse": ("Ad", "ads")}[name]
        pool = all_payloads[inner[0]]
        rng = np.random.default_rng(len(name))
        objs = []
        for k in range(500):
            c = int(rng.integers(0, 6))
            objs.append({inner[1]: [pool[int(j)] for j in rng.integers(0, len(pool), c)]} if c else {})
    _gpu_check(codec, dev, s, objs)

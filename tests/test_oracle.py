"""The CPU oracle against the hand-derived known-answer vectors (tests/golden/kats.json).

Mirrors the reference's own test strategy -- round trips as in
cmd/symphony-gen-arpc/test/serialization_test.go:19-38 (runRoundTrip) and the
determinism check of examples/echo_symphony/echo_symphony_example.go:52-60 -- plus
byte-level KATs, which the reference does not have.
"""
import hashlib

import numpy as np
import pytest

from arpc_amd import datagen, schemas
from oracle import oracle


def _decode_fields(k):
    return [bytes.fromhex(f) for f in k["fields"]]


def test_encode_kats(kats):
    for k in kats["encode"]:
        fields = [bytes.fromhex(f) for f in k["fields"]]
        got = oracle.marshal(k["fixed"], fields, k["service_id"], k["method_id"])
        assert got.hex() == k["expected"], k["name"]


def test_decode_kats(kats):
    for k in kats["decode"]:
        s = schemas.BY_NAME[k["schema"]]
        st, fx, flds = oracle.unmarshal(s.nfixed, s.nvar, bytes.fromhex(k["input"]))
        assert st == k["status"], k["name"]
        assert fx == k["fixed"], k["name"]
        assert flds == _decode_fields(k), k["name"]


def test_encode_kats_roundtrip(kats):
    """Marshal -> Unmarshal -> equal (serialization_test.go:19-38), determinism (echo example :52-60)."""
    for k in kats["encode"]:
        s = schemas.BY_NAME[k["schema"]]
        fields = [bytes.fromhex(f) for f in k["fields"]]
        enc = oracle.marshal(k["fixed"], fields, k["service_id"], k["method_id"])
        st, fx, got = oracle.unmarshal(s.nfixed, s.nvar, enc)
        assert st == 0 and fx == k["fixed"] and got == fields
        assert oracle.marshal(fx, got, k["service_id"], k["method_id"]) == enc


@pytest.mark.parametrize("name", sorted(datagen.CORPORA))
def test_corpora_digests(corpora, name):
    kw = datagen.CORPORA[name]
    b = datagen.make_batch(**kw)
    data, off = oracle.encode_batch(b.fixed, b.var, kw.get("service_id", 0), kw.get("method_id", 0))
    pin = corpora[name]
    assert int(off[-1]) == pin["bytes"] == b.encoded_size()
    assert hashlib.sha256(data.tobytes()).hexdigest() == pin["sha256_stream"]
    assert hashlib.sha256(off.tobytes()).hexdigest() == pin["sha256_offsets"]


@pytest.mark.parametrize("name", ["set_mixed", "set_tiny", "echo_small", "get_response_mixed"])
def test_batch_roundtrip(name):
    kw = datagen.CORPORA[name]
    b = datagen.make_batch(**kw)
    data, off = oracle.encode_batch(b.fixed, b.var)
    fixed, var, status = oracle.decode_batch(b.schema.nfixed, b.schema.nvar, data, off)
    assert not status.any()
    for f in range(b.schema.nfixed):
        np.testing.assert_array_equal(fixed[f], b.fixed[f])
    for f in range(b.schema.nvar):
        np.testing.assert_array_equal(var[f][0], b.var[f][0])
        np.testing.assert_array_equal(var[f][1], b.var[f][1] - b.var[f][1][0])


def test_record_layout_matches_batch():
    """Batch encoder == concatenation of single-record marshals, offsets affine."""
    b = datagen.make_batch(**datagen.CORPORA["set_tiny"])
    data, off = oracle.encode_batch(b.fixed, b.var)
    (kb, ko), (vb, vo) = b.var
    for i in range(0, b.n, 97):
        rec = oracle.marshal([], [kb[ko[i]:ko[i + 1]].tobytes(), vb[vo[i]:vo[i + 1]].tobytes()])
        assert data[off[i]:off[i + 1]].tobytes() == rec
        assert int(off[i]) == 30 * i + int(ko[i]) + int(vo[i])


def test_decode_batch_status_and_packing():
    """Adversarial records in one batch: statuses per record, skipped fields packed as empty."""
    recs = [bytes.fromhex(k) for k in ("", "01" * 12, "02" + "00" * 12)]
    good = oracle.marshal([], [b"key", b"value"])
    recs += [good, good[:25], good + b"\xff"]
    rec_off = np.zeros(len(recs) + 1, dtype=np.uint64)
    np.cumsum([len(r) for r in recs], out=rec_off[1:])
    stream = np.frombuffer(b"".join(recs), dtype=np.uint8)
    _, var, status = oracle.decode_batch(0, 2, stream, rec_off)
    assert status.tolist() == [1, 1, 2, 0, 0, 0]
    keys = [var[0][0][var[0][1][i]:var[0][1][i + 1]].tobytes() for i in range(len(recs))]
    assert keys == [b"", b"", b"", b"key", b"", b"key"]

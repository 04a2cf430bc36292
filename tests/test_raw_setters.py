"""Batched Raw setters: XxxRaw.SetF on n buffers.

Reference: generator cmd/symphony-gen-arpc/protoc-gen-symphony/main.go:1038-1093 (assertions),
:1296-1336 (fixed), :1567-1620 (string / bytes), :1685-1740 (repeated fixed), :371-437 (remarshal);
generated e.g. benchmark/kv-store-symphony-element/symphony/kv.syn.go:340-412.  The reference's own
sequences (cmd/symphony-gen-arpc/test/serialization_test.go:56-128 TestFixed/Raw_Lifecycle_AllFields,
:140-174 TestVar/Raw_Mutation_Lifecycle, :555-703 TestPublicPrivateAccessControl) are replayed here,
with the bytes after each step written out by hand from the generator's layout, against the oracle
(oracle/flat_oracle.c sym_oracle_raw_set) and, on the GPU, against sym_raw_set through the C ABI.
"""
import struct

import numpy as np
import pytest

from oracle import oracle

REP = oracle.REPEATED
FIXED = [(0, 4), (1, 8), (0, 4), (1, 8), (0, 1), (1, 4), (0, 8)]  # test.proto:13-22
VAR = [(0, 0), (1, 0)]                                               # test.proto:25-28


def one(rec: bytes):
    return np.frombuffer(rec, np.uint8).copy(), np.array([0, len(rec)], np.uint64)


def fixed_zero() -> bytes:
    """Fixed{} marshalled: 17 public bytes inline at 13 (off2p = 30), private at 30."""
    return bytes.fromhex("01" "1e000000" + "00" * 8 + "00" * 17 + "01" + "00" * 20)


def set1(fields, k, rec: bytes, value):
    """One buffer through the oracle setter -> (bytes, status)."""
    d, o = one(rec)
    seg, w = fields[k]
    if w and not w & REP:
        vals = np.frombuffer(value, np.uint8).reshape(1, -1)
    else:
        vals = (np.frombuffer(value, np.uint8).copy(), np.array([0, len(value)], np.uint64))
    out, off, st = oracle.raw_set(fields, k, d, o, vals)
    return out[:int(off[1])].tobytes(), int(st[0])


# ---------------------------------------------------------------- CPU: the oracle against the reference sequences
def test_fixed_raw_lifecycle():
    """serialization_test.go:56-128: private setters on the complete buffer, public setters on the
    public-only prefix; every write lands in place at the field's table offset."""
    data = fixed_zero()
    b, st = set1(FIXED, 1, data, struct.pack("<q", -2**63))     # SetFInt64(MinInt64): off2p + 1
    assert st == oracle.SET_OK and b == data[:31] + struct.pack("<q", -2**63) + data[39:]
    b, st = set1(FIXED, 3, b, struct.pack("<Q", 2**64 - 1))     # SetFUint64(MaxUint64): off2p + 9
    assert st == oracle.SET_OK and b[39:47] == b"\xff" * 8
    b, st = set1(FIXED, 5, b, struct.pack("<f", 1.234))         # SetFFloat(1.234): off2p + 17
    assert st == oracle.SET_OK and b[47:51] == struct.pack("<f", 1.234) and len(b) == 51
    pub = data[:30]                                             # data[:offsetToPrivate]
    for k, v, at in ((0, struct.pack("<i", -2**31), 13), (2, struct.pack("<I", 2**32 - 1), 17),
                     (4, b"\x01", 21), (6, struct.pack("<d", 5.6789), 22)):
        pub, st = set1(FIXED, k, pub, v)
        assert st == oracle.SET_OK and pub[at:at + len(v)] == v and len(pub) == 30


def test_var_raw_mutation_lifecycle():
    """serialization_test.go:140-174: SetVBytes grows a private field of a complete buffer (remarshal:
    bytes [5:13] become 0), SetVString grows a public field of the public-only buffer (remarshal through
    a fake private segment, truncated to the public part, [5:13] restored)."""
    complete = bytes.fromhex("01" "19000000" "00000000" "00000000" "11000000" "04000000" "696e6974"
                             "01" "05000000" "00000000")                       # Var{"init", []}
    got, _ = oracle.flat_encode(VAR, [one(b"init"), one(b"")], 1)
    assert got.tobytes() == complete
    b, st = set1(VAR, 1, complete, b"\x01\x02\x03\x04")
    assert st == oracle.SET_OK
    assert b == bytes.fromhex("01" "19000000" "00000000" "00000000" "11000000" "04000000" "696e6974"
                              "01" "05000000" "04000000" "01020304")
    pub, st = set1(VAR, 0, complete[:25], b"modified_string")
    assert st == oracle.SET_OK
    assert pub == bytes.fromhex("01" "24000000" "00000000" "00000000" "11000000" "0f000000") + b"modified_string"
    # the client's IDs survive a public remarshal, not a private one
    with_ids = complete[:5] + struct.pack("<II", 1, 2) + complete[13:]
    pub2, _ = set1(VAR, 0, with_ids[:25], b"modified_string")
    assert pub2[5:13] == struct.pack("<II", 1, 2)
    priv2, _ = set1(VAR, 1, with_ids, b"\x01\x02\x03\x04")
    assert priv2[5:13] == b"\x00" * 8


def test_in_place_keeps_slack():
    """newLen <= oldLen: length prefix rewritten, new bytes copied, the old tail left as slack."""
    complete = bytes.fromhex("01" "19000000" "00000000" "00000000" "11000000" "04000000" "696e6974"
                             "01" "05000000" "00000000")
    pub, st = set1(VAR, 0, complete[:25], b"ab")
    assert st == oracle.SET_OK and pub == complete[:17] + bytes.fromhex("02000000") + b"ab" + b"it"


def test_access_control_statuses():
    """TestPublicPrivateAccessControl (serialization_test.go:555-703): a public setter on a complete
    buffer and a private setter on a public-only or short buffer panic; the buffer is returned
    unchanged with the panic's status."""
    data = fixed_zero()
    assert set1(FIXED, 0, data, b"\x00" * 4)[1] == oracle.SET_COMPLETE_BUFFER
    assert set1(FIXED, 1, data[:30], b"\x00" * 8)[1] == oracle.SET_PUBLIC_ONLY
    assert set1(FIXED, 1, data[:4], b"\x00" * 8)[1] == oracle.SET_INVALID_BUFFER
    assert set1(FIXED, 0, data[:16], b"\x00" * 4) == (data[:16], oracle.SET_TOO_SHORT)  # "buffer too short"
    b, st = set1(VAR, 0, b"\x01\x05\x00\x00\x00", b"x")
    assert st == oracle.SET_TOO_SHORT and b == b"\x01\x05\x00\x00\x00"


def test_repeated_fixed_setter():
    """TestRepeatedFixed/Raw_GetSet_AllTypes (serialization_test.go:190-275) shape: RepeatedFixed{}
    then SetRInt32({1, 2, 3}) on the complete buffer (count 0 -> 3: remarshal), then a shorter list
    in place."""
    fields = [(1, REP | 4), (0, REP | 8), (1, REP | 4), (0, REP | 8), (1, REP | 4), (0, REP | 8), (1, REP | 1)]
    cols = [one(b"") for _ in fields]
    rec, _ = oracle.flat_encode(fields, cols, 1)
    b, st = set1(fields, 0, rec.tobytes(), struct.pack("<3i", 1, 2, 3))
    assert st == oracle.SET_OK and len(b) == len(rec) + 12
    got, gst = oracle.flat_decode(fields, np.frombuffer(b, np.uint8), np.array([0, len(b)], np.uint64))
    assert gst[0] == 0 and got[0][0].tobytes() == struct.pack("<3i", 1, 2, 3)
    b2, st = set1(fields, 0, b, struct.pack("<i", 9))  # one element: in place, count 1
    assert st == oracle.SET_OK and len(b2) == len(b)
    got, _ = oracle.flat_decode(fields, np.frombuffer(b2, np.uint8), np.array([0, len(b2)], np.uint64))
    assert got[0][0].tobytes() == struct.pack("<i", 9)


def test_repeated_value_not_whole_elements():
    """A repeated int32 value of 6 bytes is not a whole number of elements: Go's typed setters cannot
    express it, and the batch setter reports SET_BAD_LENGTH and copies the buffer unchanged (in place
    and remarshal cases alike), as sym_flat_encode rejects the same column."""
    fields = [(1, REP | 4), (0, REP | 8)]
    rec, _ = oracle.flat_encode(fields, [one(struct.pack("<3i", 1, 2, 3)), one(b"")], 1)
    for v in (b"\x01" * 6, b"\x01" * 13, b"\x07"):
        b, st = set1(fields, 0, rec.tobytes(), v)
        assert st == oracle.SET_BAD_LENGTH and b == rec.tobytes()
    b, st = set1(fields, 0, rec.tobytes(), b"\x01" * 8)  # two whole elements: in place
    assert st == oracle.SET_OK and len(b) == len(rec)


# ---------------------------------------------------------------- batch generators shared with the GPU tests
def make_batch(rng, fields, n):
    """n buffers of `fields`: complete records, public-only prefixes, truncated and corrupted ones."""
    recs = []
    for i in range(n):
        cols = []
        for seg, w in fields:
            if w and not w & REP:
                cols.append(rng.integers(0, 256, (1, w), dtype=np.uint8))
            else:
                ew = (w & ~REP) if w else 1
                ln = int(rng.integers(0, 12)) * ew
                cols.append((rng.integers(0, 256, ln, dtype=np.uint8), np.array([0, ln], np.uint64)))
        rec, _ = oracle.flat_encode(fields, cols, 1)
        r = bytearray(rec.tobytes())
        kind = rng.integers(0, 10)
        if kind < 4:  # public-only prefix
            r = r[:struct.unpack_from("<I", r, 1)[0]]
        elif kind == 4:
            r = r[:int(rng.integers(0, len(r) + 1))]
        elif kind == 5 and len(r) > 13:
            r[int(rng.integers(0, min(len(r), 40)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 6 and len(r) >= 13:
            r[5:13] = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        recs.append(bytes(r))
    off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


def make_values(rng, fields, k, n):
    seg, w = fields[k]
    if w and not w & REP:
        return rng.integers(0, 256, (n, w), dtype=np.uint8)
    ew = (w & ~REP) if w else 1
    ln = (rng.integers(0, 16, n) * ew).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    np.cumsum(ln, out=off[1:])
    return rng.integers(0, 256, int(off[-1]), dtype=np.uint8), off


SCHEMAS = {"Fixed": FIXED, "Var": VAR,
           "Element": [(0, 4), (0, 0), (1, 0), (1, 0)],  # kv-store-symphony-element SetRequest
           "Mixed": [(1, 4), (0, 0), (1, REP | 8), (0, 1), (1, 0), (0, REP | 4)]}


@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_oracle_batch_matches_single_calls(name):
    """The batched oracle equals buffer-by-buffer calls; statuses cover several branches."""
    fields = SCHEMAS[name]
    rng = np.random.default_rng(len(name))
    for k in range(len(fields)):
        data, off = make_batch(rng, fields, 60)
        vals = make_values(rng, fields, k, 60)
        out, ooff, st = oracle.raw_set(fields, k, data, off, vals)
        for i in range(60):
            rec = data[int(off[i]):int(off[i + 1])].tobytes()
            v = vals[i].tobytes() if not isinstance(vals, tuple) else vals[0][int(vals[1][i]):int(vals[1][i + 1])].tobytes()
            b, s = set1(fields, k, rec, v)
            assert s == st[i] and b == out[int(ooff[i]):int(ooff[i + 1])].tobytes()


# ---------------------------------------------------------------- GPU parity
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


def gpu_set(codec, dev, fields, k, data, off, vals):
    from arpc_amd import flat
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    o = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    if isinstance(vals, tuple):
        v = (torch.from_numpy(np.concatenate([vals[0], np.zeros(16, np.uint8)])).to(dev),
             torch.from_numpy(vals[1].view(np.int64).copy()).to(dev))
    else:
        v = torch.from_numpy(np.ascontiguousarray(vals).reshape(-1)).to(dev)
    out, ooff, st = flat.raw_set(codec, fields, k, d, o, v, n=len(off) - 1)
    codec.check()
    ooff = ooff.cpu().numpy().view(np.uint64)
    return out.cpu().numpy()[:int(ooff[-1])], ooff, st.cpu().numpy()


@pytest.mark.gpu
def test_gpu_reference_sequences(codec, dev):
    """The Fixed and Var lifecycles of the reference tests, each buffer repeated across tiles."""
    n = 700
    steps = [(FIXED, 1, fixed_zero(), struct.pack("<q", -2**63)), (FIXED, 6, fixed_zero()[:30], struct.pack("<d", 5.6789)),
             (FIXED, 0, fixed_zero(), b"\x00" * 4),
             (VAR, 1, bytes.fromhex("01190000000000000000000000110000000400000069 6e697401050000000000 0000".replace(" ", "")),
              b"\x01\x02\x03\x04"),
             (VAR, 0, bytes.fromhex("0119000000000000000000000011000000040000 00696e6974".replace(" ", "")), b"modified_string")]
    for fields, k, rec, v in steps:
        data = np.frombuffer(rec * n, np.uint8).copy()  # writable copies throughout
        off = np.arange(n + 1, dtype=np.uint64) * len(rec)
        vals = (np.frombuffer(v * n, np.uint8).copy(), np.arange(n + 1, dtype=np.uint64) * len(v)) \
            if not (fields[k][1] and not fields[k][1] & REP) else np.frombuffer(v * n, np.uint8).reshape(n, -1).copy()
        want, woff, wst = oracle.raw_set(fields, k, data, off, vals)
        got, goff, gst = gpu_set(codec, dev, fields, k, data, off, vals)
        np.testing.assert_array_equal(gst, wst)
        np.testing.assert_array_equal(goff, woff)
        np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_gpu_repeated_value_not_whole_elements(codec, dev):
    """SET_BAD_LENGTH on the GPU: ragged value lengths against a repeated int32 field, in-place and
    remarshal candidates mixed, bit-exact with the oracle."""
    fields = [(1, REP | 4), (0, REP | 8), (1, 0)]
    rng = np.random.default_rng(77)
    n = 900
    data, off = make_batch(rng, fields, n)
    ln = rng.integers(0, 20, n).astype(np.uint64)  # any byte length, most not multiples of 4
    voff = np.zeros(n + 1, np.uint64)
    np.cumsum(ln, out=voff[1:])
    vals = (rng.integers(0, 256, int(voff[-1]), dtype=np.uint8), voff)
    want, woff, wst = oracle.raw_set(fields, 0, data, off, vals)
    assert (wst == oracle.SET_BAD_LENGTH).any() and (wst == oracle.SET_OK).any()
    got, goff, gst = gpu_set(codec, dev, fields, 0, data, off, vals)
    np.testing.assert_array_equal(gst, wst)
    np.testing.assert_array_equal(goff, woff)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SCHEMAS))
def test_gpu_setters_match_oracle(codec, dev, name):
    fields = SCHEMAS[name]
    rng = np.random.default_rng(100 + len(name))
    for k in range(len(fields)):
        n = int(rng.choice([1, 63, 257, 1500]))
        data, off = make_batch(rng, fields, n)
        vals = make_values(rng, fields, k, n)
        want, woff, wst = oracle.raw_set(fields, k, data, off, vals)
        got, goff, gst = gpu_set(codec, dev, fields, k, data, off, vals)
        np.testing.assert_array_equal(gst, wst, err_msg=f"{name} field {k} status")
        np.testing.assert_array_equal(goff, woff, err_msg=f"{name} field {k} offsets")
        np.testing.assert_array_equal(got, want, err_msg=f"{name} field {k} bytes")
        assert n < 50 or ((wst == 0).any() and (wst != 0).any())

"""The reference's own test inputs through the GPU codec (parity as far as the reference pins it).

The reference holds no byte vectors for the current format; its generator tests pin round trips:
cmd/symphony-gen-arpc/test/serialization_test.go:19-38 (runRoundTrip: Marshal -> Unmarshal ->
reflect.DeepEqual) on the messages of cmd/symphony-gen-arpc/test/test.proto:13-80.  Here each of
those inputs is marshalled by the GPU flat codec (sym_flat_encode) and must

  * equal the oracle's bytes (oracle/flat_oracle.c) and the layout written out below by hand from
    the generator (main.go:196-368 marshal: public fields in a table at byte 13 with absolute
    offsets, private ones after the private version byte with offsets relative to it; fixed fields
    inline, little-endian; strings and repeated fixed fields as [u32 length or count][payload]), and
  * unmarshal on the GPU (sym_flat_decode) back to exactly the input values (the reference's
    DeepEqual), bit for bit for floats.

Byte parity with Go itself stays "unpinned": no Go toolchain exists here or on the GPU box and the
reference ships no vectors.  RepeatedVar / nested messages are not covered by the flat codec.
"""
import struct

import numpy as np
import pytest

from oracle import oracle

REP = oracle.REPEATED
FMT = {1: "<?", 4: "<I", 8: "<Q"}

# test.proto:13-22 message Fixed; public = [(Test.is_public) = true]
FIXED_FIELDS = [(0, 4), (1, 8), (0, 4), (1, 8), (0, 1), (1, 4), (0, 8)]
# serialization_test.go:44-52 (TestFixed/Struct_RoundTrip): MinInt32, MinInt64, MaxUint32, MaxUint64,
# true, float32(3.14159), 1.23456789
FIXED_VALUES = [struct.pack("<i", -2**31), struct.pack("<q", -2**63), struct.pack("<I", 2**32 - 1),
                struct.pack("<Q", 2**64 - 1), b"\x01", struct.pack("<f", 3.14159), struct.pack("<d", 1.23456789)]
# test.proto:25-28 message Var; TestVar inputs (:133-136) and the Raw lifecycle origin (:141)
VAR_FIELDS = [(0, 0), (1, 0)]
VAR_VALUES = [[b"Symphony", b"\xff\xaa"], [b"init", b""]]
# test.proto:31-39 message RepeatedFixed; TestRepeatedFixed input (:179-187)
REPF_FIELDS = [(1, REP | 4), (0, REP | 8), (1, REP | 4), (0, REP | 8), (1, REP | 4), (0, REP | 8), (1, REP | 1)]
REPF_VALUES = [struct.pack("<3i", 1, -1, 2**31 - 1), struct.pack("<3q", 100, -100, 2**63 - 1),
               struct.pack("<3I", 0, 100, 2**32 - 1), struct.pack("<3Q", 0, 1000, 2**64 - 1),
               struct.pack("<3f", 1.1, 2.2, -3.3), struct.pack("<3d", 10.01, 20.02, -30.03), b"\x01\x00\x01"]


def hand_marshal(fields, values) -> bytes:
    """The generator's layout written out directly (main.go:196-368, 439-535), for checking the oracle."""
    def seg_bytes(seg, table_start, relative_to):
        items = [(w, v) for (s, w), v in zip(fields, values) if s == seg]
        table = sum(w if w and not w & REP else 4 for w, _ in items)
        tab, pay = b"", b""
        for w, v in items:
            if w and not w & REP:
                tab += v
            else:
                count = len(v) // (w & ~REP) if w else len(v)
                tab += struct.pack("<I", table_start + table + len(pay) - relative_to)
                pay += struct.pack("<I", count) + v
        return tab + pay
    pub = seg_bytes(0, 13, 0)
    off2p = 13 + len(pub)
    priv = seg_bytes(1, off2p + 1, off2p)
    return b"\x01" + struct.pack("<I", off2p) + b"\x00" * 8 + pub + b"\x01" + priv


def cols_of(fields, records):
    """Column layout of test_flat / sym_flat_*: fixed fields as (n, w) u8 rows, payload fields as
    (bytes, offsets)."""
    cols = []
    for k, (_, w) in enumerate(fields):
        vals = [r[k] for r in records]
        if w and not w & REP:
            cols.append(np.frombuffer(b"".join(vals), np.uint8).reshape(len(vals), w).copy())
        else:
            off = np.zeros(len(vals) + 1, np.uint64)
            np.cumsum([len(v) for v in vals], out=off[1:])
            cols.append((np.frombuffer(b"".join(vals), np.uint8).copy(), off))
    return cols


CASES = {"Fixed": (FIXED_FIELDS, [FIXED_VALUES, [b"\x00" * 4, b"\x00" * 8, b"\x00" * 4, b"\x00" * 8, b"\x00",
                                                 b"\x00" * 4, b"\x00" * 8]]),
         "Var": (VAR_FIELDS, VAR_VALUES),
         "RepeatedFixed": (REPF_FIELDS, [REPF_VALUES, [b""] * 7])}


def test_hand_kat_var():
    """Var{VString: "Symphony", VBytes: {0xFF, 0xAA}}: 40 bytes, read off the generator by hand."""
    want = bytes.fromhex("01" "1d000000" "00000000" "00000000" "11000000" "08000000" "53796d70686f6e79"
                         "01" "05000000" "02000000" "ffaa")
    assert hand_marshal(VAR_FIELDS, VAR_VALUES[0]) == want
    got, _ = oracle.flat_encode(VAR_FIELDS, cols_of(VAR_FIELDS, [VAR_VALUES[0]]), 1)
    assert got.tobytes() == want


def test_hand_kat_fixed_extremes():
    """TestFixed's extremes: 17 public bytes inline at 13 (off2p = 30), 20 private after [30]."""
    want = bytes.fromhex("01" "1e000000" "00000000" "00000000" "00000080" "ffffffff" "01" "1bde8342cac0f33f"
                         "01" "0000000000000080" "ffffffffffffffff" "d00f4940")
    assert hand_marshal(FIXED_FIELDS, FIXED_VALUES) == want
    got, _ = oracle.flat_encode(FIXED_FIELDS, cols_of(FIXED_FIELDS, [FIXED_VALUES]), 1)
    assert got.tobytes() == want


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_hand_layout(name):
    fields, values = CASES[name]
    for v in values:
        got, _ = oracle.flat_encode(fields, cols_of(fields, [v]), 1)
        assert got.tobytes() == hand_marshal(fields, v), name


def test_repeated_fixed_offsets_by_hand():
    """RepeatedFixed (test.proto:31-39): public table 25 / 53 / 81, off2p 109, private offsets 17 / 33 / 49 / 65."""
    b = hand_marshal(REPF_FIELDS, REPF_VALUES)
    assert len(b) == 181
    assert struct.unpack_from("<4I", b, 1)[0] == 109
    assert struct.unpack_from("<3I", b, 13) == (25, 53, 81)
    assert b[109] == 1 and struct.unpack_from("<4I", b, 110) == (17, 33, 49, 65)


# ---------------------------------------------------------------- GPU
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


def _schema(fields):
    from arpc_amd import flat
    kinds = {1: "bool", 4: "uint32", 8: "uint64", 0: "bytes"}
    return flat.FlatSchema("ref", tuple(flat.FlatField(f"f{k}", kinds[w & ~REP], seg == 0, bool(w & REP))
                                        for k, (seg, w) in enumerate(fields)))


def _to_dev(cols, fields, dev):
    out = []
    for (_, w), c in zip(fields, cols):
        if w and not w & REP:
            out.append(torch.from_numpy(c.reshape(-1).view({1: np.uint8, 4: np.int32, 8: np.int64}[w]).copy()).to(dev))
        else:
            b = c[0] if c[0].size else np.zeros(1, np.uint8)
            out.append((torch.from_numpy(np.concatenate([b, np.zeros(16, np.uint8)])).to(dev)[:max(1, c[0].size)],
                        torch.from_numpy(c[1].view(np.int64).copy()).to(dev)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_reference_round_trip(codec, dev, name):
    """runRoundTrip on the GPU: each reference input, interleaved with the message's zero value,
    repeated across tiles (3000 records): GPU bytes == oracle == hand layout, and the GPU decode
    returns the inputs exactly (serialization_test.go:19-38's DeepEqual)."""
    from arpc_amd import flat
    fields, values = CASES[name]
    recs = [values[i % len(values)] for i in range(3000)]
    cols = cols_of(fields, recs)
    want, woff = oracle.flat_encode(fields, cols, len(recs))
    sch = _schema(fields)
    data, off = flat.encode(codec, sch, _to_dev(cols, fields, dev), n=len(recs))
    codec.check()
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), woff)
    got = data.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    assert got[:int(woff[1])].tobytes() == hand_marshal(fields, values[0])
    dcols, st = flat.decode(codec, sch, data, off)
    codec.check()
    assert int(st.sum().item()) == 0
    for k, (_, w) in enumerate(fields):
        if w and not w & REP:
            np.testing.assert_array_equal(dcols[k].cpu().numpy().view(np.uint8).reshape(len(recs), w), cols[k])
        else:
            b, o = dcols[k]
            o = o.cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(o, cols[k][1])
            np.testing.assert_array_equal(b.cpu().numpy()[:int(o[-1])], cols[k][0])

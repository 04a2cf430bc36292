"""Any flat schema (the flat part): fixed-width and string fields, public or private.

CPU tests pin the generic restatement (oracle/flat_oracle.c):
  * byte-identical to the kv-store / echo restatement (symphony_oracle.c, pinned by
    tests/golden/kats.json) for those all-private schemas, encode and decode (statuses included)
    on valid and corrupted streams;
  * byte-identical to the element-schema marshal of raw_oracle.c (public Score / Username);
  * the reference access-control test's Fixed message (serialization_test.go:555-703), whose bytes
    tests/test_raw_fields.py restates from the generated MarshalSymphony (test.syn.go:152).
GPU tests compare the HIP flat codec with that oracle on random schemas (up to 16 fields of every
width, both segments), corrupted buffers and edge counts.
"""
import struct

import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle
from test_raw_fields import corrupted_batch, fixed_message

KIND_NP = {1: np.uint8, 4: np.uint32, 8: np.uint64}
REP = oracle.REPEATED  # width | REP: repeated fixed-width field


def scalar(w):
    return bool(w) and not w & REP


def random_schema(rng, nf=None):
    nf = int(rng.integers(0, 17)) if nf is None else nf
    return [(int(rng.integers(0, 2)), int(rng.choice([0, 0, 1, 4, 8, REP | 1, REP | 4, REP | 8]))) for _ in range(nf)]


def random_columns(rng, fields, n):
    cols = []
    for seg, w in fields:
        if scalar(w):
            cols.append(rng.integers(0, 256, (n, w), dtype=np.uint8))
        else:
            ew = w & ~REP if w else 1  # repeated: whole elements
            ln = rng.choice([rng.integers(0, 8, n), rng.integers(0, 200, n)]).astype(np.uint64) // ew * ew
            off = np.zeros(n + 1, np.uint64)
            np.cumsum(ln, out=off[1:])
            cols.append((rng.integers(0, 256, int(off[-1]), dtype=np.uint8), off))
    return cols


def corrupt(data, off, rng, frac=0.3):
    recs = []
    for i in range(len(off) - 1):
        r = bytearray(data[int(off[i]):int(off[i + 1])].tobytes())
        if r and rng.random() < frac:
            kind = rng.integers(0, 4)
            if kind == 0:
                r = r[:int(rng.integers(0, len(r) + 1))]
            elif kind == 1:
                r[int(rng.integers(0, len(r)))] ^= 1 << int(rng.integers(0, 8))
            elif kind == 2 and len(r) >= 5:
                struct.pack_into("<I", r, 1, int(rng.integers(0, len(r) + 4)))
            elif len(r) > 13:
                j = int(rng.integers(13, len(r) - 3)) if len(r) > 16 else 13
                struct.pack_into("<I", r, min(j, len(r) - 4), int(rng.choice([0, 0xFFFFFFFF, rng.integers(0, 600)])))
        recs.append(bytes(r))
    o = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=o[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), o


# ------------------------------------------------------------------ oracle pinning (CPU)
def test_oracle_matches_kv_and_echo_restatement():
    for name, fields in (("set_tiny", [(1, 0), (1, 0)]), ("get_64", [(1, 0)]), ("echo_small", [(1, 4), (1, 4), (1, 0), (1, 0)]),
                         ("set_ids", [(1, 0), (1, 0)])):
        kw = datagen.CORPORA[name]
        b = datagen.make_batch(**kw)
        sid, mid = kw.get("service_id", 0), kw.get("method_id", 0)
        want, woff = oracle.encode_batch(b.fixed, b.var, sid, mid)
        got, goff = oracle.flat_encode(fields, [c.view(np.uint8).reshape(-1, 4) for c in b.fixed] + list(b.var), b.n,
                                       sid, mid)
        assert np.array_equal(got, want) and np.array_equal(goff, woff), name
        # decode of valid and corrupted streams agrees with the kv / echo restatement
        for data, off in ((want, woff), corrupt(want, woff, np.random.default_rng(3))):
            fx, vr, st = oracle.decode_batch(b.schema.nfixed, b.schema.nvar, data, off)
            cols, st2 = oracle.flat_decode(fields, data, off)
            assert np.array_equal(st, st2), name
            for k in range(b.schema.nfixed):
                assert np.array_equal(fx[k], cols[k].view(np.int32).ravel()), name
            for k in range(b.schema.nvar):
                assert np.array_equal(vr[k][0], cols[b.schema.nfixed + k][0]), name
                assert np.array_equal(vr[k][1], cols[b.schema.nfixed + k][1]), name


def test_oracle_matches_element_marshal():
    e = datagen.make_element_batch(500, (("uniform", 0, 20), ("uniform", 0, 30), ("uniform", 0, 90)), 5)
    got, goff = oracle.flat_encode([(0, 4), (0, 0), (1, 0), (1, 0)], [e.score.view(np.uint8).reshape(-1, 4)] + e.strings,
                                   500)
    assert np.array_equal(got, e.data) and np.array_equal(goff, e.rec_off)


FIXED_FIELDS = [(0, 4), (1, 8), (0, 4), (1, 8), (0, 1), (1, 4), (0, 8)]  # test.proto:13-22 (message Fixed)


def fixed_cols(vals):
    fi32, fi64, fu32, fu64, fb, ff, fd = vals
    enc = [("<i", fi32), ("<q", fi64), ("<I", fu32), ("<Q", fu64), ("<?", fb), ("<f", ff), ("<d", fd)]
    return [np.frombuffer(struct.pack(fmt, v), np.uint8).reshape(1, -1).copy() for fmt, v in enc]


def test_oracle_fixed_message_kat():
    got, off = oracle.flat_encode(FIXED_FIELDS, fixed_cols((10, 20, 30, 40, True, 1.5, 2.5)), 1)
    assert got.tobytes() == fixed_message()
    cols, st = oracle.flat_decode(FIXED_FIELDS, got, off)
    assert st[0] == 0 and struct.unpack("<q", cols[1].tobytes())[0] == 20 and struct.unpack("<d", cols[6].tobytes())[0] == 2.5
    # UnmarshalSymphony rejects the public-only buffer (serialization_test.go:692-702)
    _, st = oracle.flat_decode(FIXED_FIELDS, np.frombuffer(fixed_message()[:30], np.uint8), np.array([0, 30], np.uint64))
    assert st[0] == oracle.STATUS_NO_PRIVATE


def test_oracle_repeated_fixed_kats():
    """Repeated fixed-width fields, bytes hand-derived from generateRepeatedFixedFieldMarshal
    (main.go:493-535): a 4-byte table entry, then [u32 count][count elements] in the payload."""
    # message {repeated int32 xs = 1;} xs = [1, -2]: private table entry 5 (relative), count 2
    xs = np.array([1, -2], np.int32).view(np.uint8)
    got, off = oracle.flat_encode([(1, REP | 4)], [(xs, np.array([0, 8], np.uint64))], 1)
    want = bytes.fromhex("01 0d000000 00000000 00000000 01 05000000 02000000 01000000 feffffff".replace(" ", ""))
    assert got.tobytes() == want
    cols, st = oracle.flat_decode([(1, REP | 4)], got, off)
    assert st[0] == 0 and cols[0][0].tobytes() == xs.tobytes()
    # message {repeated uint64 ys = 1 [is_public]; string s = 2;} ys = [7], s = "ab": public
    # segment 13 + 4 + 4 + 8 = 29; public entry absolute 17; private entry (34 - 29) = 5
    ys = np.array([7], np.uint64).view(np.uint8)
    fields = [(0, REP | 8), (1, 0)]
    got, off = oracle.flat_encode(fields, [(ys, np.array([0, 8], np.uint64)),
                                           (np.frombuffer(b"ab", np.uint8), np.array([0, 2], np.uint64))], 1)
    want = bytes.fromhex("01 1d000000 00000000 00000000 11000000 01000000 0700000000000000 01 05000000 02000000 6162"
                         .replace(" ", ""))
    assert got.tobytes() == want
    # decode: a count whose elements run past the end leaves the field empty (:811-813)
    bad = bytearray(want)
    struct.pack_into("<I", bad, 17, 3)  # 17 + 4 + 24 > 40
    cols, st = oracle.flat_decode(fields, np.frombuffer(bytes(bad), np.uint8), np.array([0, len(bad)], np.uint64))
    assert st[0] == 0 and cols[0][0].size == 0 and cols[1][0].tobytes() == b"ab"


def test_oracle_empty_message():
    got, off = oracle.flat_encode([], [], 3)
    assert got.tobytes() == (b"\x01" + struct.pack("<I", 13) + bytes(8) + b"\x01") * 3
    _, st = oracle.flat_decode([], np.frombuffer(got.tobytes() + bytes(13), np.uint8), np.array([0, 14, 28, 42, 55], np.uint64))
    assert list(st) == [0, 0, 0, oracle.STATUS_TOO_SHORT]


# ------------------------------------------------------------------ HIP flat codec (GPU)
@pytest.fixture(scope="module")
def gdev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def gcodec(gdev):
    from arpc_amd.codec import Codec
    c = Codec(gdev)
    yield c
    c.close()


def _schema(fields):
    from arpc_amd import flat
    kinds = {1: "bool", 4: "uint32", 8: "uint64", 0: "bytes"}
    return flat.FlatSchema("random", tuple(flat.FlatField(f"f{k}", kinds[w & ~REP], seg == 0, bool(w & REP))
                                           for k, (seg, w) in enumerate(fields)))


def _to_dev(cols, fields, dev):
    import torch
    out = []
    for (seg, w), c in zip(fields, cols):
        if scalar(w):
            t = torch.from_numpy(np.ascontiguousarray(c).view(KIND_NP[w]).reshape(-1).view(
                {1: np.uint8, 4: np.int32, 8: np.int64}[w]).copy()).to(dev)
            out.append(t)
        else:
            b = torch.from_numpy(c[0].copy() if c[0].size else np.zeros(1, np.uint8)).to(dev)
            out.append((b, torch.from_numpy(c[1].view(np.int64).copy()).to(dev)))
    return out


def _check_decode(codec, dev, fields, data, off):
    import torch
    from arpc_amd import flat
    want_cols, want_st = oracle.flat_decode(fields, data, off)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)[:len(data)] if len(data) else \
        torch.zeros(0, dtype=torch.uint8, device=dev)
    o = torch.from_numpy(off.view(np.int64).copy()).to(dev)
    got_cols, got_st = flat.decode(codec, _schema(fields), d, o)
    codec.check()
    np.testing.assert_array_equal(got_st.cpu().numpy(), want_st, err_msg="status")
    for k, (seg, w) in enumerate(fields):
        if scalar(w):
            np.testing.assert_array_equal(got_cols[k].cpu().numpy().view(np.uint8).reshape(-1, w),
                                          want_cols[k].reshape(-1, w), err_msg=f"fixed field {k}")
        else:
            go = got_cols[k][1].cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(go, want_cols[k][1], err_msg=f"offsets of field {k}")
            np.testing.assert_array_equal(got_cols[k][0][:int(go[-1])].cpu().numpy(), want_cols[k][0],
                                          err_msg=f"bytes of field {k}")


def _check_encode(codec, dev, fields, cols, n, sid=0, mid=0):
    from arpc_amd import flat
    want, woff = oracle.flat_encode(fields, cols, n, sid, mid)
    data, off = flat.encode(codec, _schema(fields), _to_dev(cols, fields, dev), sid, mid, n=n)
    codec.check()
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), woff, err_msg="record offsets")
    np.testing.assert_array_equal(data.cpu().numpy(), want, err_msg="encoded bytes")
    return want, woff


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_flat_random_schemas_gpu(gcodec, gdev, seed):
    rng = np.random.default_rng(seed)
    fields = random_schema(rng, nf=[1, 3, 7, 16, 0, int(rng.integers(2, 17))][seed])
    n = int(rng.choice([1, 257, 3000]))
    cols = random_columns(rng, fields, n)
    data, off = _check_encode(gcodec, gdev, fields, cols, n, sid=seed, mid=seed * 7)
    _check_decode(gcodec, gdev, fields, data, off)
    _check_decode(gcodec, gdev, fields, *corrupt(data, off, rng, frac=0.5))


@pytest.mark.gpu
def test_flat_known_schemas_gpu(gcodec, gdev):
    _check_encode(gcodec, gdev, FIXED_FIELDS, fixed_cols((10, 20, 30, 40, True, 1.5, 2.5)), 1)
    data, off = batch_of([fixed_message(), fixed_message()[:30], b"", b"\x02" * 40])
    _check_decode(gcodec, gdev, FIXED_FIELDS, data, off)
    e = datagen.make_element_batch(2000, (("uniform", 0, 20), ("uniform", 0, 30), ("uniform", 0, 300)), 9)
    fields = [(0, 4), (0, 0), (1, 0), (1, 0)]
    _check_encode(gcodec, gdev, fields, [e.score.view(np.uint8).reshape(-1, 4)] + e.strings, 2000)
    recs = corrupted_batch(2000, 4)
    _check_decode(gcodec, gdev, fields, *batch_of(recs))


@pytest.mark.gpu
@pytest.mark.parametrize("fields", [[(0, 0)] * 16, [(1, 8)] * 16, [(0, 0)] * 8 + [(1, 0)] * 8, [(0, 1)] * 16,
                                    [(1, 0), (0, 0)] * 8, [(0, 8), (0, 0)] * 4 + [(1, 4), (1, 0)] * 4,
                                    [(0, REP | 4), (1, REP | 8), (1, 0), (0, REP | 1)] * 4],
                         ids=["pub16str", "priv16u64", "pub8priv8", "pub16bool", "alt16str", "mixed16", "rep16"])
def test_flat_wide_schemas_gpu(gcodec, gdev, fields):
    """The widest generated images (up to 142 bytes per record; fewer waves per workgroup)."""
    rng = np.random.default_rng(len(fields) + sum(w for _, w in fields))
    cols = random_columns(rng, fields, 1500)
    data, off = _check_encode(gcodec, gdev, fields, cols, 1500, sid=3, mid=4)
    _check_decode(gcodec, gdev, fields, data, off)
    _check_decode(gcodec, gdev, fields, *corrupt(data, off, rng, frac=0.4))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 255, 256, 257])
def test_flat_edge_counts_gpu(gcodec, gdev, n):
    rng = np.random.default_rng(n + 50)
    fields = [(0, 8), (1, 0), (0, 0), (1, 1)]
    cols = random_columns(rng, fields, n)
    data, off = _check_encode(gcodec, gdev, fields, cols, n)
    _check_decode(gcodec, gdev, fields, data, off)


def batch_of(recs):
    off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off

"""Parity of the HIP codec (through the C ABI) with the CPU oracle and the golden fixtures.

Bar: bit-exact bytes, offsets, int32 fields and per-record status.  Every call goes
through libsymphony_hip.so; the oracle is only the checker.
"""
import hashlib

import numpy as np
import pytest

from arpc_amd import datagen, schemas
from oracle import oracle

pytestmark = pytest.mark.gpu

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


DECODE_IMPLS = {"pipe": 0, "three_kernel": 1, "lookback": 2}  # SYM_DECODE_* (include/symphony_hip.h)


@pytest.fixture(autouse=True, params=sorted(DECODE_IMPLS))
def decode_impl(request, codec):
    """Every test runs against each decode implementation behind the same C ABI, selected with
    sym_ctx_set_decode_impl: the default single-launch pipeline (decode_pipe.hip), its forced
    look-back mode (the progress fallback: parsers and scanner idle, every copier resolves its own
    prefix), and the three-kernel path (decode.hip)."""
    codec.set_decode_impl(DECODE_IMPLS[request.param])
    yield request.param
    codec.set_decode_impl(0)


def put(arr: np.ndarray, dev, misalign: int = 0, guard: int = 32, fill: int = 0xA5):
    """Copy arr to the GPU at byte offset `misalign` inside a guarded allocation."""
    raw = np.ascontiguousarray(arr).view(np.uint8)
    buf = torch.full((raw.size + misalign + guard,), fill, dtype=torch.uint8, device=dev)
    if raw.size:
        buf[misalign:misalign + raw.size].copy_(torch.from_numpy(raw.copy()))
    view = buf[misalign:misalign + raw.size]
    if arr.dtype == np.int32:
        view = view.view(torch.int32)
    elif arr.dtype in (np.uint64, np.int64):
        view = view.view(torch.int64)
    return buf, view


def columns_to_gpu(batch, dev, misalign=0, base_pad=0):
    """Device columns; string columns get `base_pad` junk bytes in front (offs[0] = base_pad)."""
    keep, fixed, var = [], [], []
    for c in batch.fixed:
        b, v = put(c, dev, 0)
        keep.append(b)
        fixed.append(v)
    for i, (by, of) in enumerate(batch.var):
        padded = np.concatenate([np.full(base_pad, 0x5A, np.uint8), by, np.zeros(1, np.uint8)])
        b, v = put(padded, dev, (misalign + 3 * i) % 16)
        o = (of - of[0] + base_pad).astype(np.uint64)
        ob, ov = put(o, dev, 0)
        keep += [b, ob]
        var.append((v, ov))
    return keep, fixed, var


def encode_gpu(codec, batch, dev, sid=0, mid=0, misalign=0, base_pad=0, out_misalign=0):
    keep, fixed, var = columns_to_gpu(batch, dev, misalign, base_pad)
    total = batch.encoded_size()
    obuf = torch.full((total + out_misalign + 48,), 0xC3, dtype=torch.uint8, device=dev)
    out = obuf[out_misalign:out_misalign + max(total, 1)]
    enc = codec.encode(batch.schema, fixed, var, sid, mid, out=out)
    torch.cuda.synchronize()
    g = obuf.cpu().numpy()
    assert (g[:out_misalign] == 0xC3).all(), "wrote before the output range"
    assert (g[out_misalign + total:] == 0xC3).all(), "wrote past the output range"
    return g[out_misalign:out_misalign + total], enc.offsets.cpu().numpy().view(np.uint64)


def decode_gpu(codec, schema, stream: np.ndarray, rec_off: np.ndarray, dev, misalign=0, pre=0):
    """Decode with the stream placed after `pre` junk bytes (rec_off shifted: rec_off[0] != 0)."""
    s = schemas.BY_NAME[schema] if isinstance(schema, str) else schema
    data = np.concatenate([np.full(pre, 0x77, np.uint8), stream.astype(np.uint8), np.zeros(1, np.uint8)])
    _, d = put(data, dev, misalign)
    _, ro = put((rec_off.astype(np.uint64) + np.uint64(pre)), dev, 0)
    out = codec.decode(s, d, ro)
    codec.check()
    n = len(rec_off) - 1
    fixed = [f.cpu().numpy()[:n] for f in out.fixed]
    var = []
    for b, o in out.var:
        o = o.cpu().numpy().view(np.uint64)
        var.append((b.cpu().numpy()[:int(o[-1])], o))
    return fixed, var, out.status.cpu().numpy()[:n]


def assert_decode_equal(got, want, ctx=""):
    gf, gv, gs = got
    wf, wv, ws = want
    np.testing.assert_array_equal(gs, ws, err_msg=f"status {ctx}")
    for a, b in zip(gf, wf):
        np.testing.assert_array_equal(a, b, err_msg=f"fixed {ctx}")
    for (ab, ao), (bb, bo) in zip(gv, wv):
        np.testing.assert_array_equal(ao, bo, err_msg=f"offsets {ctx}")
        np.testing.assert_array_equal(ab, bb, err_msg=f"bytes {ctx}")


# ---------------------------------------------------------------- known answers
def test_encode_kats(codec, dev, kats):
    for k in kats["encode"]:
        b = datagen.from_records(k["schema"], [(k["fixed"], [bytes.fromhex(f) for f in k["fields"]])])
        got, off = encode_gpu(codec, b, dev, k["service_id"], k["method_id"])
        assert got.tobytes().hex() == k["expected"], k["name"]
        assert off.tolist() == [0, len(k["expected"]) // 2]


def test_encode_kats_batched_per_schema(codec, dev, kats):
    by = {}
    for k in kats["encode"]:
        if k["service_id"] == 0:
            by.setdefault(k["schema"], []).append(k)
    for schema, ks in by.items():
        recs = [(k["fixed"], [bytes.fromhex(f) for f in k["fields"]]) for k in ks] * 300  # spans tiles
        got, off = encode_gpu(codec, datagen.from_records(schema, recs), dev, out_misalign=5)
        want = "".join(k["expected"] for k in ks) * 300
        assert got.tobytes().hex() == want, schema


def test_decode_kats(codec, dev, kats):
    by = {}
    for k in kats["decode"]:
        by.setdefault(k["schema"], []).append(k)
    for schema, ks in by.items():
        s = schemas.BY_NAME[schema]
        recs = [bytes.fromhex(k["input"]) for k in ks]
        rec_off = np.zeros(len(recs) + 1, np.uint64)
        np.cumsum([len(r) for r in recs], out=rec_off[1:])
        stream = np.frombuffer(b"".join(recs), np.uint8)
        fixed, var, status = decode_gpu(codec, s, stream, rec_off, dev, misalign=7, pre=3)
        for i, k in enumerate(ks):
            assert status[i] == k["status"], k["name"]
            assert [int(f[i]) for f in fixed] == k["fixed"], k["name"]
            got = [col[int(o[i]):int(o[i + 1])].tobytes() for col, o in var]
            assert got == [bytes.fromhex(f) for f in k["fields"]], k["name"]


# ---------------------------------------------------------------- pinned corpora
@pytest.mark.parametrize("name", sorted(datagen.CORPORA))
def test_encode_corpora_match_pins(codec, dev, corpora, name):
    kw = datagen.CORPORA[name]
    b = datagen.make_batch(**kw)
    got, off = encode_gpu(codec, b, dev, kw.get("service_id", 0), kw.get("method_id", 0), misalign=9,
                          base_pad=11, out_misalign=13)
    assert hashlib.sha256(got.tobytes()).hexdigest() == corpora[name]["sha256_stream"]
    assert hashlib.sha256(off.tobytes()).hexdigest() == corpora[name]["sha256_offsets"]


@pytest.mark.parametrize("name", sorted(datagen.CORPORA))
def test_decode_corpora_roundtrip(codec, dev, name):
    kw = datagen.CORPORA[name]
    b = datagen.make_batch(**kw)
    stream, off = oracle.encode_batch(b.fixed, b.var, kw.get("service_id", 0), kw.get("method_id", 0))
    got = decode_gpu(codec, b.schema, stream, off, dev, misalign=1, pre=17)
    want = oracle.decode_batch(b.schema.nfixed, b.schema.nvar, stream, off)
    assert_decode_equal(got, want, name)
    for f in range(b.schema.nvar):  # and equal to the original columns
        np.testing.assert_array_equal(got[1][f][0], b.var[f][0])


# ---------------------------------------------------------------- alignment / edges
@pytest.mark.parametrize("misalign", [0, 1, 2, 3, 5, 8, 15])
def test_encode_any_alignment(codec, dev, misalign):
    b = datagen.make_batch(schema="kv_set_request", n=777, lens=(("uniform", 0, 40), ("uniform", 0, 90)), seed=3)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got, off = encode_gpu(codec, b, dev, misalign=misalign, base_pad=misalign * 7, out_misalign=misalign)
    np.testing.assert_array_equal(off, woff)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("n", [0, 1, 2, 255, 256, 257, 513])
@pytest.mark.parametrize("schema", ["kv_get_request", "kv_set_request", "echo_request"])
def test_edge_counts(codec, dev, n, schema):
    s = schemas.BY_NAME[schema]
    lens = tuple(("uniform", 0, 5) for _ in range(s.nvar))
    b = datagen.make_batch(schema=schema, n=n, lens=lens, seed=n + 1)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got, off = encode_gpu(codec, b, dev, out_misalign=n % 16)
    np.testing.assert_array_equal(off, woff)
    np.testing.assert_array_equal(got, want)
    dec = decode_gpu(codec, s, want, woff, dev, misalign=n % 5)
    assert_decode_equal(dec, oracle.decode_batch(s.nfixed, s.nvar, want, woff), f"{schema} n={n}")


def test_all_empty_fields(codec, dev):
    b = datagen.make_batch(schema="kv_set_request", n=1000, lens=(0, 0), seed=1)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got, off = encode_gpu(codec, b, dev)
    np.testing.assert_array_equal(got, want)
    dec = decode_gpu(codec, b.schema, want, woff, dev)
    assert_decode_equal(dec, oracle.decode_batch(0, 2, want, woff))


def test_large_values_span_tiles(codec, dev):
    b = datagen.make_batch(schema="kv_set_request", n=600, lens=(("uniform", 0, 300), ("uniform", 0, 70000)),
                           seed=99)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got, off = encode_gpu(codec, b, dev, misalign=3, out_misalign=6)
    np.testing.assert_array_equal(off, woff)
    np.testing.assert_array_equal(got, want)
    dec = decode_gpu(codec, b.schema, want, woff, dev, misalign=2)
    assert_decode_equal(dec, oracle.decode_batch(0, 2, want, woff))


def test_echo_int32_extremes(codec, dev):
    recs = [([-2147483648, 2147483647], [b"", b"x"]), ([0, -1], [b"u" * 33, b""]), ([42, 300], [b"alice", b"hi"])]
    b = datagen.from_records("echo_request", recs * 200)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got, _ = encode_gpu(codec, b, dev)
    np.testing.assert_array_equal(got, want)
    dec = decode_gpu(codec, b.schema, want, woff, dev)
    np.testing.assert_array_equal(dec[0][0], b.fixed[0])
    np.testing.assert_array_equal(dec[0][1], b.fixed[1])


# ---------------------------------------------------------------- adversarial decode
def _mutated_stream(seed: int, schema: str, n: int):
    """A valid encoded batch, then byte mutations concentrated in headers/tables/length prefixes,
    truncations and re-framing (random record boundaries), plus pure-garbage records."""
    rng = np.random.default_rng(seed)
    s = schemas.BY_NAME[schema]
    lens = tuple(("uniform", 0, 24) for _ in range(s.nvar))
    b = datagen.make_batch(schema=schema, n=n, lens=lens, seed=seed)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    recs = [bytearray(stream[off[i]:off[i + 1]].tobytes()) for i in range(n)]
    out = []
    for r in recs:
        kind = rng.integers(0, 10)
        if kind <= 3:  # flip bytes in the first 40 (header, table, first length prefix)
            for _ in range(rng.integers(1, 4)):
                p = int(rng.integers(0, min(len(r), 40)))
                r[p] = int(rng.integers(0, 256))
        elif kind == 4:  # write a random u32 at a random position
            p = int(rng.integers(0, max(1, len(r) - 3)))
            r[p:p + 4] = int(rng.integers(0, 1 << 32)).to_bytes(4, "little")
        elif kind == 5:  # truncate
            r = r[:int(rng.integers(0, len(r) + 1))]
        elif kind == 6:  # small table offsets pointing into the header
            p = 14 + 4 * int(rng.integers(0, s.nfixed + s.nvar))
            if p + 4 <= len(r):
                r[p:p + 4] = int(rng.integers(0, 40)).to_bytes(4, "little")
        elif kind == 7:  # garbage
            r = bytearray(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8).tobytes())
            if len(r) > 0 and rng.integers(0, 2):
                r[0] = 1
        out.append(bytes(r))
    rec_off = np.zeros(n + 1, np.uint64)
    np.cumsum([len(r) for r in out], out=rec_off[1:])
    return np.frombuffer(b"".join(out), np.uint8).copy(), rec_off


@pytest.mark.parametrize("schema", [s.name for s in schemas.ALL])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_decode_matches_oracle(codec, dev, schema, seed):
    s = schemas.BY_NAME[schema]
    stream, rec_off = _mutated_stream(seed, schema, 3000)
    got = decode_gpu(codec, s, stream, rec_off, dev, misalign=seed)
    want = oracle.decode_batch(s.nfixed, s.nvar, stream, rec_off)
    assert_decode_equal(got, want, f"{schema}/{seed}")
    assert (want[2] != 0).any() and (want[2] == 0).any()


def test_fuzz_reframed_stream(codec, dev):
    """Random record boundaries over a valid stream: most records misframed."""
    b = datagen.make_batch(**datagen.CORPORA["set_tiny"])
    stream, _ = oracle.encode_batch(b.fixed, b.var)
    rng = np.random.default_rng(5)
    cuts = np.sort(rng.choice(np.arange(1, len(stream)), size=4000, replace=False)).astype(np.uint64)
    rec_off = np.concatenate([[0], cuts, [len(stream)]]).astype(np.uint64)
    got = decode_gpu(codec, b.schema, stream, rec_off, dev)
    assert_decode_equal(got, oracle.decode_batch(0, 2, stream, rec_off))


def test_decode_capacity_overflow_reported(codec, dev):
    from arpc_amd._native import SYM_ERR_CAPACITY, SymphonyHipError
    b = datagen.make_batch(schema="kv_set_request", n=500, lens=(8, 32), seed=4)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    _, d = put(stream, dev)
    _, ro = put(off, dev)
    out = codec.decode("kv_set_request", d, ro, caps=[8 * 500, 1000])
    with pytest.raises(SymphonyHipError) as ei:
        codec.check()
    assert ei.value.code == SYM_ERR_CAPACITY
    torch.cuda.synchronize()
    assert out.var[0][0].cpu().numpy().tobytes() == b.var[0][0].tobytes()  # the column that fit is intact
    codec.check()  # the error word was cleared


# ---------------------------------------------------------------- full-size properties
def _roundtrip_full(codec, dev, kw):
    from arpc_amd.codec import to_device
    b = datagen.make_batch(**kw)
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    dec = codec.decode(b.schema, enc.data, enc.offsets, caps=[int(o[-1]) for _, o in b.var])
    codec.check()
    n = b.n
    # record offsets are affine in the input offsets
    expect = torch.arange(n + 1, device=dev, dtype=torch.int64) * b.schema.overhead
    for _, o in var:
        expect += o - o[0]
    assert torch.equal(enc.offsets, expect)
    assert int(dec.status.sum().item()) == 0
    for f, (bcol, ocol) in enumerate(var):
        assert torch.equal(dec.var[f][1], ocol - ocol[0])
        assert torch.equal(dec.var[f][0][:bcol.numel()], bcol)
    # the WHOLE stream equals the oracle's encoding of the same records (digest, then offsets)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got = enc.data[:len(want)].cpu().numpy()
    assert hashlib.sha256(got.tobytes()).hexdigest() == hashlib.sha256(want.tobytes()).hexdigest()
    np.testing.assert_array_equal(enc.offsets.cpu().numpy().view(np.uint64), woff)
    return b, enc


def test_config2_full_roundtrip(codec, dev):
    b, enc = _roundtrip_full(codec, dev, datagen.CONFIG2)
    assert enc.data.numel() == 350 * (1 << 20)


def test_config3_full_roundtrip(codec, dev):
    _roundtrip_full(codec, dev, datagen.CONFIG3)


def test_nondefault_stream(codec, dev):
    from arpc_amd.codec import to_device
    b = datagen.make_batch(**datagen.CORPORA["set_mixed"])
    want, woff = oracle.encode_batch(b.fixed, b.var)
    s = torch.cuda.Stream(dev)
    fixed, var = to_device(b, dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        enc = codec.encode(b.schema, fixed, var, var_total=int(sum(o[-1] for _, o in b.var)))
    s.synchronize()
    np.testing.assert_array_equal(enc.data.cpu().numpy()[:len(want)], want)


# ---------------------------------------------------------------- the Serializer mirror
def test_serializer_roundtrip_like_reference_tests(dev):
    """TestVar / TestFixed-style cases (cmd/symphony-gen-arpc/test/serialization_test.go:42-175)."""
    from arpc_amd.serializer import EchoRequest, GetRequest, SetRequest, SetResponse, SymphonySerializer
    ser = SymphonySerializer(0)
    cases = [SetRequest(b"", b""), SetRequest(b"k", b"v" * 1000), SetRequest("héllo".encode(), b"\x00\xff" * 7),
             GetRequest(b"key-1"), SetResponse(b"ok"),
             EchoRequest(-2147483648, 2147483647, b"alice", b"hello world"), EchoRequest(42, 300, b"", b"")]
    for m in cases:
        data = ser.marshal(m)
        assert data == oracle.marshal([getattr(m, f) for f in m.SCHEMA.fixed_fields],
                                      [getattr(m, f) for f in m.SCHEMA.var_fields])
        out = type(m)()
        ser.unmarshal(data, out)
        assert out == m
    batch = ser.marshal_batch(cases)
    outs = [type(m)() for m in cases]
    assert ser.unmarshal_batch(batch, outs) == [None] * len(cases)
    assert outs == cases


def test_serializer_errors_carry_go_text(dev):
    from arpc_amd.serializer import EchoRequest, SetRequest, SymphonyError, SymphonySerializer
    ser = SymphonySerializer(0)
    for data, text in [(b"", "invalid data: too short"), (b"\x02" * 13, "invalid data: wrong public version"),
                       (bytes.fromhex("010d00000000000000000000000000"), "missing private segment")]:
        with pytest.raises(SymphonyError, match=text):
            ser.unmarshal(data, SetRequest())
    out = EchoRequest()
    with pytest.raises(SymphonyError, match="too short for field"):
        ser.unmarshal(bytes.fromhex("010d0000000000000000000000012a000000"), out)
    assert out.Id == 42 and out.Score == 0
    with pytest.raises(TypeError):
        ser.marshal(object())

"""Mixed GetRequest / SetRequest batches (BASELINE config 2 as written: "Get/Set records").

The kv-store's request stream interleaves GetRequest{Key} (kv.syn.go:74-185) and SetRequest{Key,Value}
(:611-745) records; the client patches the method of each call into [9:13] (client.go:267-271,
KVService Get = 1, Set = 2, kv_arpc.syn.go:25-28).  sym_encode_kv_mixed / sym_decode_kv_mixed take a
per-record type column.  Bar: bit-exact against the oracle (oracle/symphony_oracle.c
sym_oracle_*_kv_mixed), whose mixed form is pinned here to the per-type hand-derived KATs.
"""
import hashlib

import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle


def _kat(kats, name):
    return next(k for k in kats["encode"] if k["name"] == name)


def _cols(values):
    offs = np.zeros(len(values) + 1, np.uint64)
    np.cumsum([len(v) for v in values], out=offs[1:])
    return np.frombuffer(b"".join(values), np.uint8).copy(), offs


# A hand-written request stream: Get "ab", Set "ab"/"xyz", Set ""/"", Get "ab" (the per-type KATs of
# tests/golden/kats.json, which are hand-derived from kv.syn.go).
KAT_TYPES = np.array([0, 1, 1, 0], np.uint8)
KAT_KEYS = [b"ab", b"ab", b"", b"ab"]
KAT_VALS = [b"", b"xyz", b"", b""]


def kat_stream(kats, ids: bool) -> str:
    if ids:
        return _kat(kats, "get_ab_ids")["expected"] + _kat(kats, "set_ab_xyz_ids")["expected"] + \
            "010d000000" + "01000000" + "02000000" + "01" + "090000000d0000000000000000000000" + \
            _kat(kats, "get_ab_ids")["expected"]
    return _kat(kats, "get_ab")["expected"] + _kat(kats, "set_ab_xyz")["expected"] + \
        _kat(kats, "set_empty")["expected"] + _kat(kats, "get_ab")["expected"]


# ---------------------------------------------------------------- CPU: the oracle's mixed form
@pytest.mark.parametrize("ids", [False, True])
def test_oracle_mixed_matches_per_type_kats(kats, ids):
    sid, gm, sm = (1, 1, 2) if ids else (0, 0, 0)
    stream, off = oracle.encode_kv_mixed(KAT_TYPES, _cols(KAT_KEYS), _cols(KAT_VALS), sid, gm, sm)
    assert stream.tobytes().hex() == kat_stream(kats, ids)
    assert off.tolist() == [0, 24, 59, 89, 113]


def test_oracle_mixed_equals_per_record_marshal():
    b = datagen.make_mixed_batch(n=500, key=("uniform", 0, 30), value=("uniform", 0, 90), set_fraction=0.5, seed=4)
    stream, off = oracle.encode_kv_mixed(b.type, b.key, b.val, 1, 1, 2)
    (kb, ko), (vb, vo) = b.key, b.val
    for i in range(b.n):
        fields = [kb[ko[i]:ko[i + 1]].tobytes()] + ([vb[vo[i]:vo[i + 1]].tobytes()] if b.type[i] else [])
        assert stream[off[i]:off[i + 1]].tobytes() == oracle.marshal([], fields, 1, 2 if b.type[i] else 1)
    assert len(stream) == b.encoded_size()


def test_oracle_mixed_decode_is_per_type_unmarshal():
    rng = np.random.default_rng(3)
    b = datagen.make_mixed_batch(n=400, key=("uniform", 0, 12), value=("uniform", 0, 20), set_fraction=0.4, seed=8)
    stream, off = oracle.encode_kv_mixed(b.type, b.key, b.val)
    recs = [bytearray(stream[off[i]:off[i + 1]].tobytes()) for i in range(b.n)]
    for r in recs:  # corrupt headers / tables: every skip branch of kv.syn.go:134-185 / :680-745
        if rng.integers(0, 3) == 0 and len(r):
            r[int(rng.integers(0, min(len(r), 30)))] = int(rng.integers(0, 256))
    rtype = b.type.copy()
    rtype[rng.integers(0, b.n, 40)] ^= 1  # some records decoded as the other type
    data, ro = _cols([bytes(r) for r in recs])
    cols, st = oracle.decode_kv_mixed(data, ro, rtype)
    for i in range(b.n):
        nv = 2 if rtype[i] else 1
        s, _, fields = oracle.unmarshal(0, nv, bytes(recs[i]))
        assert st[i] == s
        assert cols[0][0][cols[0][1][i]:cols[0][1][i + 1]].tobytes() == fields[0]
        assert cols[1][0][cols[1][1][i]:cols[1][1][i + 1]].tobytes() == (fields[1] if nv == 2 else b"")


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


def _put(arr, dev, misalign=0):
    raw = np.ascontiguousarray(arr).view(np.uint8)
    buf = torch.full((raw.size + misalign + 32,), 0xA5, dtype=torch.uint8, device=dev)
    if raw.size:
        buf[misalign:misalign + raw.size].copy_(torch.from_numpy(raw.copy()))
    v = buf[misalign:misalign + raw.size]
    return v.view(torch.int64) if arr.dtype in (np.uint64, np.int64) else v


def _gpu_encode(codec, dev, rtype, key, val, ids=(0, 0, 0), misalign=0, out_misalign=0):
    total = 22 * len(rtype) + int(key[1][-1] - key[1][0]) + int((8 + np.diff(val[1]).astype(np.int64))[rtype != 0].sum())
    obuf = torch.full((total + out_misalign + 48,), 0xC3, dtype=torch.uint8, device=dev)
    out = obuf[out_misalign:out_misalign + max(total, 1)]
    enc = codec.encode_kv_mixed(_put(rtype, dev), (_put(np.concatenate([key[0], [0]]).astype(np.uint8), dev, misalign), _put(key[1], dev)),
                                (_put(np.concatenate([val[0], [0]]).astype(np.uint8), dev, (misalign + 5) % 16), _put(val[1], dev)),
                                *ids, out=out)
    codec.check()
    g = obuf.cpu().numpy()
    assert (g[:out_misalign] == 0xC3).all() and (g[out_misalign + total:] == 0xC3).all(), "wrote outside the output"
    return g[out_misalign:out_misalign + total], enc.offsets.cpu().numpy().view(np.uint64)


def _gpu_decode(codec, dev, stream, rec_off, rtype, misalign=0):
    d = _put(np.concatenate([stream, np.zeros(1, np.uint8)]).astype(np.uint8), dev, misalign)
    out = codec.decode_kv_mixed(d, _put(rec_off.astype(np.uint64), dev), _put(rtype, dev))
    codec.check()
    n = len(rec_off) - 1
    cols = []
    for b, o in out.var:
        o = o.cpu().numpy().view(np.uint64)
        cols.append((b.cpu().numpy()[:int(o[-1])], o))
    return cols, out.status.cpu().numpy()[:n]


# SYM_DECODE_* and SYM_ENCODE_* (include/symphony_hip.h): the same three shapes for the decode's and
# the mixed encode's scans -- one pipelined launch, three launches, the launch's look-back fallback
IMPLS = {"pipe": 0, "three_kernel": 1, "lookback": 2}


@pytest.fixture(params=sorted(IMPLS))
def impl(request, codec):
    codec.set_decode_impl(IMPLS[request.param])
    codec.set_encode_impl(IMPLS[request.param])
    yield request.param
    codec.set_decode_impl(0)
    codec.set_encode_impl(0)


@pytest.mark.gpu
@pytest.mark.parametrize("ids", [False, True])
def test_gpu_mixed_kat(codec, dev, impl, kats, ids):
    idt = (1, 1, 2) if ids else (0, 0, 0)
    got, off = _gpu_encode(codec, dev, KAT_TYPES, _cols(KAT_KEYS), _cols(KAT_VALS), idt, misalign=3, out_misalign=7)
    assert got.tobytes().hex() == kat_stream(kats, ids)
    assert off.tolist() == [0, 24, 59, 89, 113]
    # repeated across tiles and size-pass groups
    reps = 1500
    t = np.tile(KAT_TYPES, reps)
    got, off = _gpu_encode(codec, dev, t, _cols(KAT_KEYS * reps), _cols(KAT_VALS * reps), idt)
    assert got.tobytes().hex() == kat_stream(kats, ids) * reps


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 255, 257, 4095, 4096, 4097, 9000])
@pytest.mark.parametrize("frac", [0.0, datagen.TRACE_SET_FRACTION, 1.0])
def test_gpu_mixed_random(codec, dev, impl, n, frac):
    b = datagen.make_mixed_batch(n=n, key=("uniform", 0, 40), value=("uniform", 0, 120), set_fraction=frac, seed=n + 7)
    want, woff = oracle.encode_kv_mixed(b.type, b.key, b.val, 1, 1, 2)
    got, off = _gpu_encode(codec, dev, b.type, b.key, b.val, (1, 1, 2), misalign=n % 16, out_misalign=(n * 7) % 16)
    np.testing.assert_array_equal(off, woff)
    np.testing.assert_array_equal(got, want)
    cols, st = _gpu_decode(codec, dev, want, woff, b.type, misalign=n % 11)
    wcols, wst = oracle.decode_kv_mixed(want, woff, b.type)
    np.testing.assert_array_equal(st, wst)
    for (gb, go), (wb, wo) in zip(cols, wcols):
        np.testing.assert_array_equal(go, wo)
        np.testing.assert_array_equal(gb, wb)
    np.testing.assert_array_equal(cols[0][0], b.key[0])
    np.testing.assert_array_equal(cols[1][0], b.val[0])


@pytest.mark.gpu
def test_gpu_mixed_get_values_are_not_encoded(codec, dev):
    """A GetRequest's value slice is not part of its record (GetRequest has no Value field)."""
    rng = np.random.default_rng(1)
    n = 3000
    rtype = (rng.random(n) < 0.5).astype(np.uint8)
    keys = [rng.bytes(int(rng.integers(0, 20))) for _ in range(n)]
    vals = [rng.bytes(int(rng.integers(0, 50))) for _ in range(n)]  # Gets carry junk values too
    want, woff = oracle.encode_kv_mixed(rtype, _cols(keys), _cols(vals))
    got, off = _gpu_encode(codec, dev, rtype, _cols(keys), _cols(vals))
    np.testing.assert_array_equal(off, woff)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
def test_gpu_mixed_large_and_empty_values(codec, dev, impl):
    b = datagen.make_mixed_batch(n=700, key=("uniform", 0, 300), value=("loguniform", 1, 70000), set_fraction=0.5,
                                 seed=77)
    want, woff = oracle.encode_kv_mixed(b.type, b.key, b.val)
    got, off = _gpu_encode(codec, dev, b.type, b.key, b.val, misalign=9, out_misalign=2)
    np.testing.assert_array_equal(got, want)
    cols, st = _gpu_decode(codec, dev, want, woff, b.type, misalign=4)
    assert (st == 0).all()
    np.testing.assert_array_equal(cols[1][0], b.val[0])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_mixed_fuzz_decode(codec, dev, impl, seed):
    rng = np.random.default_rng(seed)
    b = datagen.make_mixed_batch(n=3000, key=("uniform", 0, 24), value=("uniform", 0, 24), set_fraction=0.4, seed=seed)
    stream, off = oracle.encode_kv_mixed(b.type, b.key, b.val)
    recs = [bytearray(stream[off[i]:off[i + 1]].tobytes()) for i in range(b.n)]
    for i, r in enumerate(recs):
        k = rng.integers(0, 8)
        if k <= 2 and len(r):
            for _ in range(int(rng.integers(1, 4))):
                r[int(rng.integers(0, min(len(r), 40)))] = int(rng.integers(0, 256))
        elif k == 3:
            recs[i] = r[:int(rng.integers(0, len(r) + 1))]
    rtype = b.type.copy()
    rtype[rng.integers(0, b.n, 200)] ^= 1
    data, ro = _cols([bytes(r) for r in recs])
    cols, st = _gpu_decode(codec, dev, data, ro, rtype, misalign=seed)
    wcols, wst = oracle.decode_kv_mixed(data, ro, rtype)
    np.testing.assert_array_equal(st, wst)
    for (gb, go), (wb, wo) in zip(cols, wcols):
        np.testing.assert_array_equal(go, wo)
        np.testing.assert_array_equal(gb, wb)
    assert (wst != 0).any() and (wst == 0).any()


@pytest.mark.gpu
def test_gpu_mixed_full_size_trace_ratio(codec, dev):
    """BASELINE config 2 as written: 2^20 Get/Set records at the trace's 36.9 % Set, K=64, V=256."""
    b = datagen.make_mixed_batch(**datagen.CONFIG2_MIXED)
    t = torch.from_numpy(b.type).to(dev)
    key = (torch.from_numpy(b.key[0]).to(dev), torch.from_numpy(b.key[1].view(np.int64)).to(dev))
    val = (torch.from_numpy(b.val[0]).to(dev), torch.from_numpy(b.val[1].view(np.int64)).to(dev))
    enc = codec.encode_kv_mixed(t, key, val, 1, 1, 2, out_bytes=b.encoded_size())
    dec = codec.decode_kv_mixed(enc.data, enc.offsets, t, caps=[b.key[0].size, max(1, b.val[0].size)])
    codec.check()
    n = b.n
    size = 22 + 64 + (8 + 256) * t.to(torch.int64)  # record sizes by type
    expect = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    expect[1:] = torch.cumsum(size, 0)
    assert torch.equal(enc.offsets, expect)
    assert int(dec.status.sum().item()) == 0
    assert torch.equal(dec.var[0][1], key[1]) and torch.equal(dec.var[0][0][:key[0].numel()], key[0])
    assert torch.equal(dec.var[1][1], val[1]) and torch.equal(dec.var[1][0][:val[0].numel()], val[0])
    # the WHOLE stream equals the oracle's encoding of the same records (kv.syn.go:74-132, :611-678)
    want, woff = oracle.encode_kv_mixed(b.type, b.key, b.val, 1, 1, 2)
    got = enc.data[:b.encoded_size()].cpu().numpy()
    assert hashlib.sha256(got.tobytes()).hexdigest() == hashlib.sha256(want.tobytes()).hexdigest()
    np.testing.assert_array_equal(enc.offsets.cpu().numpy().view(np.uint64), woff)
    # and the decode of the oracle's stream equals the oracle's decode, column by column
    wcols, wst = oracle.decode_kv_mixed(want, woff, b.type)
    np.testing.assert_array_equal(dec.status.cpu().numpy()[:n], wst)
    for (gb, go), (wb, wo) in zip(dec.var, wcols):
        np.testing.assert_array_equal(go.cpu().numpy().view(np.uint64), wo)
        np.testing.assert_array_equal(gb[:len(wb)].cpu().numpy(), wb)


@pytest.mark.gpu
def test_gpu_mixed_short_type_column_rejected(codec, dev):
    """The decode reads type[r] for every record: a type column shorter than the batch is refused on
    the host (as the encode does) instead of being read past its end on the device."""
    b = datagen.make_mixed_batch(n=100, key=8, value=16, set_fraction=0.5, seed=3)
    stream, off = oracle.encode_kv_mixed(b.type, b.key, b.val)
    d = _put(np.concatenate([stream, np.zeros(1, np.uint8)]).astype(np.uint8), dev)
    with pytest.raises(ValueError, match="type column"):
        codec.decode_kv_mixed(d, _put(off, dev), _put(b.type[:99], dev))


@pytest.mark.gpu
def test_gpu_mixed_many_groups_offsets(codec, dev, impl):
    """More than 4096 size-pass groups (1024 records each), so the one-workgroup group scan takes a
    second round: 4.3M small Get/Set records; offsets equal the cumulative record sizes, and the
    decode returns every column."""
    n = 4200 * 1024 + 77
    g = torch.Generator(device="cpu").manual_seed(11)
    rtype = (torch.rand(n, generator=g) < datagen.TRACE_SET_FRACTION).to(torch.uint8)
    klen = torch.randint(0, 9, (n,), generator=g, dtype=torch.int64)
    vlen = torch.randint(0, 17, (n,), generator=g, dtype=torch.int64) * rtype.to(torch.int64)
    koff = torch.zeros(n + 1, dtype=torch.int64)
    koff[1:] = torch.cumsum(klen, 0)
    voff = torch.zeros(n + 1, dtype=torch.int64)
    voff[1:] = torch.cumsum(vlen, 0)
    kb = torch.randint(0, 256, (int(koff[-1]) + 1,), generator=g, dtype=torch.int64).to(torch.uint8)
    vb = torch.randint(0, 256, (int(voff[-1]) + 1,), generator=g, dtype=torch.int64).to(torch.uint8)
    t = rtype.to(dev)
    key = (kb.to(dev), koff.to(dev))
    val = (vb.to(dev), voff.to(dev))
    size = 22 + klen + (8 + vlen) * rtype.to(torch.int64)
    expect = torch.zeros(n + 1, dtype=torch.int64)
    expect[1:] = torch.cumsum(size, 0)
    enc = codec.encode_kv_mixed(t, key, val, 1, 1, 2, out_bytes=int(expect[-1]))
    dec = codec.decode_kv_mixed(enc.data, enc.offsets, t, caps=[kb.numel(), vb.numel()])
    codec.check()
    assert torch.equal(enc.offsets.cpu(), expect)
    assert int(dec.status.sum().item()) == 0
    assert torch.equal(dec.var[0][1].cpu(), koff) and torch.equal(dec.var[0][0][:int(koff[-1])].cpu(), kb[:int(koff[-1])])
    assert torch.equal(dec.var[1][1].cpu(), voff) and torch.equal(dec.var[1][0][:int(voff[-1])].cpu(), vb[:int(voff[-1])])

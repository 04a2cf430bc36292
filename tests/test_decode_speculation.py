"""The default decode's speculative parsers and its gate (decode_pipe.hip).

For kv layouts the parsers take each record's field lengths from the generator's layout (the last
string field runs to the record's end) instead of reading every length prefix; every copier checks
them against Go's exact parse, and the gate decodes the batch again exactly when any was wrong.
These tests build batches in which the speculation fails for a few records only -- a record with
bytes after its last field, which Go accepts (kv.syn.go:717-742 checks only that the field fits) --
so the first launch writes most of the output correctly and the re-decode must rewrite all of it,
and check the result bit for bit against the oracle under every decode implementation.
"""
import numpy as np
import pytest

from arpc_amd import datagen, schemas
from oracle import oracle

from test_gpu_parity import assert_decode_equal, decode_gpu, put  # noqa: F401  (fixtures below)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

DECODE_IMPLS = {"pipe": 0, "three_kernel": 1, "lookback": 2}


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


@pytest.fixture(autouse=True, params=sorted(DECODE_IMPLS))
def decode_impl(request, codec):
    """Setting the impl also clears the ctx's speculation hold, so every test starts speculating."""
    codec.set_decode_impl(DECODE_IMPLS[request.param])
    yield request.param
    codec.set_decode_impl(0)


def _with_trailers(stream, off, which, extra=7, seed=0):
    """The records `which` get `extra` junk bytes after their last field."""
    rng = np.random.default_rng(seed)
    recs = [stream[off[i]:off[i + 1]].tobytes() for i in range(len(off) - 1)]
    for i in which:
        recs[i] = recs[i] + rng.integers(0, 256, extra, dtype=np.uint8).tobytes()
    rec_off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=rec_off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), rec_off


@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_one_misfit_record_is_redecoded(codec, dev, where):
    n = 50000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(("uniform", 0, 80), ("uniform", 0, 300)), seed=11)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    i = {"first": 0, "middle": n // 2 + 3, "last": n - 1}[where]
    data, rec_off = _with_trailers(stream, off, [i])
    got = decode_gpu(codec, "kv_set_request", data, rec_off, dev)
    want = oracle.decode_batch(0, 2, data, rec_off)
    assert_decode_equal(got, want, where)
    assert (want[2] == 0).all()  # Go accepts the trailing bytes: every record decodes


@pytest.mark.parametrize("schema", ["kv_get_request", "kv_set_request", "kv_get_response"])
def test_sparse_misfits_every_kv_schema(codec, dev, schema):
    s = schemas.BY_NAME[schema]
    n = 20000
    b = datagen.make_batch(schema=schema, n=n, lens=tuple(("uniform", 0, 64) for _ in range(s.nvar)), seed=12)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    data, rec_off = _with_trailers(stream, off, range(17, n, 4099), extra=1, seed=1)
    got = decode_gpu(codec, s, data, rec_off, dev, misalign=5)
    assert_decode_equal(got, oracle.decode_batch(s.nfixed, s.nvar, data, rec_off), schema)


def test_misfit_first_field_prefix_overstates(codec, dev):
    """A SetRequest whose first length prefix says more than the key it holds: the speculative
    second field comes out short, Go's exact parse gives different lengths (or none)."""
    n = 9000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(16, 40), seed=13)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    data = stream.copy()
    for i in (5, 4000, 8999):
        data[int(off[i]) + 22:int(off[i]) + 26] = np.frombuffer((20).to_bytes(4, "little"), np.uint8)
    got = decode_gpu(codec, "kv_set_request", data, off, dev)
    assert_decode_equal(got, oracle.decode_batch(0, 2, data, off))


def test_mixed_batch_with_misfits(codec, dev):
    m = datagen.make_mixed_batch(n=40000, key=("uniform", 0, 64), value=("uniform", 0, 256),
                                 set_fraction=datagen.TRACE_SET_FRACTION, seed=14)
    stream, off = oracle.encode_kv_mixed(m.type, m.key, m.val)
    gets = np.flatnonzero(m.type == 0)[[3, 700]]
    sets = np.flatnonzero(m.type != 0)[[9, 900]]
    data, rec_off = _with_trailers(stream, off, sorted(list(gets) + list(sets)), extra=3, seed=2)
    _, d = put(data, dev, 3)
    _, ro = put(rec_off, dev)
    t = torch.from_numpy(m.type).to(dev)
    out = codec.decode_kv_mixed(d, ro, t)
    codec.check()
    wcols, wst = oracle.decode_kv_mixed(data, rec_off, m.type)
    np.testing.assert_array_equal(out.status.cpu().numpy()[:m.n], wst)
    for (gb, go), (wb, wo) in zip(out.var, wcols):
        go = go.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(go, wo)
        np.testing.assert_array_equal(gb.cpu().numpy()[:int(wo[-1])], wb)


def test_capacity_error_only_from_the_speculation_is_dropped(codec, dev):
    """Capacities exactly the true column sizes; the speculative lengths of the misfit records are
    larger, so the first launch sees its prefixes run past the capacity.  The exact re-decode fits:
    no error may be reported."""
    n = 3000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(8, 24), seed=15)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    data, rec_off = _with_trailers(stream, off, [n - 3, n - 2, n - 1], extra=40)
    want = oracle.decode_batch(0, 2, data, rec_off)
    _, d = put(data, dev)
    _, ro = put(rec_off, dev)
    caps = [int(want[1][0][1][-1]), int(want[1][1][1][-1])]
    out = codec.decode("kv_set_request", d, ro, caps=caps)
    codec.check()  # raises on any error bit
    o1 = out.var[1][1].cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(o1, want[1][1][1])
    np.testing.assert_array_equal(out.var[1][0].cpu().numpy()[:caps[1]], want[1][1][0])


def test_capacity_error_with_speculation_holding_is_reported(codec, dev):
    from arpc_amd._native import SYM_ERR_CAPACITY, SymphonyHipError
    b = datagen.make_batch(schema="kv_set_request", n=4000, lens=(8, 32), seed=16)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    _, d = put(stream, dev)
    _, ro = put(off, dev)
    codec.decode("kv_set_request", d, ro, caps=[8 * 4000, 32 * 4000 - 1])
    with pytest.raises(SymphonyHipError) as ei:
        codec.check()
    assert ei.value.code == SYM_ERR_CAPACITY


def test_small_decode_after_large_mixed_encode(codec, dev):
    """The gate's control words sit after this call's words, where a larger earlier call (here a
    mixed encode's words) left other values: they carry other tags and must not read as errors."""
    m = datagen.make_mixed_batch(n=300000, key=("uniform", 0, 64), value=("uniform", 0, 256),
                                 set_fraction=datagen.TRACE_SET_FRACTION, seed=17)
    t = torch.from_numpy(m.type).to(dev)
    key = (torch.from_numpy(m.key[0]).to(dev), torch.from_numpy(m.key[1].view(np.int64)).to(dev))
    val = (torch.from_numpy(m.val[0]).to(dev), torch.from_numpy(m.val[1].view(np.int64)).to(dev))
    codec.encode_kv_mixed(t, key, val, 1, 1, 2, out_bytes=m.encoded_size())
    codec.check()
    for n in (1, 63, 64, 65, 1000):
        b = datagen.make_batch(schema="kv_set_request", n=n, lens=(("uniform", 0, 40), ("uniform", 0, 90)), seed=n)
        stream, off = oracle.encode_batch(b.fixed, b.var)
        got = decode_gpu(codec, "kv_set_request", stream, off, dev)  # checks the error word
        assert_decode_equal(got, oracle.decode_batch(0, 2, stream, off), f"n={n}")


def test_hold_after_a_miss_then_speculation_again(codec, dev):
    """After a batch the speculation missed, the ctx parses exactly for a while (the gate's hold);
    batches decoded in that time -- clean ones and ones with misfits -- and after it are all exact."""
    n = 6000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(("uniform", 0, 40), ("uniform", 0, 200)), seed=21)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    bad, bad_off = _with_trailers(stream, off, [7, 4000], extra=2, seed=3)
    want_bad = oracle.decode_batch(0, 2, bad, bad_off)
    want_ok = oracle.decode_batch(0, 2, stream, off)
    seq = [True, False, True] + [False] * 70 + [True, False]  # past the hold (64 calls) and a miss again
    for i, misfit in enumerate(seq):
        got = decode_gpu(codec, "kv_set_request", bad if misfit else stream, bad_off if misfit else off, dev)
        assert_decode_equal(got, want_bad if misfit else want_ok, f"call {i}")


@pytest.mark.parametrize("seed", [31, 32, 33, 34])
def test_random_batches_with_random_misfits(codec, dev, seed):
    """Random kv schema, record count (ragged: not a multiple of 64), value sizes and misfit density
    (none, one, a few, every record), each checked bit for bit against the oracle."""
    rng = np.random.default_rng(seed)
    schema = ["kv_get_request", "kv_set_request", "kv_get_response"][seed % 3]
    s = schemas.BY_NAME[schema]
    n = int(rng.integers(1000, 120000))
    lens = tuple(("uniform", 0, int(rng.choice([16, 64, 300, 2000]))) for _ in range(s.nvar))
    b = datagen.make_batch(schema=schema, n=n, lens=lens, seed=seed)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    density = [0, 1, 7, n][seed % 4]
    which = sorted(set(int(x) for x in rng.integers(0, n, density))) if density < n else range(n)
    data, rec_off = _with_trailers(stream, off, which, extra=int(rng.integers(1, 9)), seed=seed)
    got = decode_gpu(codec, s, data, rec_off, dev, misalign=int(rng.integers(0, 16)))
    assert_decode_equal(got, oracle.decode_batch(s.nfixed, s.nvar, data, rec_off), f"{schema}/{n}/{density}")


# ---------------------------------------------------------------- tile-key speculation (round 6)
# The parsers read one first length prefix per 64-record tile -- the tile's first SetRequest's -- and
# take it for every SetRequest of the tile; a tile whose keys differ is caught by its copier, the gate
# decodes the batch again exactly and the ctx reads every record's own key length for 1024 calls.
# sym_ctx_decode_redos counts the gate's re-decodes, so these tests see which path ran.

def _pipe_only(decode_impl):
    if decode_impl != "pipe":
        pytest.skip("the speculation and its gate run under the pipeline only")


def _odd_key(b, which, delta=-1):
    """The batch's key column with record(s) `which` given a key `delta` bytes longer (or shorter)."""
    kb, ko = b.var[0]
    keys = [kb[int(ko[i]):int(ko[i + 1])] for i in range(len(ko) - 1)]
    for i in which:
        k = keys[i]
        keys[i] = k[:len(k) + delta] if delta < 0 else np.concatenate([k, np.full(delta, 0x5A, np.uint8)])
    off = np.zeros(len(keys) + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=off[1:])
    return np.concatenate(keys).astype(np.uint8), off


def test_tile_key_fixed_keys_no_redo(codec, dev, decode_impl):
    _pipe_only(decode_impl)
    n = 70001  # ragged last tile
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(64, ("uniform", 0, 300)), seed=41)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    want = oracle.decode_batch(0, 2, stream, off)
    r0 = codec.decode_redos()
    for k in range(3):
        assert_decode_equal(decode_gpu(codec, "kv_set_request", stream, off, dev, misalign=k), want, f"call {k}")
    assert codec.decode_redos() == r0  # one key length per tile was right every time


@pytest.mark.parametrize("where", ["tile_head", "middle", "last"])
def test_tile_key_one_odd_key_is_redecoded(codec, dev, decode_impl, where):
    _pipe_only(decode_impl)
    n = 30000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(64, 256), seed=42)
    i = {"tile_head": 64 * 17, "middle": 64 * 200 + 31, "last": n - 1}[where]
    var = [_odd_key(b, [i], -1 if where != "last" else 5), b.var[1]]
    stream, off = oracle.encode_batch(b.fixed, var)
    want = oracle.decode_batch(0, 2, stream, off)
    r0 = codec.decode_redos()
    assert_decode_equal(decode_gpu(codec, "kv_set_request", stream, off, dev), want, where)
    assert codec.decode_redos() == r0 + 1
    # held: the next calls read every record's own key length (no re-decode), results unchanged
    assert_decode_equal(decode_gpu(codec, "kv_set_request", stream, off, dev), want, where + " held")
    assert codec.decode_redos() == r0 + 1


def test_tile_key_hold_then_layout_miss_then_impl_reset(codec, dev, decode_impl):
    """Varying keys: one re-decode, then the tile hold (per-record key lengths, no re-decode); a batch
    off the generator's layout during it re-decodes too; set_decode_impl clears the holds."""
    _pipe_only(decode_impl)
    n = 20000
    b = datagen.make_batch(schema="kv_set_request", n=n, lens=(("uniform", 0, 80), ("uniform", 0, 300)), seed=43)
    stream, off = oracle.encode_batch(b.fixed, b.var)
    want = oracle.decode_batch(0, 2, stream, off)
    bad, bad_off = _with_trailers(stream, off, [5, 9000], extra=3, seed=4)
    want_bad = oracle.decode_batch(0, 2, bad, bad_off)
    r0 = codec.decode_redos()
    steps = [(False, 1), (False, 1), (False, 1), (True, 2), (False, 2), (False, 2)]
    for k, (misfit, redos) in enumerate(steps):
        got = decode_gpu(codec, "kv_set_request", bad if misfit else stream, bad_off if misfit else off, dev)
        assert_decode_equal(got, want_bad if misfit else want, f"step {k}")
        assert codec.decode_redos() == r0 + redos, f"step {k}"
    codec.set_decode_impl(0)  # clears both holds: tile-key speculation again, which misses again
    assert_decode_equal(decode_gpu(codec, "kv_set_request", stream, off, dev), want, "after reset")
    assert codec.decode_redos() == r0 + 3


def test_tile_key_mixed_batches(codec, dev, decode_impl):
    """Mixed Get/Set batches: the tile's key length is its first SetRequest's (tiles may start with
    GetRequests, whose key lengths are never read); fixed keys never re-decode, one odd SetRequest key
    re-decodes once."""
    _pipe_only(decode_impl)
    m = datagen.make_mixed_batch(n=50000, key=64, value=("uniform", 0, 256), set_fraction=datagen.TRACE_SET_FRACTION,
                                 seed=44)
    t = torch.from_numpy(m.type).to(dev)

    def run(key):
        stream, off = oracle.encode_kv_mixed(m.type, key, m.val)
        _, d = put(stream, dev, 1)
        _, ro = put(off, dev)
        out = codec.decode_kv_mixed(d, ro, t)
        codec.check()
        wcols, wst = oracle.decode_kv_mixed(stream, off, m.type)
        np.testing.assert_array_equal(out.status.cpu().numpy()[:m.n], wst)
        for (gb, go), (wb, wo) in zip(out.var, wcols):
            go = go.cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(go, wo)
            np.testing.assert_array_equal(gb.cpu().numpy()[:int(wo[-1])], wb)

    r0 = codec.decode_redos()
    run(m.key)
    run(m.key)
    assert codec.decode_redos() == r0
    sets = np.flatnonzero(m.type != 0)
    tile = int(sets[500]) // 64
    first_set = int(sets[np.searchsorted(sets, 64 * tile)])  # the first SetRequest of that tile
    odd = _odd_key(type("B", (), {"var": [m.key]})(), [first_set], -3)
    run(odd)
    assert codec.decode_redos() == r0 + 1

"""Repeated string / bytes and nested messages: the GPU codec vs the generator.

Schemas are cmd/symphony-gen-arpc/test/test.proto:41-77 (RepeatedVar, Leaf, Level2, Level1, Root,
ComplexMixed); the inputs are the reference's own test inputs (serialization_test.go:277-284
TestRepeatedVar, :325-337 TestDeepNested, :414-427 TestComplexMixed, and the Raw_Manipulation
values :433-507), checked as the reference checks them (Marshal -> Unmarshal -> DeepEqual) and,
byte for byte, against layouts written out by hand from the generator and against the CPU
restatement oracle/nested_ref.py.  Byte parity with Go itself stays unpinned (no Go toolchain,
no vectors in the reference).
"""
import random
import struct

import numpy as np
import pytest

from arpc_amd.flat import FlatField as F, FlatSchema as S, ListColumn, MessageColumn
from oracle import nested_ref as ref

# test.proto:41-77
REPEATED_VAR = S("RepeatedVar", (F("RString", "string", True, True), F("RBytes", "bytes", False, True)))
LEAF = S("Leaf", (F("LeafId", "int32", True), F("LeafVal", "string")))
LEVEL2 = S("Level2", (F("Leaf", "message", True, message=LEAF),))
LEVEL1 = S("Level1", (F("L2", "message", message=LEVEL2), F("L1Data", "string", True)))
ROOT = S("Root", (F("L1", "message", True, message=LEVEL1), F("RootId", "int32")))
COMPLEX = S("ComplexMixed", (F("FInt32", "int32"), F("VString", "string", True), F("RInt64", "int64", False, True),
                             F("NestedLeaf", "message", True, message=LEAF), F("RString", "string", False, True),
                             F("FBool", "bool", True), F("RepeatedNested", "message", False, True, message=ROOT),
                             F("VBytes", "bytes", True)))
EMPTY = S("Empty", ())

i32 = lambda v: struct.pack("<i", v)  # noqa: E731
u32 = lambda v: struct.pack("<I", v)  # noqa: E731

# serialization_test.go:279-282
REPVAR_IN = {"RString": [b"one", b"two", b""], "RBytes": [b"\x01", b"\x02\x03", b""]}
# :327-335
ROOT_IN = {"RootId": i32(1), "L1": {"L1Data": b"L1", "L2": {"Leaf": {"LeafId": i32(10), "LeafVal": b"Deep"}}}}
# :416-425
COMPLEX_IN = {"FInt32": i32(123), "VString": b"Mixed", "RInt64": struct.pack("<2q", 1, 2),
              "NestedLeaf": {"LeafId": i32(0), "LeafVal": b"Nested"}, "RString": [b"S1", b"S2"], "FBool": b"\x01",
              "RepeatedNested": [ROOT_IN], "VBytes": b"\x00"}
# :433-437 and the values the Raw_Manipulation steps set (:447-507)
COMPLEX_RAW = {"FInt32": i32(999), "VString": b"NewString", "RInt64": struct.pack("<3q", 5, 6, 7),
               "NestedLeaf": {"LeafId": i32(42), "LeafVal": b"NewLeaf"}, "RString": [b"Str1", b"Str2", b"Str3"],
               "FBool": b"\x01", "RepeatedNested": [{"RootId": i32(1), "L1": {"L1Data": b"R1", "L2": None}},
                                                   {"RootId": i32(2), "L1": {"L1Data": b"R2", "L2": None}}],
               "VBytes": b"\xaa\xbb\xcc"}


def full(schema, rec):
    """The fresh-struct defaults filled in (what Unmarshal returns)."""
    out = {f.name: ref.default(f) for f in schema.fields}
    for f in schema.fields:
        v = rec.get(f.name, out[f.name])
        if f.kind == "message":
            v = None if v is None and not f.repeated else ([full(f.message, x) for x in v] if f.repeated else full(f.message, v))
        out[f.name] = v
    return out


def test_hand_kat_repeated_var():
    """RepeatedVar{["one","two",""], [{1},{2,3},{}]}: r_string public at 17 (off2p 39), r_bytes
    private at 44 (entry 44 - 39 = 5), 63 bytes."""
    want = (b"\x01" + u32(39) + b"\x00" * 8 + u32(17) + u32(3) + u32(3) + b"one" + u32(3) + b"two" + u32(0) +
            b"\x01" + u32(5) + u32(3) + u32(1) + b"\x01" + u32(2) + b"\x02\x03" + u32(0))
    assert len(want) == 63
    assert ref.marshal(REPEATED_VAR, REPVAR_IN) == want


def test_hand_kat_deep_nested():
    """Root{1, L1{"L1", L2{Leaf{10, "Deep"}}}}: Leaf 30 B, Level2 52 B (no private fields: marker
    only), Level1 84 B (l2 private, entry 28 - 23 = 5), Root 110 B (off2p 105)."""
    leaf = b"\x01" + u32(17) + b"\x00" * 8 + i32(10) + b"\x01" + u32(5) + u32(4) + b"Deep"
    lvl2 = b"\x01" + u32(51) + b"\x00" * 8 + u32(17) + u32(30) + leaf + b"\x01"
    lvl1 = b"\x01" + u32(23) + b"\x00" * 8 + u32(17) + u32(2) + b"L1" + b"\x01" + u32(5) + u32(52) + lvl2
    root = b"\x01" + u32(105) + b"\x00" * 8 + u32(17) + u32(84) + lvl1 + b"\x01" + i32(1)
    assert (len(leaf), len(lvl2), len(lvl1), len(root)) == (30, 52, 84, 110)
    assert ref.marshal(ROOT, ROOT_IN) == root


def test_hand_kat_nil_nested():
    """A nil nested message: 0 table entry, no payload (main.go:586-588)."""
    b = ref.marshal(ROOT, {"RootId": i32(7)})
    assert b == b"\x01" + u32(17) + b"\x00" * 8 + u32(0) + b"\x01" + i32(7)


@pytest.mark.parametrize("schema,rec", [(REPEATED_VAR, REPVAR_IN), (ROOT, ROOT_IN), (COMPLEX, COMPLEX_IN),
                                        (COMPLEX, COMPLEX_RAW), (EMPTY, {})])
def test_oracle_round_trip(schema, rec):
    """runRoundTrip (serialization_test.go:19-38) on the restatement."""
    st, got, fail = ref.unmarshal(schema, ref.marshal(schema, rec))
    assert st == ref.OK and fail == len(schema.fields)
    assert got == full(schema, rec)


def test_oracle_unmarshal_edges():
    """A list keeps the items that fit; a bad inner message is NESTED at the field's position."""
    b = bytearray(ref.marshal(REPEATED_VAR, REPVAR_IN))
    st, got, _ = ref.unmarshal(REPEATED_VAR, bytes(b[:30]))  # cuts r_string after "one"'s bytes
    assert st == ref.NO_PRIVATE
    b2 = bytearray(ref.marshal(ROOT, ROOT_IN))
    b2[17 + 4] = 7  # Level1's public version byte
    st, got, fail = ref.unmarshal(ROOT, bytes(b2))
    assert st == ref.NESTED and fail == 0
    st, got, fail = ref.unmarshal(ROOT, bytes(b2[:106]))  # also cuts root_id: the nested error comes first
    assert st == ref.NESTED


# ---------------------------------------------------------------- random trees
def rand_value(rng, f, depth):
    if f.kind == "message":
        if f.repeated:
            return [rand_rec(rng, f.message, depth + 1) for _ in range(rng.randrange(0, 4))]
        return None if rng.random() < 0.3 else rand_rec(rng, f.message, depth + 1)
    w = ref.WIDTH[f.kind]
    if f.repeated and not w:
        return [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 9))) for _ in range(rng.randrange(0, 5))]
    if f.repeated:
        return bytes(rng.randrange(256) for _ in range(w * rng.randrange(0, 4)))
    if w:
        return bytes(rng.randrange(256) for _ in range(w))
    return bytes(rng.randrange(256) for _ in range(rng.randrange(0, 20)))


def rand_rec(rng, schema, depth=0):
    return {f.name: rand_value(rng, f, depth) for f in schema.fields}


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


def _packed(vals, dev):
    off = np.zeros(len(vals) + 1, np.int64)
    np.cumsum([len(v) for v in vals], out=off[1:])
    b = np.frombuffer(b"".join(vals) + b"\x00" * 16, np.uint8).copy()
    return torch.from_numpy(b).to(dev)[:max(1, int(off[-1]))], torch.from_numpy(off).to(dev)


def to_columns(schema, recs, dev):
    """Python records -> the column layout of arpc_amd.flat (recursively)."""
    cols = []
    for f in schema.fields:
        vals = [r.get(f.name, ref.default(f)) for r in recs]
        w = ref.WIDTH[f.kind]
        if f.kind == "message":
            items = [x for v in vals for x in (v if f.repeated else ([] if v is None else [v]))]
            counts = [len(v) if f.repeated else (0 if v is None else 1) for v in vals]
            rec = np.zeros(len(vals) + 1, np.int64)
            np.cumsum(counts, out=rec[1:])
            cols.append(MessageColumn(to_columns(f.message, items, dev), torch.from_numpy(rec).to(dev)))
        elif f.repeated and not w:
            items = [x for v in vals for x in v]
            rec = np.zeros(len(vals) + 1, np.int64)
            np.cumsum([len(v) for v in vals], out=rec[1:])
            b, io = _packed(items, dev)
            cols.append(ListColumn(b, io, torch.from_numpy(rec).to(dev)))
        elif w and not f.repeated:
            dt = {1: torch.uint8, 4: torch.int32, 8: torch.int64}[w]
            a = np.frombuffer(b"".join(vals), np.uint8).copy() if vals else np.zeros(0, np.uint8)
            cols.append(torch.from_numpy(a.view({1: np.uint8, 4: np.int32, 8: np.int64}[w]).copy()).to(dev).view(dt))
        else:
            cols.append(_packed(vals, dev))
    return cols


def from_columns(schema, cols, n):
    """Decoded columns -> Python records (recursively)."""
    recs = [dict() for _ in range(n)]
    for f, c in zip(schema.fields, cols):
        w = ref.WIDTH[f.kind]
        if f.kind == "message":
            inner = from_columns(f.message, c.cols, c.n_items)
            rec = c.rec.cpu().numpy()
            for i in range(n):
                its = inner[rec[i] - rec[0]:rec[i + 1] - rec[0]]
                recs[i][f.name] = its if f.repeated else (its[0] if its else None)
        elif f.repeated and not w:
            b = c.bytes.cpu().numpy().tobytes()
            io = c.item_off.cpu().numpy()
            rec = c.rec.cpu().numpy()
            for i in range(n):
                recs[i][f.name] = [b[io[j]:io[j + 1]] for j in range(rec[i], rec[i + 1])]
        elif w and not f.repeated:
            a = c.cpu().numpy().view(np.uint8).reshape(-1, w) if n else np.zeros((0, w), np.uint8)
            for i in range(n):
                recs[i][f.name] = a[i].tobytes()
        else:
            b, o = c
            b = b.cpu().numpy().tobytes()
            o = o.cpu().numpy()
            for i in range(n):
                recs[i][f.name] = b[o[i]:o[i + 1]]
    return recs


def gpu_round_trip(codec, schema, recs, dev):
    from arpc_amd import flat
    data, off = flat.encode(codec, schema, to_columns(schema, recs, dev), n=len(recs))
    codec.check()
    got = data.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    want = [ref.marshal(schema, r) for r in recs]
    assert [got[o[i]:o[i + 1]] for i in range(len(recs))] == want
    cols, st = flat.decode(codec, schema, data, off)
    codec.check()
    assert (st.cpu().numpy() == 0).all()
    assert from_columns(schema, cols, len(recs)) == [full(schema, r) for r in recs]


@pytest.mark.gpu
@pytest.mark.parametrize("name,schema,rec", [("RepeatedVar", REPEATED_VAR, REPVAR_IN), ("DeepNested", ROOT, ROOT_IN),
                                             ("ComplexMixed", COMPLEX, COMPLEX_IN),
                                             ("ComplexMixedRaw", COMPLEX, COMPLEX_RAW)])
def test_gpu_reference_inputs(codec, dev, name, schema, rec):
    """The reference's inputs, interleaved with the zero value, across tiles: GPU bytes == the
    generator's, and Marshal -> Unmarshal returns the input."""
    recs = [rec if i % 3 else {} for i in range(700)]
    gpu_round_trip(codec, schema, recs, dev)


@pytest.mark.gpu
@pytest.mark.parametrize("schema", [REPEATED_VAR, ROOT, COMPLEX, LEVEL1])
def test_gpu_random_trees(codec, dev, schema):
    rng = random.Random(7 + len(schema.fields))
    for n in (1, 63, 300):
        gpu_round_trip(codec, schema, [rand_rec(rng, schema) for _ in range(n)], dev)


@pytest.mark.gpu
@pytest.mark.parametrize("schema", [REPEATED_VAR, ROOT, COMPLEX])
def test_gpu_decode_corrupted(codec, dev, schema):
    """Truncated and byte-flipped records: statuses (including NESTED from inner messages) and the
    values of OK records match the restatement."""
    from arpc_amd import flat
    rng = random.Random(11 + len(schema.fields))
    bufs = []
    for _ in range(400):
        b = bytearray(ref.marshal(schema, rand_rec(rng, schema)))
        r = rng.random()
        if r < 0.3:
            b = b[:rng.randrange(0, len(b) + 1)]
        elif r < 0.7 and b:
            for _ in range(rng.randrange(1, 4)):
                b[rng.randrange(len(b))] = rng.choice([0, 1, 2, 0xff, rng.randrange(256)])
        bufs.append(bytes(b))
    data, off = _packed(bufs, dev)
    cols, st, fail = flat.decode(codec, schema, data, off, with_fail=True)
    codec.check()
    st = st.cpu().numpy()
    fail = fail.cpu().numpy()
    got = from_columns(schema, cols, len(bufs))
    for i, b in enumerate(bufs):
        ws, wrec, wfail = ref.unmarshal(schema, b)
        assert st[i] == ws, (i, b.hex())
        if ws == ref.OK:
            assert got[i] == wrec, i
        elif ws != ref.NESTED:
            assert fail[i] == wfail, i


@pytest.mark.gpu
def test_gpu_nested_item_count_checked(codec, dev):
    """Two items for a (non-repeated) nested field is an argument error."""
    from arpc_amd import flat
    recs = [{"L1": {"L1Data": b"x"}}, {"L1": {"L1Data": b"y"}}]
    cols = to_columns(ROOT, recs, dev)
    cols[0].rec = torch.tensor([0, 2, 2], dtype=torch.int64, device=dev)
    flat.encode(codec, ROOT, cols, n=2)
    with pytest.raises(Exception):
        codec.check()


WRAP = S("Wrap", (F("Inner", "message", message=LEVEL1),))  # one private nested message: a wrapper


@pytest.mark.gpu
@pytest.mark.parametrize("nil_every", [0, 1, 7])
@pytest.mark.parametrize("ids", [(0, 0), (3, 4)])
def test_gpu_wrapper_level(codec, dev, nil_every, ids):
    """A wrapper message (one private nested field: flat._wrapper) is written by its inner level's
    kernel -- the 18 wrapper bytes as that kernel's frame prefix -- when every record has its item,
    and by its own kernel when one is nil (both queued, gated on the device).  Bytes == the
    generator's either way (with the client's ID patch in [5:13]), offsets included, and the round
    trip returns the input."""
    from arpc_amd import flat
    rng = random.Random(31 + nil_every)
    n = 700
    recs = [{"Inner": None if nil_every and i % nil_every == 3 else rand_rec(rng, LEVEL1)} for i in range(n)]
    if nil_every == 1:  # every record nil
        recs = [{"Inner": None} for _ in range(n)]
    data, off = flat.encode(codec, WRAP, to_columns(WRAP, recs, dev), service_id=ids[0], method_id=ids[1])
    codec.check()
    got = data.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    want = []
    for r in recs:
        b = bytearray(ref.marshal(WRAP, r))
        b[5:13] = struct.pack("<II", *ids)
        want.append(bytes(b))
    assert o[0] == 0 and [got[o[i]:o[i + 1]] for i in range(n)] == want
    assert len(got) == sum(len(w) for w in want)
    cols, st = flat.decode(codec, WRAP, data, off)
    codec.check()
    assert (st.cpu().numpy() == 0).all()
    assert from_columns(WRAP, cols, n) == [full(WRAP, r) for r in recs]


@pytest.mark.gpu
def test_gpu_wrapper_level_bad_item_ranges(codec, dev):
    """Item ranges that sum to n but give one record two items (and another none): the fused path's
    gate passes, and its per-record check reports what the wrapper's own kernel would
    (SYM_ERR_INVALID, "more than one item for a nested field")."""
    from arpc_amd import flat
    recs = [{"Inner": {"L1Data": b"x"}}, {"Inner": {"L1Data": b"y"}}]
    cols = to_columns(WRAP, recs, dev)
    cols[0].rec = torch.tensor([0, 2, 2], dtype=torch.int64, device=dev)
    flat.encode(codec, WRAP, cols)
    with pytest.raises(Exception):
        codec.check()


@pytest.mark.gpu
def test_gpu_wrapper_under_graph_capture(dev):
    """The two gated alternatives replay from one captured graph, which follows the data: item ranges
    refilled in place switch a replay from the fused path to the wrapper's own kernel."""
    from arpc_amd import flat
    rng = random.Random(5)
    n = 300
    recs = [{"Inner": rand_rec(rng, LEVEL1)} for _ in range(n)]
    cols = to_columns(WRAP, recs, dev)
    g = flat.EncodeGraph(dev, WRAP, cols)
    for rep in range(2):
        data, off = g.replay()
        torch.cuda.synchronize()
        g.codec.check()
        o = off.cpu().numpy()
        got = data.cpu().numpy().tobytes()
        assert [got[o[i]:o[i + 1]] for i in range(n)] == [ref.marshal(WRAP, r) for r in recs], rep
        # refill the item ranges in place: record 5 loses its item, records after it take the next one
        rec = np.arange(n + 1, dtype=np.int64)
        rec[6:] -= 1
        cols[0].rec.copy_(torch.from_numpy(rec))
        recs = recs[:5] + [{"Inner": None}] + recs[5:-1]


def tree_records(schema, nodes, n):
    """arpc_amd.datagen column trees -> Python records (the restatement's input form)."""
    recs = [dict() for _ in range(n)]
    for f, nd in zip(schema.fields, nodes):
        w = ref.WIDTH[f.kind]
        if f.kind == "message":
            _, children, rec = nd
            m = int(rec[-1] - rec[0])
            inner = tree_records(f.message, children, m)
            for i in range(n):
                its = inner[rec[i] - rec[0]:rec[i + 1] - rec[0]]
                recs[i][f.name] = its if f.repeated else (its[0] if its else None)
        elif f.repeated and not w:
            _, b, io, rec = nd
            for i in range(n):
                recs[i][f.name] = [b[io[j]:io[j + 1]].tobytes() for j in range(rec[i], rec[i + 1])]
        elif w and not f.repeated:
            for i in range(n):
                recs[i][f.name] = nd[i:i + 1].tobytes()
        else:
            b, o = nd
            for i in range(n):
                recs[i][f.name] = b[o[i]:o[i + 1]].tobytes()
    return recs


@pytest.mark.gpu
def test_gpu_online_boutique(codec, dev):
    """PlaceOrderResponse batches (onlineboutique.proto, three message levels, repeated nested):
    GPU bytes == the restatement's MarshalSymphony per record, and the decode round trips."""
    from arpc_amd import datagen, flat
    sch = flat.OB_PLACE_ORDER_RESPONSE
    n = 500
    tree = datagen.ob_place_order(n, seed=3)
    recs = tree_records(sch, tree[1], n)
    data, off = flat.encode(codec, sch, flat.columns_from_tree(sch, tree[1], dev))
    codec.check()
    got = data.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    assert [got[o[i]:o[i + 1]] for i in range(n)] == [ref.marshal(sch, r) for r in recs]
    cols, st = flat.decode(codec, sch, data, off)
    codec.check()
    assert (st.cpu().numpy() == 0).all()
    assert from_columns(sch, cols, n) == [full(sch, r) for r in recs]


@pytest.mark.gpu
def test_gpu_in_place_level_matches_packed_items(codec, dev):
    """sym_flat_decode_ex with d_item_len leaves a message field's items in place ((offset, length)
    into the input); without it the items are gathered into an item column.  The inner level decoded from
    either is the same (boutique OrderResults -> their repeated OrderItems)."""
    from arpc_amd import _native, datagen, flat
    from arpc_amd.codec import _dptr
    outer = flat.OB_ORDER_RESULT
    n = 700
    tree = datagen.ob_place_order(n, seed=9)
    ob, oo = flat.encode(codec, outer, flat.columns_from_tree(outer, tree[1][0][1], dev))
    codec.check()
    k = [f.name for f in outer.fields].index("Items")
    span = ob.numel()
    icap = span // 4 + 1

    def run(inplace):
        cols, caps, offs, items, ilens, icaps, t = [], [], [], [], [], [], {}
        for j, f in enumerate(outer.fields):
            if f.list_like:
                msg = inplace and j == k
                t[j] = dict(b=torch.empty(1 if msg else span, dtype=torch.uint8, device=dev),
                            io=torch.empty(icap + 1, dtype=torch.int64, device=dev),
                            il=torch.empty(icap, dtype=torch.int64, device=dev),
                            rec=torch.empty(n + 1, dtype=torch.int64, device=dev))
                cols.append(_dptr(t[j]["b"]))
                caps.append(0 if msg else span)
                offs.append(_dptr(t[j]["rec"]))
                items.append(_dptr(t[j]["io"]))
                ilens.append(_dptr(t[j]["il"]) if msg else 0)
                icaps.append(icap)
            else:
                t[j] = dict(b=torch.empty(span, dtype=torch.uint8, device=dev),
                            o=torch.empty(n + 1, dtype=torch.int64, device=dev))
                cols.append(_dptr(t[j]["b"]))
                caps.append(span)
                offs.append(_dptr(t[j]["o"]))
                items.append(0)
                ilens.append(0)
                icaps.append(0)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        _native.check(codec._lib.sym_flat_decode_ex(
            codec._ctx, outer.c_fields(), len(outer.fields), n, None, _dptr(ob), _dptr(oo), 0, 0, 0,
            _native.ptr_array(cols), _native.u64_array(caps), _native.ptr_array(offs), _native.ptr_array(items),
            _native.ptr_array(ilens), _native.u64_array(icaps), _dptr(st), 0, 0), "sym_flat_decode_ex")
        codec.check()
        assert (st.cpu().numpy() == 0).all()
        it = t[k]
        m = int((it["rec"][n] - it["rec"][0]).item())
        if inplace:
            icols, ist = flat.decode(codec, outer.fields[k].message, ob, it["io"][:m], span=span,
                                     rec_len=it["il"][:m], extent=(_dptr(oo), _dptr(oo) + 8 * n))
        else:
            nb = int(it["io"][m].item())
            icols, ist = flat.decode(codec, outer.fields[k].message, it["b"][:nb], it["io"][:m + 1])
        codec.check()
        return m, icols, ist

    m1, c1, s1 = run(True)
    m2, c2, s2 = run(False)
    assert m1 == m2 > n
    assert torch.equal(s1, s2) and (s1.cpu().numpy() == 0).all()
    assert from_columns(outer.fields[k].message, c1, m1) == from_columns(outer.fields[k].message, c2, m2)


@pytest.mark.gpu
def test_gpu_decode_ex_in_place_argument_checks(codec, dev):
    from arpc_amd import _native, flat
    from arpc_amd.codec import _dptr
    sch = flat.OB_MONEY  # no message field
    data = torch.zeros(64, dtype=torch.uint8, device=dev)
    off = torch.tensor([0, 20], dtype=torch.int64, device=dev)
    ln = torch.tensor([20], dtype=torch.int64, device=dev)
    b = torch.empty(64, dtype=torch.uint8, device=dev)
    o = torch.empty(2, dtype=torch.int64, device=dev)
    v = torch.empty(8, dtype=torch.uint8, device=dev)
    st = torch.empty(1, dtype=torch.uint8, device=dev)
    cf = sch.c_fields()
    args = dict(cols=_native.ptr_array([_dptr(b), _dptr(v), _dptr(v)]), caps=_native.u64_array([64, 0, 0]),
                offs=_native.ptr_array([_dptr(o), 0, 0]))
    # records in place need the input's extent
    rc = codec._lib.sym_flat_decode_ex(codec._ctx, cf, 3, 1, None, _dptr(data), _dptr(off), _dptr(ln), 0, 0, args["cols"],
                                        args["caps"], args["offs"], None, None, None, _dptr(st), 0, 0)
    assert rc == _native.SYM_ERR_INVALID
    # an in-place item column only for a message field
    io = torch.empty(2, dtype=torch.int64, device=dev)
    sch2 = flat.FlatSchema("L", (flat.FlatField("S", "string", repeated=True),))
    rc = codec._lib.sym_flat_decode_ex(codec._ctx, sch2.c_fields(), 1, 1, None, _dptr(data), _dptr(off), 0, 0, 0,
                                        _native.ptr_array([_dptr(b)]), _native.u64_array([64]),
                                        _native.ptr_array([_dptr(o)]), _native.ptr_array([_dptr(io)]),
                                        _native.ptr_array([_dptr(io)]), _native.u64_array([1]), _dptr(st), 0, 0)
    assert rc == _native.SYM_ERR_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("recs", [[], [{"RootId": i32(5)}, {"RootId": i32(6)}, {"RootId": i32(7)}]],
                         ids=["no records", "every nested message nil"])
def test_gpu_empty_levels(codec, dev, recs):
    """A batch of no records, and one whose nested fields are all nil: the inner levels (decoded in
    place) have no records."""
    gpu_round_trip(codec, ROOT, recs, dev)

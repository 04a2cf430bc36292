"""The 16-field maximum-width schema through EVERY schema-driven C entry point (kernel-argument guard).

A GPU fault once came from a per-field byte array in a kernel-argument struct: the compiler folded
the field index into a scalar load base at a misaligned kernarg offset (general
schemas).  The arrays are 32-bit now and `SYMHIP_KERNARG_ARRAY` (arpc_amd/csrc/codec.hpp)
static-asserts that for every indexed kernarg array; this test drives SYM_MAX_FLAT_FIELDS = 16 fields
-- narrow and wide kinds interleaved, public and private alternating, the last field indexed 15 --
through sym_flat_encoded_size / sym_flat_encode / sym_flat_decode (plain), sym_flat_encoded_size_ex /
sym_flat_encode_ex / sym_flat_decode_ex / sym_flat_nested_status (list-like and nested fields),
sym_raw_set on every field, and sym_raw_get_fixed / sym_raw_get_bytes at every table position,
bit-exact against the restatements (oracle/flat_oracle.c, oracle/raw_oracle.c,
oracle/nested_ref.py; generator main.go:196-368, :439-620, :622-947, :984-1099, :1296-1740).
"""
import random

import numpy as np
import pytest

from arpc_amd.flat import FlatField as F, FlatSchema as S
from oracle import nested_ref as ref
from oracle import oracle
from test_flat import REP, _check_decode, _check_encode, corrupt, random_columns, scalar
from test_nested import LEAF, from_columns, full, gpu_round_trip, rand_rec, to_columns
from test_raw_setters import gpu_set, make_batch, make_values

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

# 16 flat fields: (segment 0 public / 1 private, width | REP)
WIDE16 = [(0, 1), (1, 1), (0, REP | 1), (1, 0), (0, 8), (1, REP | 4), (0, 0), (1, 4),
          (0, REP | 8), (1, 1), (0, 4), (1, 0), (0, 1), (1, REP | 1), (0, 0), (1, 8)]
# 16 fields with list-like ones: repeated strings, a nested message, a repeated message last (index 15)
WIDE16_NESTED = S("Wide16Nested", (
    F("b0", "bool", True), F("s1", "string"), F("rs2", "string", True, True), F("m3", "message", message=LEAF),
    F("u4", "uint64", True), F("ri5", "int32", False, True), F("s6", "bytes", True), F("i7", "int32"),
    F("rb8", "bytes", True, True), F("b9", "bool"), F("f10", "float", True), F("m11", "message", True, message=LEAF),
    F("b12", "bool", True), F("rl13", "int64", False, True), F("s14", "string", True),
    F("rm15", "message", False, True, message=LEAF)))


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


def _c_fields(fields):
    from arpc_amd import _native
    arr = (_native.SymField * len(fields))()
    for k, (seg, w) in enumerate(fields):
        arr[k].segment, arr[k].width = seg, w
    return arr


def test_wide16_plain_entry_points(codec, dev):
    """sym_flat_encoded_size, sym_flat_encode, sym_flat_decode called directly through the C ABI."""
    from arpc_amd import _native
    from arpc_amd.codec import _dptr, _stream_handle
    rng = np.random.default_rng(16)
    n = 1300
    cols = random_columns(rng, WIDE16, n)
    want, woff = oracle.flat_encode(WIDE16, cols, n, 7, 9)
    L, cf = codec._lib, _c_fields(WIDE16)
    var_total = sum(int(c[1][-1]) for (seg, w), c in zip(WIDE16, cols) if not scalar(w))
    size = L.sym_flat_encoded_size(cf, 16, n, var_total)
    assert size == len(want)
    keep, ptrs, offs = [], [], []
    for (seg, w), c in zip(WIDE16, cols):
        if scalar(w):
            t = torch.from_numpy(np.ascontiguousarray(c).reshape(-1).copy()).to(dev)
            keep.append(t)
            ptrs.append(_dptr(t))
            offs.append(0)
        else:
            b = torch.from_numpy(np.concatenate([c[0], np.zeros(16, np.uint8)])).to(dev)
            o = torch.from_numpy(c[1].view(np.int64).copy()).to(dev)
            keep += [b, o]
            ptrs.append(_dptr(b))
            offs.append(_dptr(o))
    out = torch.empty(size + 16, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    hs = _stream_handle(dev, None)
    _native.check(L.sym_flat_encode(codec._ctx, cf, 16, n, _native.ptr_array(ptrs), _native.ptr_array(offs), 7, 9,
                                    _dptr(out), _dptr(off), hs), "sym_flat_encode")
    codec.check()
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), woff)
    np.testing.assert_array_equal(out[:size].cpu().numpy(), want)
    # decode a corrupted copy of the stream with the plain entry point
    data, doff = corrupt(want, woff, rng, frac=0.4)
    wcols, wst = oracle.flat_decode(WIDE16, data, doff)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)
    ro = torch.from_numpy(doff.view(np.int64).copy()).to(dev)
    span = int(doff[-1])
    dcols, dptrs, caps, doffs = [], [], [], []
    for seg, w in WIDE16:
        if scalar(w):
            t = torch.empty(n * w, dtype=torch.uint8, device=dev)
            dcols.append(t)
            dptrs.append(_dptr(t))
            caps.append(0)
            doffs.append(0)
        else:
            b = torch.empty(span + 16, dtype=torch.uint8, device=dev)
            o = torch.empty(n + 1, dtype=torch.int64, device=dev)
            dcols.append((b, o))
            dptrs.append(_dptr(b))
            caps.append(span)
            doffs.append(_dptr(o))
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    _native.check(L.sym_flat_decode(codec._ctx, cf, 16, n, _dptr(d), _dptr(ro), _native.ptr_array(dptrs),
                                    _native.u64_array(caps), _native.ptr_array(doffs), _dptr(st), hs),
                  "sym_flat_decode")
    codec.check()
    np.testing.assert_array_equal(st.cpu().numpy(), wst)
    assert (wst != 0).any() and (wst == 0).any()
    for k, (seg, w) in enumerate(WIDE16):
        if scalar(w):
            np.testing.assert_array_equal(dcols[k].cpu().numpy().reshape(-1, w), wcols[k].reshape(-1, w),
                                          err_msg=f"field {k}")
        else:
            go = dcols[k][1].cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(go, wcols[k][1], err_msg=f"offsets {k}")
            np.testing.assert_array_equal(dcols[k][0][:int(go[-1])].cpu().numpy(), wcols[k][0], err_msg=f"bytes {k}")


def test_wide16_ex_entry_points_flat(codec, dev):
    """The same schema through the _ex entry points (arpc_amd.flat), valid and corrupted streams."""
    rng = np.random.default_rng(61)
    cols = random_columns(rng, WIDE16, 2100)
    data, off = _check_encode(codec, dev, WIDE16, cols, 2100, sid=1, mid=2)
    _check_decode(codec, dev, WIDE16, data, off)
    _check_decode(codec, dev, WIDE16, *corrupt(data, off, rng, frac=0.5))


def test_wide16_nested_entry_points(codec, dev):
    """16 fields with repeated strings, nested and repeated nested messages (index 15): encode_ex /
    decode_ex / nested_status vs the restatement, valid and corrupted records."""
    from arpc_amd import flat
    rng = random.Random(1616)
    gpu_round_trip(codec, WIDE16_NESTED, [rand_rec(rng, WIDE16_NESTED) for _ in range(300)], dev)
    bufs = []
    for _ in range(400):
        b = bytearray(ref.marshal(WIDE16_NESTED, rand_rec(rng, WIDE16_NESTED)))
        if rng.random() < 0.6 and b:
            for _ in range(rng.randrange(1, 4)):
                b[rng.randrange(len(b))] = rng.choice([0, 1, 2, 0xff, rng.randrange(256)])
        bufs.append(bytes(b))
    off = np.zeros(len(bufs) + 1, np.int64)
    np.cumsum([len(b) for b in bufs], out=off[1:])
    data = torch.from_numpy(np.frombuffer(b"".join(bufs) + b"\0" * 16, np.uint8).copy()).to(dev)
    cols, st, fail = flat.decode(codec, WIDE16_NESTED, data[:int(off[-1])], torch.from_numpy(off).to(dev),
                                 with_fail=True)
    codec.check()
    st = st.cpu().numpy()
    fail = fail.cpu().numpy()
    got = from_columns(WIDE16_NESTED, cols, len(bufs))
    nested = 0
    for i, b in enumerate(bufs):
        ws, wrec, wfail = ref.unmarshal(WIDE16_NESTED, b)
        assert st[i] == ws, i
        nested += ws == ref.NESTED
        if ws == ref.OK:
            assert got[i] == wrec, i
        elif ws != ref.NESTED:
            assert fail[i] == wfail, i
    assert (st == 0).any() and (st != 0).any()
    _ = full, to_columns  # the helpers gpu_round_trip uses


def test_wide16_raw_setters_every_field(codec, dev):
    """sym_raw_set on each of the 16 fields, buffers complete / public-only / truncated / corrupted."""
    rng = np.random.default_rng(1617)
    for k in range(16):
        data, off = make_batch(rng, WIDE16, 300)
        vals = make_values(rng, WIDE16, k, 300)
        want, woff, wst = oracle.raw_set(WIDE16, k, data, off, vals)
        got, goff, gst = gpu_set(codec, dev, WIDE16, k, data, off, vals)
        np.testing.assert_array_equal(gst, wst, err_msg=f"field {k} status")
        np.testing.assert_array_equal(goff, woff, err_msg=f"field {k} offsets")
        np.testing.assert_array_equal(got, want, err_msg=f"field {k} bytes")


def test_wide16_raw_getters_every_field(codec, dev):
    """sym_raw_get_fixed / sym_raw_get_bytes at each field's table position of the 16-field schema
    (fixed widths 1 / 4 / 8; strings; the count prefix of a repeated field is not a getter case)."""
    rng = np.random.default_rng(1618)
    n = 1000
    want, woff = oracle.flat_encode(WIDE16, random_columns(rng, WIDE16, n), n)
    data, doff = corrupt(want, woff, rng, frac=0.3)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).to(dev)[:len(data)]
    ro = torch.from_numpy(doff.view(np.int64).copy()).to(dev)
    pos = {0: 13, 1: 1}
    for k, (seg, w) in enumerate(WIDE16):
        t = pos[seg]
        pos[seg] += w if scalar(w) else 4
        if scalar(w):
            gv, gs = codec.raw_get_fixed(d, ro, t, w, seg)
            wv, ws = oracle.raw_fixed(data, doff, t, w, bool(seg))
            codec.check()
            np.testing.assert_array_equal(gs.cpu().numpy(), ws, err_msg=f"field {k} status")
            np.testing.assert_array_equal(gv.cpu().numpy().view({1: np.uint8, 4: np.uint32, 8: np.uint64}[w]), wv,
                                          err_msg=f"field {k}")
        elif w == 0:
            gb, go, gs = codec.raw_get_bytes(d, ro, t, seg)
            wb, wo, ws = oracle.raw_bytes(data, doff, t, bool(seg))
            codec.check()
            go = go.cpu().numpy().view(np.uint64)
            np.testing.assert_array_equal(gs.cpu().numpy(), ws, err_msg=f"field {k} status")
            np.testing.assert_array_equal(go, wo, err_msg=f"field {k} offsets")
            np.testing.assert_array_equal(gb[:int(go[-1])].cpu().numpy(), wb, err_msg=f"field {k} bytes")

"""Batched Raw getters and the proxy firewall element.

CPU tests pin the oracle (oracle/raw_oracle.c):
  * with the values of the reference's own access-control test (cmd/symphony-gen-arpc/test/
    serialization_test.go:555-703) on the Fixed message, whose bytes are restated here from the
    generated MarshalSymphony (test.syn.go:152-) -- public getters succeed on complete and
    public-only buffers, private getters succeed on complete buffers and "panic" on public-only ones;
  * with hand-derived vectors for GetRequestRaw.GetScore / GetUsername / GetKey
    (benchmark/kv-store-symphony-element/symphony/kv.syn.go:285-335) and the firewall verdicts
    (cmd/proxy/element/firewall.go:34-52).
GPU tests compare the HIP getters and firewall with the oracle bit-exactly, on valid records and on
corrupted ones (truncations, wild table entries, bad private markers), at batch edges and at the
bench's full size.
"""
import struct

import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle


def batch(recs):
    off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


def fixed_message(f_int32=10, f_int64=20, f_uint32=30, f_uint64=40, f_bool=True, f_float=1.5, f_double=2.5):
    """Fixed{...}.MarshalSymphony() (test.syn.go:152-): 13-byte header, public table of 17 bytes
    (FInt32 @13, FUint32 @17, FBool @21, FDouble @22), private segment at 30: marker, FInt64 @+1,
    FUint64 @+9, FFloat @+17."""
    b = bytearray(51)
    b[0] = 1
    struct.pack_into("<I", b, 1, 30)
    struct.pack_into("<iIBd", b, 13, f_int32, f_uint32, int(f_bool), f_double)
    b[30] = 1
    struct.pack_into("<qQf", b, 31, f_int64, f_uint64, f_float)
    return bytes(b)


# Fixed's fields as (segment private?, table offset, width, struct format)
FIXED_FIELDS = {
    "FInt32": (False, 13, 4, "<i"), "FUint32": (False, 17, 4, "<I"), "FBool": (False, 21, 1, "<?"),
    "FDouble": (False, 22, 8, "<d"), "FInt64": (True, 1, 8, "<q"), "FUint64": (True, 9, 8, "<Q"),
    "FFloat": (True, 17, 4, "<f"),
}
WANT = {"FInt32": 10, "FUint32": 30, "FBool": True, "FDouble": 2.5, "FInt64": 20, "FUint64": 40, "FFloat": 1.5}


def _decode(v, width, fmt):
    return struct.unpack(fmt, int(v).to_bytes(width, "little"))[0]


def element_record(score: int, user: bytes, key: bytes, value: bytes | None = None) -> bytes:
    strings = [(np.frombuffer(x, np.uint8).copy(), np.array([0, len(x)], np.uint64))
               for x in ([user, key] + ([value] if value is not None else []))]
    d, _ = oracle.marshal_element_batch(np.array([score], np.int32), strings)
    return d.tobytes()


# ------------------------------------------------------------------ oracle pinning (CPU)
def test_oracle_access_control_kats():
    """TestPublicPrivateAccessControl (serialization_test.go:555-703), field by field."""
    full = fixed_message()
    public_only = full[:30]  # completeBuffer[:offsetToPrivate]
    data, off = batch([full, public_only])
    for name, (priv, toff, w, fmt) in FIXED_FIELDS.items():
        v, st = oracle.raw_fixed(data, off, toff, w, priv)
        assert st[0] == oracle.RAW_OK and _decode(v[0], w, fmt) == WANT[name], name
        if priv:  # PrivateGetters_PanicOnPublicOnlyBuffer
            assert st[1] == oracle.RAW_PUBLIC_ONLY, name
        else:     # PublicGetters_WorkOnPublicOnlyBuffer
            assert st[1] == oracle.RAW_OK and _decode(v[1], w, fmt) == WANT[name], name


def test_oracle_get_request_raw_kats():
    r = element_record(-7, b"alice", b"k1")
    assert r[:5] == b"\x01" + struct.pack("<I", 30) and r[13:17] == struct.pack("<i", -7)
    assert r[17:21] == struct.pack("<I", 21) and r[21:30] == struct.pack("<I", 5) + b"alice"
    assert r[30] == 1 and r[31:35] == struct.pack("<I", 5) and r[35:] == struct.pack("<I", 2) + b"k1"
    bad_marker = bytearray(r)
    bad_marker[30] = 0
    unset_user = bytearray(r)
    unset_user[17:21] = b"\0\0\0\0"
    wild_user = bytearray(r)
    wild_user[17:21] = struct.pack("<I", 0xFFFFFFF0)
    long_user = bytearray(r)
    long_user[21:25] = struct.pack("<I", 1000)
    recs = [r, r[:16], r[:17], r[:21], r[:29], r[:30], r[:4], bytes(bad_marker), bytes(unset_user), bytes(wild_user),
            bytes(long_user), b""]
    data, off = batch(recs)
    score, _ = oracle.raw_fixed(data, off, 13, 4)
    assert list(score.view(np.int32)) == [-7, 0, -7, -7, -7, -7, 0, -7, -7, -7, -7, 0]  # len < 17 -> 0
    u, uo, _ = oracle.raw_bytes(data, off, 17)
    users = [u[int(uo[i]):int(uo[i + 1])].tobytes() for i in range(len(recs))]
    assert users == [b"alice", b"", b"", b"", b"", b"alice", b"", b"alice", b"", b"", b"", b""]
    k, ko, st = oracle.raw_bytes(data, off, 1, private=True)
    keys = [k[int(ko[i]):int(ko[i + 1])].tobytes() for i in range(len(recs))]
    assert keys[0] == b"k1" and keys[7] == b"" and keys[8] == b"k1"
    assert list(st) == [0, 2, 2, 2, 2, 2, 1, 2, 0, 0, 0, 1]


def test_oracle_firewall_kats():
    recs = [element_record(s, b"u", b"key") for s in (5, 9, 10, 11, -(1 << 31), (1 << 31) - 1)] + [b"\x01" * 16]
    data, off = batch(recs)
    score, verdict, kept, kept_off, kept_index = oracle.firewall(data, off, 10)
    assert list(score) == [5, 9, 10, 11, -(1 << 31), (1 << 31) - 1, 0]
    assert list(verdict) == [1, 1, 2, 2, 1, 2, 1]  # shouldBlock: score >= threshold
    assert list(kept_index) == [0, 1, 4, 6]
    assert kept.tobytes() == recs[0] + recs[1] + recs[4] + recs[6]
    assert list(np.diff(kept_off)) == [len(recs[i]) for i in (0, 1, 4, 6)]


@pytest.mark.parametrize("lens", [(16, 64, 256), (("uniform", 0, 30), ("uniform", 0, 80)),
                                  (("uniform", 0, 9), 0, ("loguniform", 1, 3000))])
@pytest.mark.parametrize("n", [0, 1, 2, 3000])
def test_element_datagen_matches_oracle_marshal(lens, n):
    b = datagen.make_element_batch(n, lens, seed=len(lens) * 7 + 1)
    d, o = oracle.marshal_element_batch(b.score, b.strings)
    np.testing.assert_array_equal(d, b.data)
    np.testing.assert_array_equal(o, b.rec_off)


def corrupted_batch(n: int, seed: int):
    """Element records, a third of them damaged: truncated anywhere (often to the public segment),
    a table entry replaced by a random / huge / zero value, or the private marker cleared."""
    rng = np.random.default_rng(seed)
    b = datagen.make_element_batch(n, (("uniform", 0, 40), ("uniform", 0, 100), ("loguniform", 1, 2000)), seed)
    recs = []
    for i in range(n):
        r = bytearray(b.data[int(b.rec_off[i]):int(b.rec_off[i + 1])].tobytes())
        kind = rng.integers(0, 9)
        off2p = struct.unpack_from("<I", r, 1)[0]
        if kind == 0:
            r = r[:int(rng.integers(0, len(r) + 1))]
        elif kind == 1:
            r = r[:off2p]
        elif kind == 2:
            pos = int(rng.choice([17, 21, off2p + 1, off2p + 5]))
            val = int(rng.choice([0, rng.integers(0, len(r) + 8), 0xFFFFFFFF, rng.integers(0, 1 << 32)]))
            struct.pack_into("<I", r, pos, val)
        elif kind == 3:
            r[off2p] = 0
        elif kind == 4:
            struct.pack_into("<I", r, 1, int(rng.choice([len(r), len(r) + 3, 0xFFFFFFFF])))
        recs.append(bytes(r))
    return recs


def test_oracle_corrupted_batch_is_mixed():
    data, off = batch(corrupted_batch(3000, 5))
    _, st = oracle.raw_fixed(data, off, 1, 4, private=True)
    assert {0, 1, 2} <= set(st.tolist())


# ------------------------------------------------------------------ HIP getters (GPU)
def put(arr: np.ndarray, dev, misalign: int = 0):
    """Copy arr to the GPU at byte offset `misalign` inside a guarded allocation."""
    import torch
    raw = np.ascontiguousarray(arr).view(np.uint8)
    buf = torch.full((raw.size + misalign + 32,), 0xA5, dtype=torch.uint8, device=dev)
    if raw.size:
        buf[misalign:misalign + raw.size].copy_(torch.from_numpy(raw.copy()))
    view = buf[misalign:misalign + raw.size]
    return buf, view.view(torch.int64) if arr.dtype in (np.uint64, np.int64) else view


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


def _on_gpu(dev, data, off, misalign):
    import torch
    _, d = put(np.concatenate([data, np.zeros(1, np.uint8)]), dev, misalign)
    d = d[:len(data)] if len(data) else d[:0]
    _, o = put(off.astype(np.uint64), dev)
    torch.cuda.synchronize()
    return d, o


def _check_getters(codec, dev, data, off, misalign=0):
    d, o = _on_gpu(dev, data, off, misalign)
    n = len(off) - 1
    for priv, toff, w in [(False, 13, 4), (False, 17, 4), (False, 21, 1), (False, 22, 8), (False, 0, 8),
                          (True, 1, 8), (True, 9, 8), (True, 17, 4), (True, 1, 1), (False, 3, 1)]:
        want_v, want_s = oracle.raw_fixed(data, off, toff, w, priv)
        got_v, got_s = codec.raw_get_fixed(d, o, toff, w, int(priv))
        codec.check()
        np.testing.assert_array_equal(got_v.cpu().numpy().view(want_v.dtype), want_v, err_msg=f"fixed {priv} {toff} {w}")
        np.testing.assert_array_equal(got_s.cpu().numpy(), want_s, err_msg=f"status {priv} {toff} {w}")
    for priv, toff in [(False, 17), (True, 1), (True, 5), (False, 13), (False, 1)]:
        want_b, want_o, want_s = oracle.raw_bytes(data, off, toff, priv)
        got_b, got_o, got_s = codec.raw_get_bytes(d, o, toff, int(priv))
        codec.check()
        go = got_o.cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(go, want_o, err_msg=f"offsets {priv} {toff}")
        np.testing.assert_array_equal(got_b[:int(go[n])].cpu().numpy(), want_b, err_msg=f"bytes {priv} {toff}")
        np.testing.assert_array_equal(got_s.cpu().numpy(), want_s, err_msg=f"status {priv} {toff}")


def _check_firewall(codec, dev, data, off, threshold, misalign=0):
    d, o = _on_gpu(dev, data, off, misalign)
    want = oracle.firewall(data, off, threshold)
    r = codec.firewall(d, o, threshold)
    codec.check()
    k = int(r.nkept.item())
    assert k == len(want[4])
    np.testing.assert_array_equal(r.score.cpu().numpy(), want[0], err_msg="score")
    np.testing.assert_array_equal(r.verdict.cpu().numpy(), want[1], err_msg="verdict")
    np.testing.assert_array_equal(r.kept_off[:k + 1].cpu().numpy().view(np.uint64), want[3], err_msg="kept_off")
    np.testing.assert_array_equal(r.kept_index[:k].cpu().numpy().view(np.uint64), want[4], err_msg="kept_index")
    np.testing.assert_array_equal(r.kept[:int(want[3][-1])].cpu().numpy(), want[2], err_msg="kept bytes")
    return want


@pytest.mark.gpu
def test_access_control_kats_gpu(gcodec, gdev):
    data, off = batch([fixed_message(), fixed_message()[:30], fixed_message(-1, -2, 3, 4, False, -0.0, 1e300)])
    _check_getters(gcodec, gdev, data, off, misalign=3)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_getters_corrupted_gpu(gcodec, gdev, seed):
    data, off = batch(corrupted_batch(3000, seed))
    _check_getters(gcodec, gdev, data, off, misalign=seed * 5)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 257])
def test_getters_edge_counts_gpu(gcodec, gdev, n):
    b = datagen.make_element_batch(n, (("uniform", 0, 20), 64, 256), seed=n + 100)
    _check_getters(gcodec, gdev, b.data, b.rec_off)
    _check_firewall(gcodec, gdev, b.data, b.rec_off, 50)


@pytest.mark.gpu
@pytest.mark.parametrize("threshold", [-(1 << 31), 0, 37, 100, (1 << 31) - 1])
def test_firewall_corrupted_gpu(gcodec, gdev, threshold):
    data, off = batch(corrupted_batch(4000, 9))
    _check_firewall(gcodec, gdev, data, off, threshold, misalign=7)


@pytest.mark.gpu
def test_bytes_capacity_error_gpu(gcodec, gdev):
    from arpc_amd import _native
    b = datagen.make_element_batch(100, (16, 8), seed=3)
    d, o = _on_gpu(gdev, b.data, b.rec_off, 0)
    gcodec.raw_get_bytes(d, o, 17, cap=100 * 16 - 1)
    with pytest.raises(_native.SymphonyHipError):
        gcodec.check()
    v, offs, _ = gcodec.raw_get_bytes(d, o, 17, cap=100 * 16)
    gcodec.check()
    assert v.cpu().numpy().tobytes() == b.strings[0][0].tobytes()


@pytest.mark.gpu
def test_firewall_full_size_gpu(gcodec, gdev):
    """The bench's workload (datagen.ELEMENT_FW, 2^20 SetRequests of 378 bytes) against the oracle."""
    b = datagen.make_element_batch(**datagen.ELEMENT_FW)
    want = _check_firewall(gcodec, gdev, b.data, b.rec_off, 50)
    assert 0.45 < len(want[4]) / len(b.score) < 0.55


@pytest.mark.gpu
def test_proxy_firewall_element_gpu(gcodec, gdev):
    from arpc_amd import proxy
    b = datagen.make_element_batch(5000, (("uniform", 0, 20), ("uniform", 1, 64)), seed=21)
    d, o = _on_gpu(gdev, b.data, b.rec_off, 0)
    fw = proxy.FirewallElement(60, gcodec)
    kept, verdict = fw.process_request(proxy.Packets(d, o))
    sel = b.score < 60
    assert (verdict.cpu().numpy() == np.where(sel, proxy.PASS, proxy.DROP)).all()
    user, uoff, _ = proxy.get(gcodec, kept, proxy.field("GetRequest", "Username"))
    key, koff, st = proxy.get(gcodec, kept, proxy.field("GetRequest", "Key"))
    idx = np.nonzero(sel)[0]
    assert (st.cpu().numpy() == 0).all()
    for col, vals, offs in ((b.strings[0], user, uoff), (b.strings[1], key, koff)):
        cb, co = col
        want = b"".join(cb[int(co[i]):int(co[i + 1])].tobytes() for i in idx)
        assert vals[:int(offs[-1].item())].cpu().numpy().tobytes() == want

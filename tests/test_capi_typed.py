"""The typed C-ABI entry points a cgo binding calls (include/symphony_hip.h "typed entry points"),
exercised two ways on the GPU:

* tests/capi_driver.c: a plain C program compiled with gcc against the header and linked to
  libsymphony_hip.so (prototype drift between header and library breaks its build or its answers);
* ctypes calls of each typed symbol on random batches, bit-exact against the oracle.

The CPU part checks that the driver builds against the header.
"""
import os
import subprocess

import numpy as np
import pytest

from arpc_amd import _native, datagen
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "bin", "capi_driver")


def _build_driver():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests")], check=True)
    return DRIVER


def test_c_driver_builds_against_header():
    assert os.path.exists(_build_driver())


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


@pytest.mark.gpu
def test_c_driver_runs(dev):
    path = DRIVER if os.path.exists(DRIVER) else _build_driver()
    r = subprocess.run([path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks ok" in r.stdout


def _t(a: np.ndarray, dev):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.dtype == np.uint8:
        a = np.concatenate([a, np.zeros(16, np.uint8)])  # readable 16 bytes past the end (ABI rule)
    return torch.from_numpy(a.copy()).to(dev)


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _check(codec, rc, what):
    _native.check(rc, what)
    codec.check()


@pytest.mark.gpu
@pytest.mark.parametrize("schema", ["kv_set_request", "kv_get_request", "kv_get_response", "kv_set_response",
                                    "echo_request"])
def test_typed_entry_points_match_oracle(codec, dev, schema):
    L, ctx = codec._lib, codec._ctx
    s = {"kv_set_request": 1, "kv_get_request": 0, "kv_get_response": 2, "kv_set_response": 3, "echo_request": 4}[schema]
    from arpc_amd import schemas
    sch = schemas.BY_NAME[schema]
    b = datagen.make_batch(schema=schema, n=5000, lens=tuple(("uniform", 0, 90) for _ in range(sch.nvar)), seed=s + 21)
    want, woff = oracle.encode_batch(b.fixed, b.var, 3, 4)
    n = b.n
    cols = [(_t(x, dev), _t(o, dev)) for x, o in b.var]
    fx = [_t(c, dev) for c in b.fixed]
    out = torch.empty(len(want) + 16, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    sh = _stream(dev)
    if schema == "kv_set_request":
        rc = L.sym_encode_kv_set(ctx, cols[0][0].data_ptr(), cols[0][1].data_ptr(), cols[1][0].data_ptr(),
                                 cols[1][1].data_ptr(), n, 3, 4, out.data_ptr(), off.data_ptr(), sh)
    elif schema == "kv_get_request":
        rc = L.sym_encode_kv_get(ctx, cols[0][0].data_ptr(), cols[0][1].data_ptr(), n, 3, 4, out.data_ptr(),
                                 off.data_ptr(), sh)
    elif schema == "echo_request":
        rc = L.sym_encode_echo(ctx, fx[0].data_ptr(), fx[1].data_ptr(), cols[0][0].data_ptr(), cols[0][1].data_ptr(),
                               cols[1][0].data_ptr(), cols[1][1].data_ptr(), n, 3, 4, out.data_ptr(), off.data_ptr(), sh)
    else:
        rc = L.sym_encode_kv_response(ctx, s, cols[0][0].data_ptr(), cols[0][1].data_ptr(), n, 3, 4, out.data_ptr(),
                                      off.data_ptr(), sh)
    _check(codec, rc, "typed encode")
    np.testing.assert_array_equal(out[:len(want)].cpu().numpy(), want)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint64), woff)

    wf, wv, ws = oracle.decode_batch(sch.nfixed, sch.nvar, want, woff)
    cap = max(1, len(want))
    dcols = [(torch.empty(cap, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
             for _ in range(sch.nvar)]
    dfx = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(sch.nfixed)]
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    if schema == "kv_set_request":
        rc = L.sym_decode_kv_set(ctx, out.data_ptr(), off.data_ptr(), n, dcols[0][0].data_ptr(), cap,
                                 dcols[0][1].data_ptr(), dcols[1][0].data_ptr(), cap, dcols[1][1].data_ptr(),
                                 st.data_ptr(), sh)
    elif schema == "kv_get_request":
        rc = L.sym_decode_kv_get(ctx, out.data_ptr(), off.data_ptr(), n, dcols[0][0].data_ptr(), cap,
                                 dcols[0][1].data_ptr(), st.data_ptr(), sh)
    elif schema == "echo_request":
        rc = L.sym_decode_echo(ctx, out.data_ptr(), off.data_ptr(), n, dfx[0].data_ptr(), dfx[1].data_ptr(),
                               dcols[0][0].data_ptr(), cap, dcols[0][1].data_ptr(), dcols[1][0].data_ptr(), cap,
                               dcols[1][1].data_ptr(), st.data_ptr(), sh)
    else:
        rc = L.sym_decode_kv_response(ctx, s, out.data_ptr(), off.data_ptr(), n, dcols[0][0].data_ptr(), cap,
                                      dcols[0][1].data_ptr(), st.data_ptr(), sh)
    _check(codec, rc, "typed decode")
    np.testing.assert_array_equal(st.cpu().numpy(), ws)
    for f in range(sch.nfixed):
        np.testing.assert_array_equal(dfx[f].cpu().numpy(), wf[f])
    for f in range(sch.nvar):
        o = dcols[f][1].cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(o, wv[f][1])
        np.testing.assert_array_equal(dcols[f][0][:int(o[-1])].cpu().numpy(), wv[f][0])


@pytest.mark.gpu
def test_encode_host_small_batch(codec):
    L, ctx = codec._lib, codec._ctx
    n = 3
    kb = np.frombuffer(b"abc", np.uint8).copy()
    ko = np.array([0, 1, 2, 3], np.uint64)
    out = np.zeros(128, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    rc = L.sym_encode_host(ctx, 0, n, None, _native.ptr_array([kb.ctypes.data]), _native.ptr_array([ko.ctypes.data]),
                           1, 1, out.ctypes.data, off.ctypes.data)
    assert rc == 0, _native.last_error()
    assert off.tolist() == [0, 23, 46, 69]
    want, _ = oracle.encode_batch([], [(kb, ko)], 1, 1)
    np.testing.assert_array_equal(out[:69], want)


def _pinned(L, ctx, nbytes, dtype, keep):
    """A numpy view of sym_host_alloc memory (freed by the caller via `keep`)."""
    import ctypes
    p = ctypes.c_void_p()
    assert L.sym_host_alloc(ctx, max(1, nbytes), ctypes.byref(p)) == 0, _native.last_error()
    keep.append(p.value)
    buf = (ctypes.c_uint8 * max(1, nbytes)).from_address(p.value)
    return np.frombuffer(buf, np.uint8)[:nbytes].view(dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("memory", ["pageable", "pinned"])
@pytest.mark.parametrize("schema,lens", [("kv_set_request", (64, ("loguniform", 1, 4096))),
                                         ("echo_request", (("uniform", 0, 300), ("uniform", 0, 600)))])
def test_host_entry_points_many_chunks(codec, memory, schema, lens):
    """sym_encode_host / sym_decode_host over a batch of ~5 chunks (kChunkBytes = 32 MiB, 3 slots:
    every slot reused): outputs of every chunk land in place, bit-exact against the oracle; a
    corrupted record's status and the record after it come back exactly as the oracle decodes them."""
    L, ctx = codec._lib, codec._ctx
    sid = datagen.schemas.BY_NAME[schema].schema_id
    n = 260000 if schema == "kv_set_request" else 420000
    b = datagen.make_batch(schema, n, lens, seed=0x5EEDC0DE)
    want, want_off = oracle.encode_batch(b.fixed, b.var, 3, 4)
    assert int(want_off[-1]) > 4 * (32 << 20)
    keep = []
    try:
        if memory == "pinned":
            def mk(a):
                v = _pinned(L, ctx, a.nbytes, a.dtype, keep)
                v[:] = a
                return v
            fixed = [mk(f) for f in b.fixed]
            var = [(mk(x), mk(o)) for x, o in b.var]
            out = _pinned(L, ctx, int(want_off[-1]), np.uint8, keep)
            off = _pinned(L, ctx, 8 * (n + 1), np.uint64, keep)
        else:
            fixed, var = b.fixed, b.var
            out = np.zeros(int(want_off[-1]), np.uint8)
            off = np.zeros(n + 1, np.uint64)
        rc = L.sym_encode_host(ctx, sid, n, _native.ptr_array([f.ctypes.data for f in fixed]) if fixed else None,
                               _native.ptr_array([x.ctypes.data for x, _ in var]),
                               _native.ptr_array([o.ctypes.data for _, o in var]), 3, 4, out.ctypes.data,
                               off.ctypes.data)
        assert rc == 0, _native.last_error()
        np.testing.assert_array_equal(off, want_off)
        np.testing.assert_array_equal(out, want)

        # decode the stream with two records damaged in different chunks
        data = np.array(want)
        for r in (n // 3, (3 * n) // 4):
            data[int(want_off[r])] = 2  # version byte
        wf, wv, wst = oracle.decode_batch(b.schema.nfixed, b.schema.nvar, data, want_off)
        if memory == "pinned":
            d_in = _pinned(L, ctx, data.nbytes, np.uint8, keep)
            d_in[:] = data
            roff = _pinned(L, ctx, want_off.nbytes, np.uint64, keep)
            roff[:] = want_off
        else:
            d_in, roff = data, want_off
        caps = np.array([int(o[-1]) for _, o in wv], np.uint64)
        dfix = [np.zeros(n, np.int32) for _ in range(b.schema.nfixed)]
        dbytes = [np.zeros(max(1, int(c)), np.uint8) for c in caps]
        doffs = [np.zeros(n + 1, np.uint64) for _ in range(b.schema.nvar)]
        st = np.zeros(n, np.uint8)
        rc = L.sym_decode_host(ctx, sid, n, d_in.ctypes.data, roff.ctypes.data,
                               _native.ptr_array([f.ctypes.data for f in dfix]) if dfix else None,
                               _native.ptr_array([x.ctypes.data for x in dbytes]), caps.ctypes.data,
                               _native.ptr_array([o.ctypes.data for o in doffs]), st.ctypes.data)
        assert rc == 0, _native.last_error()
        np.testing.assert_array_equal(st, wst)
        assert (st != 0).sum() == 2
        for f in range(b.schema.nfixed):
            np.testing.assert_array_equal(dfix[f], wf[f])
        for f in range(b.schema.nvar):
            np.testing.assert_array_equal(doffs[f], wv[f][1])
            np.testing.assert_array_equal(dbytes[f][:int(caps[f])], wv[f][0])
    finally:
        for p in keep:
            L.sym_host_free(ctx, p)

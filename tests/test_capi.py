"""The C-ABI library: it loads, exports every symbol include/symphony_hip.h declares, and the
host-only metadata calls answer without a GPU.  No compute call is made here."""
import ctypes
import os
import re

import pytest

from arpc_amd import _native, schemas

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "symphony_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sym_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_surface():
    syms = declared_symbols()
    for name in ("sym_encode_kv_set", "sym_decode_kv_set", "sym_encode", "sym_decode", "sym_ctx_create",
                 "sym_encode_host", "sym_decode_host", "sym_encode_echo", "sym_decode_echo"):
        assert name in syms


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert set(declared_symbols()) == set(_native.SIGNATURES), "ctypes binding out of sync with the header"


def test_symbols_are_extern_c():
    out = os.popen(f"nm -D --defined-only {_native.LIB_PATH}").read()
    exported = set(re.findall(r"\bT (sym_[a-z0-9_]+)$", out, flags=re.M))
    assert set(declared_symbols()) <= exported


def test_schema_metadata_matches_python():
    L = _native.lib()
    assert L.sym_abi_version() == 2
    for s in schemas.ALL:
        nf, nv = ctypes.c_int(), ctypes.c_int()
        assert L.sym_schema_info(s.schema_id, ctypes.byref(nf), ctypes.byref(nv)) == 0
        assert (nf.value, nv.value) == (s.nfixed, s.nvar)
        assert L.sym_record_overhead(s.schema_id) == s.overhead
        assert L.sym_encoded_size(s.schema_id, 7, 123) == 7 * s.overhead + 123
    assert L.sym_schema_info(99, None, None) == _native.SYM_ERR_INVALID
    assert "unknown schema" in _native.last_error()


def test_overheads_match_reference_sizes():
    # |GetRequest| = 22+K, |SetRequest| = 30+K+V, |EchoRequest| = 38+|U|+|C|
    assert schemas.KV_GET_REQUEST.overhead == 22
    assert schemas.KV_SET_REQUEST.overhead == 30
    assert schemas.KV_GET_RESPONSE.overhead == schemas.KV_SET_RESPONSE.overhead == 22
    assert schemas.ECHO_REQUEST.overhead == 38
    assert schemas.KV_SET_REQUEST.record_size([64, 256]) == 350


def test_null_arguments_rejected_without_gpu():
    L = _native.lib()
    assert L.sym_ctx_create(0, None) == _native.SYM_ERR_INVALID
    assert L.sym_encode(None, 1, 0, None, None, None, 0, 0, None, None, None) == _native.SYM_ERR_INVALID
    assert L.sym_decode(None, 1, 0, None, None, None, None, None, None, None, None) == _native.SYM_ERR_INVALID
    assert L.sym_ctx_destroy(None) == 0


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError, match="not built"):
        _native.lib()

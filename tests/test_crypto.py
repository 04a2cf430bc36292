"""Per-segment AES-256-GCM of Symphony records.

The cipher is Go's crypto/aes + crypto/cipher GCM, absent here; the oracle (oracle/crypto_oracle.c)
restates FIPS 197 / SP 800-38D and is pinned by
  * the published GCM test vectors (McGrew & Viega, "The Galois/Counter Mode of Operation",
    test cases 13-15: the AES-256 ones), and
  * OpenSSL's EVP_aes_256_gcm from the system libcrypto, on random keys, nonces and lengths.
The segment framing follows pkg/transport/encryption.go:82-335, and the batch cases mirror the
reference's own tests (pkg/transport/encryption_test.go:132-420: createSymphonyData sizes, header
preservation, the panic cases, round trips).  GPU tests compare the HIP cipher with the oracle
bit-exactly (both directions, tampered inputs, batch edges, the bench batch).
"""
import ctypes
import ctypes.util
import struct

import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle

PK, VK = oracle.DEFAULT_PUBLIC_KEY, oracle.DEFAULT_PRIVATE_KEY


def create_symphony_data(public_size: int, private_size: int, sid: int = 0, mid: int = 0) -> bytes:
    """encryption_test.go:17-45."""
    off = 13 + public_size
    total = off + (1 + private_size if private_size > 0 else 0)
    d = bytearray(total)
    d[0] = 1
    struct.pack_into("<III", d, 1, off, sid, mid)
    for i in range(13, off):
        d[i] = i % 256
    if private_size > 0:
        d[off] = 1
        for i in range(off + 1, total):
            d[i] = (i * 2) % 256
    return bytes(d)


def batch(recs):
    off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


def nonces_for(n: int, seed: int = 0) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, (max(n, 1), 24), dtype=np.uint8)[:n]


# ------------------------------------------------------------------ oracle pinning (CPU)
def test_oracle_published_vectors():
    assert oracle.gcm_seal(bytes(32), bytes(12), b"")[1].hex() == "530f8afbc74536b9a963b4f1c4cb738b"  # TC13
    c, t = oracle.gcm_seal(bytes(32), bytes(12), bytes(16))  # TC14
    assert c.hex() == "cea7403d4d606b6e074ec5d3baf39d18" and t.hex() == "d0d1c8a799996bf0265b98b5d48ab919"
    k = bytes.fromhex("feffe9928665731c6d6a8f9467308308" * 2)  # TC15
    p = bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
                      "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255")
    c, t = oracle.gcm_seal(k, bytes.fromhex("cafebabefacedbaddecaf888"), p)
    assert c.hex() == ("522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa"
                       "8cb08e48590dbb3da7b08b1056828838c5f61e6393ba7a0abcc9f662898015ad")
    assert t.hex() == "b094dac5d93471bdec1a502270e3cc6c"


def _openssl_seal():
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("no system libcrypto")
    L = ctypes.CDLL(name)
    vp, i, cp = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
    L.EVP_CIPHER_CTX_new.restype = vp
    L.EVP_aes_256_gcm.restype = vp
    L.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, cp, cp]
    L.EVP_EncryptUpdate.argtypes = [vp, cp, ctypes.POINTER(i), cp, i]
    L.EVP_EncryptFinal_ex.argtypes = [vp, cp, ctypes.POINTER(i)]
    L.EVP_CIPHER_CTX_ctrl.argtypes = [vp, i, i, vp]
    L.EVP_CIPHER_CTX_free.argtypes = [vp]

    def seal(key, nonce, pt):
        ctx = L.EVP_CIPHER_CTX_new()
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_aes_256_gcm(), None, key, nonce) == 1  # 12-byte IV is the default
        out = ctypes.create_string_buffer(len(pt) + 16)
        n = i(0)
        if pt:
            assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
        m = i(0)
        assert L.EVP_EncryptFinal_ex(ctx, ctypes.cast(ctypes.addressof(out) + n.value, cp), ctypes.byref(m)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag) == 1  # EVP_CTRL_GCM_GET_TAG
        L.EVP_CIPHER_CTX_free(ctx)
        return out.raw[:n.value + m.value], tag.raw
    return seal


def test_oracle_matches_openssl():
    seal = _openssl_seal()
    rng = np.random.default_rng(11)
    for length in list(range(0, 40)) + [63, 64, 65, 255, 256, 1000, 1023, 1024, 1025, 4100]:
        key, nonce = rng.bytes(32), rng.bytes(12)
        pt = rng.bytes(length)
        assert oracle.gcm_seal(key, nonce, pt) == seal(key, nonce, pt), length


def _split(out, off, i):
    return out[int(off[i]):int(off[i + 1])].tobytes()


def test_oracle_segment_framing():
    """encryption_test.go:132-231 (sizes, offsetToPrivate, header) with explicit nonces."""
    recs = [create_symphony_data(p, 0) for p in (0, 10, 100, 1000, 10000)] + \
           [create_symphony_data(p, v) for p, v in ((10, 10), (100, 100), (1000, 1000), (1000, 10), (10, 1000))] + \
           [create_symphony_data(100, 50, 12345, 67890)]
    data, off = batch(recs)
    nonces = nonces_for(len(recs), 1)
    out, ooff, st = oracle.encrypt_batch(data, off, nonces)
    assert (st == oracle.CRYPT_OK).all()
    for i, r in enumerate(recs):
        e = _split(out, ooff, i)
        pub_only = struct.unpack_from("<I", r, 1)[0] == len(r)
        assert len(e) == len(r) + (28 if pub_only else 56)
        o = struct.unpack_from("<I", e, 1)[0]
        assert (o == len(e)) if pub_only else (o < len(e))
        assert e[0] == r[0] and e[5:13] == r[5:13] and e[13:25] == nonces[i, :12].tobytes()
        np_ = struct.unpack_from("<I", r, 1)[0] - 13
        c, t = oracle.gcm_seal(PK, nonces[i, :12].tobytes(), r[13:13 + np_])
        assert e[25:o] == c + t
        if not pub_only:
            c, t = oracle.gcm_seal(VK, nonces[i, 12:].tobytes(), r[13 + np_:])
            assert e[o:] == nonces[i, 12:].tobytes() + c + t
    assert struct.unpack_from("<II", _split(out, ooff, len(recs) - 1), 5) == (12345, 67890)
    dec, doff, dst = oracle.decrypt_batch(out, ooff)
    assert (dst == oracle.CRYPT_OK).all()
    assert [_split(dec, doff, i) for i in range(len(recs))] == recs  # RoundTrip


def test_oracle_errors():
    short = [b"", bytes(10), bytes(12)]
    bad = bytearray(20)
    struct.pack_into("<I", bad, 1, 5)
    bad2 = bytearray(20)
    struct.pack_into("<I", bad2, 1, 100)
    data, off = batch(short + [bytes(bad), bytes(bad2), create_symphony_data(3, 4)])
    _, ooff, st = oracle.encrypt_batch(data, off, nonces_for(6))
    assert list(st) == [1, 1, 1, 2, 2, 0] and list(np.diff(ooff)) == [0, 0, 0, 0, 0, 13 + 3 + 1 + 4 + 56]
    # decrypt: tampered public / private bytes, bad version, private shorter than nonce + tag
    good = [create_symphony_data(20, 30), create_symphony_data(0, 5), create_symphony_data(7, 0)]
    gd, goff = batch(good)
    enc, eoff, _ = oracle.encrypt_batch(gd, goff, nonces_for(3, 2))
    e = [bytearray(_split(enc, eoff, i)) for i in range(3)]
    t_pub, t_priv, t_tag = bytearray(e[0]), bytearray(e[0]), bytearray(e[0])
    t_pub[30] ^= 1
    t_priv[-20] ^= 0x80
    t_tag[-1] ^= 1
    nover = create_symphony_data(4, 6)
    nover = nover[:17] + b"\x02" + nover[18:]  # private version byte 2
    nv, nvo = batch([nover])
    nenc, _, _ = oracle.encrypt_batch(nv, nvo, nonces_for(1, 3))
    cut = bytearray(e[1])
    o1 = struct.unpack_from("<I", cut, 1)[0]
    cut = cut[:o1 + 27]
    recs = [bytes(x) for x in (e[0], t_pub, t_priv, t_tag, nenc.tobytes(), cut, e[2], bytes(50))]
    dd, doff = batch(recs)
    dec, dooff, dst = oracle.decrypt_batch(dd, doff)
    assert list(dst) == [0, oracle.CRYPT_AUTH_PUBLIC, oracle.CRYPT_AUTH_PRIVATE, oracle.CRYPT_AUTH_PRIVATE,
                         oracle.CRYPT_BAD_VERSION, oracle.CRYPT_AUTH_PRIVATE, 0, oracle.CRYPT_BAD_OFFSET]
    assert _split(dec, dooff, 0) == good[0] and _split(dec, dooff, 6) == good[2]
    assert _split(dec, dooff, 1) == bytes(len(good[0]))  # failed: zero-filled, same size
    assert dooff[6] - dooff[5] == 0 and dooff[8] - dooff[7] == 0


# ------------------------------------------------------------------ HIP cipher (GPU)
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


def _dev(arr, dev, misalign=0):
    import torch
    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
    buf = torch.full((raw.size + misalign + 32,), 0xA5, dtype=torch.uint8, device=dev)
    if raw.size:
        buf[misalign:misalign + raw.size].copy_(torch.from_numpy(raw.copy()))
    v = buf[misalign:misalign + raw.size]
    return v.view(torch.int64) if arr.dtype in (np.uint64, np.int64) else v


def _gpu_encrypt_vs_oracle(codec, dev, data, off, nonces, misalign=0, keys=(PK, VK)):
    want = oracle.encrypt_batch(data, off, nonces, *keys)
    r = codec.encrypt(_dev(data, dev, misalign), _dev(off, dev), _dev(nonces, dev), *keys)
    codec.check()
    np.testing.assert_array_equal(r.status.cpu().numpy(), want[2], err_msg="encrypt status")
    np.testing.assert_array_equal(r.offsets.cpu().numpy().view(np.uint64), want[1], err_msg="encrypt offsets")
    np.testing.assert_array_equal(r.data[:int(want[1][-1])].cpu().numpy(), want[0], err_msg="encrypt bytes")
    return want


def _gpu_decrypt_vs_oracle(codec, dev, data, off, misalign=0, keys=(PK, VK)):
    want = oracle.decrypt_batch(data, off, *keys)
    r = codec.decrypt(_dev(data, dev, misalign), _dev(off, dev), *keys)
    codec.check()
    np.testing.assert_array_equal(r.status.cpu().numpy(), want[2], err_msg="decrypt status")
    np.testing.assert_array_equal(r.offsets.cpu().numpy().view(np.uint64), want[1], err_msg="decrypt offsets")
    np.testing.assert_array_equal(r.data[:int(want[1][-1])].cpu().numpy(), want[0], err_msg="decrypt bytes")
    return want


@pytest.mark.gpu
def test_crypto_reference_cases_gpu(gcodec, gdev):
    recs = [create_symphony_data(p, 0) for p in (0, 10, 100, 1000, 10000)] + \
           [create_symphony_data(p, v) for p, v in ((10, 10), (100, 100), (1000, 1000), (1000, 10), (10, 1000))] + \
           [create_symphony_data(100, 50, 12345, 67890), b"", bytes(12), bytes(20)]
    data, off = batch(recs)
    enc = _gpu_encrypt_vs_oracle(gcodec, gdev, data, off, nonces_for(len(recs), 4), misalign=3)
    _gpu_decrypt_vs_oracle(gcodec, gdev, enc[0], enc[1], misalign=5)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_crypto_random_lengths_gpu(gcodec, gdev, seed):
    rng = np.random.default_rng(seed)
    recs = [create_symphony_data(int(rng.integers(0, 300)), int(rng.choice([0, rng.integers(0, 3000)])))
            for _ in range(700)]
    keys = (rng.bytes(32), rng.bytes(32))
    data, off = batch(recs)
    enc = _gpu_encrypt_vs_oracle(gcodec, gdev, data, off, nonces_for(len(recs), seed), misalign=seed, keys=keys)
    # tamper a few encrypted records (ciphertext, tags, nonces, offsets) before decrypting
    e = [bytearray(_split(enc[0], enc[1], i)) for i in range(len(recs))]
    for i in rng.choice(len(e), 60, replace=False):
        j = int(rng.integers(0, len(e[i])))
        e[i][j] ^= 1 << int(rng.integers(0, 8))
    dd, doff = batch([bytes(x) for x in e])
    dec = _gpu_decrypt_vs_oracle(gcodec, gdev, dd, doff, misalign=seed + 1, keys=keys)
    assert (dec[2] == 0).sum() >= 600 and (dec[2] != 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 257])
def test_crypto_edge_counts_gpu(gcodec, gdev, n):
    recs = [create_symphony_data(i % 37, (i * 7) % 90) for i in range(n)]
    data, off = batch(recs) if n else (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    enc = _gpu_encrypt_vs_oracle(gcodec, gdev, data, off, nonces_for(n, n))
    _gpu_decrypt_vs_oracle(gcodec, gdev, enc[0], enc[1])


@pytest.mark.gpu
def test_crypto_encoded_batch_gpu(gcodec, gdev):
    """Config-2 records (what the transport encrypts before packetizing), round trip."""
    b = datagen.make_batch(**dict(datagen.CONFIG2, n=20000))
    stream, off = oracle.encode_batch(b.fixed, b.var, 1, 2)
    enc = _gpu_encrypt_vs_oracle(gcodec, gdev, stream, off, nonces_for(20000, 9))
    dec = _gpu_decrypt_vs_oracle(gcodec, gdev, enc[0], enc[1])
    assert dec[0].tobytes() == stream.tobytes()

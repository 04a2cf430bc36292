"""The kv benchmark's trace as a workload (config 3's secondary variant, the config-2
Get/Set stream): the size fixture derived from benchmark/meta-kv-trace/trace_large.req
(tests/golden/make_trace_sizes.py), and GPU round trips of the trace-sized batches against the C
restatement."""
import json
import os

import numpy as np
import pytest
import torch

from arpc_amd import datagen
from oracle import oracle

FIX = os.path.join(os.path.dirname(__file__), "golden", "trace_large_sizes.json")


def test_trace_fixture_matches_survey_counts():
    t = json.load(open(FIX))
    assert t["requests"] == 25125 and len(t["ops"]) == 25125  # 9,267 SET / 25,125
    assert t["sets"] == 9267 == t["ops"].count("S")
    assert min(t["key_size"]) == 17 and max(t["key_size"]) == 166  # "key sizes 17-166"
    assert abs(datagen.TRACE_SET_FRACTION - t["sets"] / t["requests"]) < 1e-12
    # the first requests of trace_large.req
    assert t["ops"][:5] == "SGGGS" and t["key_size"][:3] == [78, 78, 85] and t["value_size"][0] == 1521


def test_trace_configs_follow_the_fixture():
    s = datagen.trace_sizes()
    c3 = datagen.config3_trace(5000)
    b = datagen.make_batch(**c3)
    kl, vl = np.diff(b.var[0][1]), np.diff(b.var[1][1])
    sets = np.flatnonzero(s["set"])
    assert np.array_equal(kl[:len(sets)], s["key"][sets][:5000])
    assert np.array_equal(vl[:len(sets)], np.clip(s["value"][sets], 16, 4096)[:5000])
    m = datagen.make_mixed_batch(**datagen.config2_trace_mixed(30000))
    assert np.array_equal(m.type[:25125], s["set"].astype(np.uint8)) and np.array_equal(m.type[25125:], m.type[:30000 - 25125])
    vm = np.diff(m.val[1])
    assert (vm[m.type == 0] == 0).all() and (vm[m.type != 0] >= 16).all() and (vm <= 4096).all()
    assert np.array_equal(np.diff(m.key[1])[:25125], s["key"])


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def codec(dev):
    from arpc_amd.codec import Codec
    c = Codec(dev)
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_config3_trace_roundtrip(codec, dev):
    """Config 3 with the trace's SET sizes at 2^20 records (3.3 GB stream): offsets from the sizes, a
    slice byte-equal to the oracle, the decode equal to the input."""
    from arpc_amd.codec import to_device
    b = datagen.make_batch(**datagen.config3_trace())
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    codec.check()
    n = b.n
    size = 30 + np.diff(b.var[0][1]).astype(np.int64) + np.diff(b.var[1][1]).astype(np.int64)
    off = enc.offsets.cpu().numpy()
    assert off[0] == 0 and np.array_equal(np.diff(off), size)
    lo, hi = n // 2, n // 2 + 500
    sub = [(c[o[lo]:o[hi]], o[lo:hi + 1] - o[lo]) for c, o in b.var]
    want, _ = oracle.encode_batch([], sub)
    np.testing.assert_array_equal(enc.data[int(off[lo]):int(off[hi])].cpu().numpy(), want)
    dec = codec.decode(b.schema, enc.data, enc.offsets)
    codec.check()
    assert int(dec.status.sum().item()) == 0
    for f, (col, o) in enumerate(var):
        assert torch.equal(dec.var[f][1], o) and torch.equal(dec.var[f][0][:col.numel()], col)


@pytest.mark.gpu
def test_gpu_trace_mixed_roundtrip(codec, dev):
    """The trace's Get/Set sequence and sizes at 2^20 requests: offsets from the sizes, a slice
    byte-equal to the oracle, the decode equal to the input."""
    m = datagen.make_mixed_batch(**datagen.config2_trace_mixed())
    t = torch.from_numpy(m.type).to(dev)
    key = (torch.from_numpy(m.key[0]).to(dev), torch.from_numpy(m.key[1].view(np.int64)).to(dev))
    val = (torch.from_numpy(m.val[0]).to(dev), torch.from_numpy(m.val[1].view(np.int64)).to(dev))
    enc = codec.encode_kv_mixed(t, key, val, 1, 1, 2, out_bytes=m.encoded_size())
    dec = codec.decode_kv_mixed(enc.data, enc.offsets, t, caps=[m.key[0].size, max(1, m.val[0].size)])
    codec.check()
    n = m.n
    size = 22 + np.diff(m.key[1]).astype(np.int64) + (m.type != 0) * (8 + np.diff(m.val[1]).astype(np.int64))
    off = enc.offsets.cpu().numpy()
    assert off[0] == 0 and np.array_equal(np.diff(off), size)
    assert int(dec.status.sum().item()) == 0
    assert torch.equal(dec.var[0][1], key[1]) and torch.equal(dec.var[0][0][:key[0].numel()], key[0])
    assert torch.equal(dec.var[1][1], val[1]) and torch.equal(dec.var[1][0][:val[0].numel()], val[0])
    lo, hi = n // 3, n // 3 + 2000
    sub_k = (m.key[0][m.key[1][lo]:m.key[1][hi]], m.key[1][lo:hi + 1] - m.key[1][lo])
    sub_v = (m.val[0][m.val[1][lo]:m.val[1][hi]], m.val[1][lo:hi + 1] - m.val[1][lo])
    want, _ = oracle.encode_kv_mixed(m.type[lo:hi], sub_k, sub_v, 1, 1, 2)
    np.testing.assert_array_equal(enc.data[int(off[lo]):int(off[hi])].cpu().numpy(), want)

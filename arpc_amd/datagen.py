"""Seeded synthetic record batches for tests and bench.py.

Bytes are splitmix64 output (uniform 0-255): Symphony stores arbitrary bytes with no
UTF-8 check (kv.syn.go:725), so random bytes exercise the same path as text.

Field f of a batch draws its bytes from splitmix64 seeded with `seed + 0x100000000*(f+1)`
and its lengths (when variable) from the stream seeded with `seed + 0x10000*(f+1)`.
Config seeds: 0x5EED0001 (config 2, K=64/V=256), 0x5EED0002 (config 3, log-uniform
V in [16, 4096]), 0x5EED0003+g (config 4 shard g).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np

from . import schemas

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int) -> np.ndarray:
    """`count` outputs of splitmix64 started at `seed` (state advances by GAMMA before each output)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (np.arange(1, count + 1, dtype=np.uint64) * GAMMA)
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def random_bytes(seed: int, nbytes: int) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


def lengths(spec, n: int, seed: int) -> np.ndarray:
    """spec: int (every record), ("uniform", lo, hi) inclusive, ("loguniform", lo, hi) = floor(exp(U(ln lo, ln(hi+1)))),
    or an array of per-record lengths (cycled to n)."""
    if isinstance(spec, (int, np.integer)):
        return np.full(n, int(spec), dtype=np.uint64)
    if isinstance(spec, np.ndarray):
        return np.resize(spec.astype(np.uint64), n)
    kind, lo, hi = spec
    u = (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
    if kind == "uniform":
        return np.minimum(lo + np.floor(u * (hi - lo + 1)), hi).astype(np.uint64)
    if kind == "loguniform":
        v = np.floor(np.exp(np.log(lo) + u * (np.log(hi + 1) - np.log(lo))))
        return np.clip(v, lo, hi).astype(np.uint64)
    raise ValueError(spec)


@dataclass
class Batch:
    schema: schemas.Schema
    fixed: list = field(default_factory=list)  # int32 [n] per fixed field
    var: list = field(default_factory=list)    # (u8 bytes, u64 offs[n+1]) per var field

    @property
    def n(self) -> int:
        return len(self.var[0][1]) - 1 if self.var else len(self.fixed[0])

    def encoded_size(self) -> int:
        return self.n * self.schema.overhead + sum(int(o[-1] - o[0]) for _, o in self.var)

    def payload_bytes(self) -> int:
        return sum(int(o[-1] - o[0]) for _, o in self.var) + 4 * self.n * self.schema.nfixed


def make_batch(schema: str, n: int, lens: tuple, seed: int, **_ignored) -> Batch:
    s = schemas.BY_NAME[schema]
    fixed = [splitmix64(seed + 0x1000 * (f + 1), n).astype(np.uint32).view(np.int32) for f in range(s.nfixed)]
    var = []
    for f in range(s.nvar):
        ln = lengths(lens[f], n, seed + 0x10000 * (f + 1))
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(ln, out=offs[1:])
        var.append((random_bytes(seed + 0x100000000 * (f + 1), int(offs[-1])), offs))
    return Batch(s, fixed, var)


def from_records(schema: str, records) -> Batch:
    """records: iterable of (fixed tuple, var tuple of bytes)."""
    s = schemas.BY_NAME[schema]
    records = list(records)
    fixed = [np.array([r[0][f] for r in records], dtype=np.int32) for f in range(s.nfixed)]
    var = []
    for f in range(s.nvar):
        vals = [bytes(r[1][f]) for r in records]
        offs = np.zeros(len(vals) + 1, dtype=np.uint64)
        np.cumsum([len(v) for v in vals], out=offs[1:])
        var.append((np.frombuffer(b"".join(vals), dtype=np.uint8).copy(), offs))
    return Batch(s, fixed, var)


# Configs of BASELINE.json (record counts as there) and small golden corpora.
CONFIG2 = dict(schema="kv_set_request", n=1 << 20, lens=(64, 256), seed=0x5EED0001)
CONFIG3 = dict(schema="kv_set_request", n=1 << 20, lens=(64, ("loguniform", 16, 4096)), seed=0x5EED0002)


# BASELINE config 2's Get/Set mix: the SET share of benchmark/meta-kv-trace/trace_large.req
# (9,267 SET of 25,125 requests, 36.9 %).
TRACE_SET_FRACTION = 9267 / 25125
CONFIG2_MIXED = dict(n=1 << 20, key=64, value=256, set_fraction=TRACE_SET_FRACTION, seed=0x5EED0001)


@dataclass
class MixedBatch:
    type: np.ndarray  # u8 [n]: 0 GetRequest, 1 SetRequest
    key: tuple        # (u8 bytes, u64 offs [n+1])
    val: tuple        # (u8 bytes, u64 offs [n+1]); empty slices for GetRequests

    @property
    def n(self) -> int:
        return len(self.type)

    def encoded_size(self) -> int:
        kl = int(self.key[1][-1] - self.key[1][0])
        vl = int(self.val[1][-1] - self.val[1][0])
        return 22 * self.n + 8 * int((self.type != 0).sum()) + kl + vl


def make_mixed_batch(n: int, key, value, set_fraction: float, seed: int, types=None, **_ignored) -> MixedBatch:
    """A kv request stream: record i is a SetRequest with probability `set_fraction` (splitmix64
    stream seed + 0x7000), else a GetRequest (or `types`, per record, cycled to n); key lengths from
    `key`, value lengths from `value` for SetRequests (GetRequests carry no value)."""
    if types is not None:
        rtype = np.resize(np.asarray(types, dtype=np.uint8), n)
    else:
        u = (splitmix64(seed + 0x7000, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))
        rtype = (u < set_fraction).astype(np.uint8)
    cols = []
    for f, spec in enumerate((key, value)):
        ln = lengths(spec, n, seed + 0x10000 * (f + 1))
        if f == 1:
            ln = ln * rtype.astype(np.uint64)
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(ln, out=offs[1:])
        cols.append((random_bytes(seed + 0x100000000 * (f + 1), int(offs[-1])), offs))
    return MixedBatch(rtype, cols[0], cols[1])


# The kv benchmark's trace (benchmark/meta-kv-trace/trace_large.req) as a size list
# (tests/golden/trace_large_sizes.json, made by tests/golden/make_trace_sizes.py): the operation
# sequence, key sizes 17-166, value sizes.
TRACE_SIZES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                           "trace_large_sizes.json")


def trace_sizes() -> dict:
    with open(TRACE_SIZES) as f:
        t = json.load(f)
    ops = np.frombuffer(t["ops"].encode(), dtype=np.uint8) == ord("S")
    return dict(set=ops, key=np.array(t["key_size"], dtype=np.uint64), value=np.array(t["value_size"], dtype=np.uint64))


def config3_trace(n: int = 1 << 20) -> dict:
    """SURVEY 8d config 3, secondary variant: SetRequests with the trace's SET key sizes and its SET
    value sizes clipped to [16, 4096], in trace order, cycled to n; bytes from the config-3 seed."""
    t = trace_sizes()
    k = t["key"][t["set"]]
    v = np.clip(t["value"][t["set"]], 16, 4096)
    return dict(schema="kv_set_request", n=n, lens=(k, v), seed=0x5EED0002)


def config2_trace_mixed(n: int = 1 << 20) -> dict:
    """The Get/Set request stream as the benchmark replays it: the trace's operation sequence, key
    sizes and (SET) value sizes clipped to [16, 4096], cycled to n records (for make_mixed_batch)."""
    t = trace_sizes()
    return dict(n=n, key=t["key"], value=np.clip(t["value"], 16, 4096), set_fraction=TRACE_SET_FRACTION,
                seed=0x5EED0001, types=t["set"].astype(np.uint8))


def config4_shard(g: int, records_per_gpu: int = 1 << 23) -> dict:
    return dict(schema="kv_set_request", n=records_per_gpu, lens=(64, 256), seed=0x5EED0003 + g)


CORPORA = {
    "set_64_256": dict(schema="kv_set_request", n=4096, lens=(64, 256), seed=0x5EED0001),
    "set_mixed": dict(schema="kv_set_request", n=2048, lens=(64, ("loguniform", 16, 4096)), seed=0x5EED0002),
    "set_tiny": dict(schema="kv_set_request", n=5000, lens=(("uniform", 0, 7), ("uniform", 0, 20)), seed=7),
    "set_ids": dict(schema="kv_set_request", n=1000, lens=(64, 256), seed=11, service_id=1, method_id=2),
    "get_64": dict(schema="kv_get_request", n=4096, lens=(64,), seed=0x5EED0004),
    "get_response_mixed": dict(schema="kv_get_response", n=3000, lens=(("loguniform", 1, 2048),), seed=5),
    "set_response_256": dict(schema="kv_set_response", n=3000, lens=(256,), seed=6),
    "echo_small": dict(schema="echo_request", n=2048, lens=(("uniform", 0, 32), ("uniform", 0, 200)), seed=13),
}


# ------------------------------------------------------------ element-schema records
# kv-store-symphony-element's {Get,Set}Request: public Score (int32, table 13) and Username (string,
# table 17), private Key [and Value].  Built here, vectorized, as synthetic INPUT for the field
# getters and the firewall (bench.py and tests); layout of kv.syn.go:1041-1124 (SetRequest) and
# :128-202 (GetRequest).  tests/test_raw_fields.py checks it against the C oracle's restatement.
ELEMENT_FW = dict(n=1 << 20, lens=(16, 64, 256), seed=0x5EED0005)  # Username 16, Key 64, Value 256


@dataclass
class ElementBatch:
    score: np.ndarray   # int32 [n]
    strings: list       # (bytes, offs[n+1]) for Username, Key[, Value]
    data: np.ndarray    # uint8 stream
    rec_off: np.ndarray  # uint64 [n+1]


def _put_u32(out: np.ndarray, pos: np.ndarray, v: np.ndarray) -> None:
    v = v.astype(np.uint64)
    for b in range(4):
        out[pos + b] = ((v >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)


def _scatter(out: np.ndarray, dst: np.ndarray, col: tuple) -> None:
    b, o = col
    lens = np.diff(o).astype(np.int64)
    n = len(lens)
    uniform = n > 0 and b.size > 0 and bool((lens == lens[0]).all()) and (n == 1 or bool((np.diff(dst) == dst[1] - dst[0]).all()))
    if uniform:  # equal lengths at equal strides: one strided 2-D copy
        L, step = int(lens[0]), int(dst[1] - dst[0]) if n > 1 else 0
        if n == 1 or step >= L:
            view = np.lib.stride_tricks.as_strided(out[int(dst[0]):], shape=(n, L), strides=(step, 1))
            view[...] = b[int(o[0]):int(o[-1])].reshape(n, L)
            return
    if b.size:
        out[np.arange(int(o[-1] - o[0]), dtype=np.int64) + np.repeat(dst.astype(np.int64) - (o[:-1] - o[0]).astype(np.int64), lens)] = b[int(o[0]):int(o[-1])]


def element_records(score: np.ndarray, strings: list) -> tuple[np.ndarray, np.ndarray]:
    """Marshal element-schema records: strings = [Username, Key] or [Username, Key, Value] columns."""
    n, npriv = len(score), len(strings) - 1
    ln = [np.diff(o).astype(np.uint64) for _, o in strings]
    pub = np.uint64(25) + ln[0]                            # publicSegmentSize
    size = pub + np.uint64(1 + 4 * npriv) + sum(np.uint64(4) + x for x in ln[1:])
    rec_off = np.zeros(n + 1, np.uint64)
    np.cumsum(size, out=rec_off[1:])
    out = np.zeros(int(rec_off[-1]), np.uint8)
    s = rec_off[:-1].astype(np.int64)
    out[s] = 1
    _put_u32(out, s + 1, pub)
    _put_u32(out, s + 13, score.view(np.uint32))
    _put_u32(out, s + 17, np.full(n, 21, np.uint64))
    _put_u32(out, s + 21, ln[0])
    _scatter(out, s + 25, strings[0])
    ps = s + pub.astype(np.int64)
    out[ps] = 1
    pay = np.int64(1 + 4 * npriv)                          # payload start, relative to the private segment
    rel = np.full(n, pay, np.int64)
    for k in range(npriv):
        _put_u32(out, ps + 1 + 4 * k, rel.astype(np.uint64))
        _put_u32(out, ps + rel, ln[k + 1])
        _scatter(out, ps + rel + 4, strings[k + 1])
        rel = rel + 4 + ln[k + 1].astype(np.int64)
    return out, rec_off


def make_element_batch(n: int, lens: tuple, seed: int, score_range=(0, 100)) -> ElementBatch:
    """Scores uniform in [lo, hi) (firewall thresholds inside that range drop a known fraction)."""
    lo, hi = score_range
    score = (lo + (splitmix64(seed + 0x1000, n) % np.uint64(hi - lo)).astype(np.int64)).astype(np.int32)
    strings = []
    for f, spec in enumerate(lens):
        ln = lengths(spec, n, seed + 0x10000 * (f + 1))
        offs = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(ln, out=offs[1:])
        strings.append((random_bytes(seed + 0x100000000 * (f + 1), int(offs[-1])), offs))
    data, rec_off = element_records(score, strings)
    return ElementBatch(score, strings, data, rec_off)


# ---- online-boutique messages (benchmark/serialization/online-boutique/proto/onlineboutique.proto):
# synthetic PlaceOrderResponse batches as column trees for arpc_amd.flat (numpy, host side).
# A tree node is: a numpy array (scalar column), (bytes, offsets) (string), ("list", bytes,
# item_off, rec) (repeated string), or ("msg", [child nodes], rec) (message / repeated message).
def _strings(rng, n: int, lo: int, hi: int):
    ln = rng.integers(lo, hi + 1, size=n, dtype=np.int64)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(ln, out=off[1:])
    return rng.integers(32, 127, size=int(off[-1]), dtype=np.uint8), off


def _present(n: int):
    return np.arange(n + 1, dtype=np.int64)


def _money(rng, n: int):
    return ("msg", [_strings(rng, n, 3, 3), rng.integers(0, 10_000, size=n, dtype=np.int64),
                    rng.integers(0, 999_999_999, size=n, dtype=np.int32)], _present(n))


def ob_place_order(n: int, seed: int = 0x5EED0B00, items=(1, 5)) -> tuple:
    """n PlaceOrderResponse{OrderResult{order id, tracking id, Money, Address, 1..5 OrderItem{CartItem,
    Money}}} as a column tree (see above); the message sizes are those of the demo's checkout."""
    rng = np.random.default_rng(seed)
    cnt = rng.integers(items[0], items[1] + 1, size=n, dtype=np.int64)
    rec_items = np.zeros(n + 1, np.int64)
    np.cumsum(cnt, out=rec_items[1:])
    m = int(rec_items[-1])
    cart = ("msg", [_strings(rng, m, 10, 10), rng.integers(1, 10, size=m, dtype=np.int32)], _present(m))
    order_item = ("msg", [cart, _money(rng, m)], rec_items)
    address = ("msg", [_strings(rng, n, 12, 30), _strings(rng, n, 5, 15), _strings(rng, n, 2, 2),
                       _strings(rng, n, 6, 20), rng.integers(10000, 99999, size=n, dtype=np.int32)], _present(n))
    order = ("msg", [_strings(rng, n, 36, 36), _strings(rng, n, 18, 18), _money(rng, n), address, order_item],
             _present(n))
    return ("msg", [order], None)

"""Send-side packetization: FragmentPackets + DataPacket framing.

CPU tests pin the oracle (oracle/fragment_oracle.c) with known answers derived by hand from
pkg/transport/symphony_fragmentation.go:23-125, pkg/transport/transport.go:146-201 and
pkg/packet/builtin_packets.go:59-114 (the reference has no test of the production fragmenter:
SURVEY.md 4).  GPU tests compare the HIP packetizer with the oracle bit-exactly.
"""
import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle

MTU = 1400 - 31  # effectiveMTU, transport.go:147-148


def record(length: int, off2p: int, seed: int = 0) -> bytes:
    rng = np.random.default_rng(seed)
    r = bytearray(rng.integers(0, 256, length, dtype=np.uint8).tobytes())
    if length >= 5:
        r[1:5] = off2p.to_bytes(4, "little")
    return bytes(r)


def batch(recs):
    off = np.zeros(len(recs) + 1, np.uint64)
    np.cumsum([len(r) for r in recs], out=off[1:])
    return np.frombuffer(b"".join(recs), np.uint8).copy(), off


def put(arr: np.ndarray, dev, misalign: int = 0):
    """Copy arr to the GPU at byte offset `misalign` inside a guarded allocation."""
    import torch
    raw = np.ascontiguousarray(arr).view(np.uint8)
    buf = torch.full((raw.size + misalign + 32,), 0xA5, dtype=torch.uint8, device=dev)
    if raw.size:
        buf[misalign:misalign + raw.size].copy_(torch.from_numpy(raw.copy()))
    view = buf[misalign:misalign + raw.size]
    return buf, view.view(torch.int64) if arr.dtype in (np.uint64, np.int64) else view


def frag_sizes(dg_off, wire, first, i):
    return [int(dg_off[j + 1] - dg_off[j]) - 31 for j in range(int(first[i]), int(first[i + 1]))]


# ------------------------------------------------------------------ oracle pinning (CPU)
@pytest.mark.parametrize("length,off2p,sizes", [
    (350, 13, [350]),                       # len <= mtu: one packet (:28-30)
    (MTU, 13, [MTU]),
    (MTU + 1, 13, [1369, 1]),               # meet 13 + head 1357 = 1370 > mtu: Case B, no full packets
    (3000, 13, [262, 1369, 1369]),          # meet 13 + head 249
    (5000, 3000, [1369, 1369, 893, 1369]),  # two full public packets, meet 262 + head 631
    (3400, 1300, [1369, 662, 1369]),        # meeting overflow (Case B, :84-101)
    (2738, 0, [0, 1369, 1369]),             # off2p 0, private a multiple of mtu: an empty packet
    (2000, 2000, [1369, 631]),              # no private data (:102-107)
    (2000, 1369, [1369, 631]),              # public exactly mtu: kept as the meeting remainder
])
def test_oracle_fragment_sizes(length, off2p, sizes):
    data, off = batch([record(length, off2p)])
    wire, dg_off, first, wire_off, status = oracle.fragment_batch(data, off, np.array([5], np.uint64))
    assert status[0] == oracle.FRAG_OK
    assert frag_sizes(dg_off, wire, first, 0) == sizes
    payload = b"".join(wire[int(dg_off[j]) + 31:int(dg_off[j + 1])].tobytes() for j in range(len(sizes)))
    assert payload == data.tobytes()  # fragments are consecutive slices of the record
    assert int(wire_off[1]) == length + 31 * len(sizes) == len(wire)


def test_oracle_header_bytes():
    data, off = batch([record(3000, 13, seed=1)])
    wire, dg_off, *_ = oracle.fragment_batch(data, off, np.array([0x0102030405060708], np.uint64), packet_type=2,
                                             dst=(bytes([10, 0, 0, 7]), 443), src=(bytes([192, 168, 1, 2]), 51000))
    h = wire[int(dg_off[1]):int(dg_off[1]) + 31].tobytes()
    want = (bytes([2]) + (0x0102030405060708).to_bytes(8, "little") + (3).to_bytes(2, "little")
            + (1).to_bytes(2, "little") + b"\x00\x00" + bytes([10, 0, 0, 7]) + (443).to_bytes(2, "little")
            + bytes([192, 168, 1, 2]) + (51000).to_bytes(2, "little") + (1369).to_bytes(4, "little"))
    assert h == want


def test_oracle_errors():
    data, off = batch([record(3000, 3001), record(100, 13), record(4, 0)])
    wire, dg_off, first, wire_off, status = oracle.fragment_batch(data, off, np.arange(3, dtype=np.uint64),
                                                                  max_udp_payload=34)
    # M = 3: 3000 > 3 with off2p 3001 > len -> "invalid offset"; 4 bytes > 3 but < 5 -> too short
    assert list(status) == [oracle.FRAG_BAD_OFFSET, oracle.FRAG_OK, oracle.FRAG_TOO_SHORT]
    assert int(first[1]) == 0 and int(first[3]) == int(first[2])


# ------------------------------------------------------------------ HIP packetizer (GPU)
def _gpu_vs_oracle(codec, dev, recs_or_batch, max_udp_payload=1400, misalign=0, rpc_seed=3):
    import torch
    data, off = recs_or_batch if isinstance(recs_or_batch, tuple) else batch(recs_or_batch)
    n = len(off) - 1
    rpc = np.random.default_rng(rpc_seed).integers(0, 1 << 63, n, dtype=np.int64).view(np.uint64)
    want = oracle.fragment_batch(data, off, rpc, packet_type=1, dst=(bytes([127, 0, 0, 1]), 9000),
                                 src=(bytes([127, 0, 0, 1]), 9001), max_udp_payload=max_udp_payload)
    _, d = put(np.concatenate([data, np.zeros(1, np.uint8)]), dev, misalign)
    d = d[:len(data)] if len(data) else d[:0]
    _, o = put(off, dev)
    _, r = put(rpc, dev)
    got = codec.fragment(d, o, r, 1, ((127, 0, 0, 1), 9000), ((127, 0, 0, 1), 9001), max_udp_payload)
    codec.check()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.status.cpu().numpy(), want[4], err_msg="status")
    np.testing.assert_array_equal(got.first.cpu().numpy().view(np.uint64), want[2], err_msg="first")
    np.testing.assert_array_equal(got.wire_off.cpu().numpy().view(np.uint64), want[3], err_msg="wire_off")
    np.testing.assert_array_equal(got.dg_off.cpu().numpy().view(np.uint64), want[1], err_msg="dg_off")
    np.testing.assert_array_equal(got.wire.cpu().numpy(), want[0], err_msg="wire bytes")
    return want


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


@pytest.mark.gpu
def test_fragment_kats_gpu(gcodec, gdev):
    recs = [record(n_, o_, seed=i) for i, (n_, o_) in enumerate(
        [(350, 13), (MTU, 13), (MTU + 1, 13), (3000, 13), (5000, 3000), (3400, 1300), (2738, 0), (2000, 2000),
         (2000, 1369), (3000, 3001), (0, 0), (13, 13)])]
    _gpu_vs_oracle(gcodec, gdev, recs, misalign=5)


@pytest.mark.gpu
@pytest.mark.parametrize("max_udp_payload", [1400, 64, 34])
@pytest.mark.parametrize("seed", [1, 2])
def test_fragment_random_gpu(gcodec, gdev, max_udp_payload, seed):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(3000):
        L = int(rng.choice([rng.integers(0, 40), rng.integers(0, 1500), rng.integers(1300, 9000)]))
        o = int(rng.choice([13, rng.integers(0, L + 2) if L else 0, L, L + 1]))
        recs.append(record(L, o, seed=seed * 10000 + i))
    want = _gpu_vs_oracle(gcodec, gdev, recs, max_udp_payload, misalign=seed)
    assert (want[4] != 0).any() and (want[4] == 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 257])
def test_fragment_edge_counts_gpu(gcodec, gdev, n):
    recs = [record(int(L), 13, seed=i) for i, L in enumerate(np.random.default_rng(n).integers(13, 3000, n))]
    _gpu_vs_oracle(gcodec, gdev, recs if n else (np.zeros(0, np.uint8), np.zeros(1, np.uint64)))


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["config2", "config3"])
def test_fragment_encoded_batches_gpu(gcodec, gdev, cfg):
    kw = dict(datagen.CONFIG2 if cfg == "config2" else datagen.CONFIG3, n=20000)
    b = datagen.make_batch(**kw)
    stream, off = oracle.encode_batch(b.fixed, b.var, 1, 2)
    want = _gpu_vs_oracle(gcodec, gdev, (stream, off))
    if cfg == "config2":  # 350-byte records: one datagram each
        assert int(want[2][-1]) == b.n

"""Receive-side reassembly of DataPackets.

CPU tests pin the oracle (oracle/reassembly_oracle.c) with hand-derived cases read off
pkg/transport/fragmentation.go:49-183 (duplicates overwrite, the ARRIVING packet's TotalPackets
decides, fragment indices, RPCID reuse after completion), the parse/routing rules of
pkg/transport/transport.go:253-317 and pkg/packet/builtin_packets.go:118-161, and round trips through
the packetizer oracle (the reference has no test of DataReassembler: SURVEY.md 4).
GPU tests compare the HIP reassembler with the oracle bit-exactly on the same batches, on
adversarial arrival orders, and on the packetized config-2/3 streams.
"""
import struct

import numpy as np
import pytest

from arpc_amd import datagen
from oracle import oracle


def dgram(rpc, total, seq, payload=b"", more=False, fidx=0, ptype=1, extra=b"", plen=None):
    """DataPacketCodec.Serialize (builtin_packets.go:59-114) plus optional trailing bytes."""
    h = struct.pack("<BQHHBB4sH4sHI", ptype, rpc, total, seq, int(more), fidx, b"\x7f\0\0\1", 9000, b"\x7f\0\0\1",
                    9001, len(payload) if plen is None else plen)
    assert len(h) == 31
    return h + payload + extra


def batch(dgs):
    off = np.zeros(len(dgs) + 1, np.uint64)
    np.cumsum([len(d) for d in dgs], out=off[1:])
    return np.frombuffer(b"".join(dgs), np.uint8).copy(), off


def messages(dgs):
    msg, off, rpc, dg, st = oracle.reassemble(*batch(dgs))
    out = [(int(rpc[i]), int(dg[i]), msg[int(off[i]):int(off[i + 1])].tobytes()) for i in range(len(rpc))]
    return out, list(st)


C, P = oracle.RX_CONSUMED, oracle.RX_PENDING


# ------------------------------------------------------------------ oracle pinning (CPU)
def test_oracle_single_and_out_of_order():
    got, st = messages([dgram(7, 1, 0, b"hello"), dgram(9, 3, 2, b"C"), dgram(9, 3, 0, b"A"), dgram(9, 3, 1, b"B")])
    assert got == [(7, 0, b"hello"), (9, 3, b"ABC")] and st == [C, C, C, C]


def test_oracle_duplicate_overwrites():
    got, st = messages([dgram(5, 2, 0, b"old"), dgram(5, 2, 0, b"new"), dgram(5, 2, 1, b"!")])
    assert got == [(5, 2, b"new!")] and st == [C, C, C]


def test_oracle_interleaved_completion_order():
    got, _ = messages([dgram(1, 2, 0, b"a0"), dgram(2, 2, 1, b"b1"), dgram(2, 2, 0, b"b0"), dgram(1, 2, 1, b"a1")])
    assert got == [(2, 2, b"b0b1"), (1, 3, b"a0a1")]


def test_oracle_incomplete_and_extra_sequences():
    got, st = messages([dgram(3, 3, 0, b"x"), dgram(3, 3, 1, b"y"),               # 2 of 3: pending
                        dgram(4, 2, 0, b"p"), dgram(4, 2, 5, b"q"), dgram(4, 2, 1, b"r"),  # seq 5 of 2: never
                        dgram(6, 0, 0, b"z")])                                    # TotalPackets 0: never
    assert got == [] and st == [P] * 6


def test_oracle_arriving_total_decides():
    got, _ = messages([dgram(8, 3, 0, b"A"), dgram(8, 2, 1, b"B")])
    assert got == [(8, 1, b"AB")]


def test_oracle_fragment_indices():
    got, _ = messages([dgram(1, 1, 0, b"-second", fidx=1), dgram(1, 1, 0, b"first", more=True, fidx=0),
                       dgram(2, 1, 0, b"a", more=True), dgram(2, 1, 0, b"b", fidx=2), dgram(2, 1, 0, b"c", fidx=1)])
    assert got == [(1, 1, b"first-second"), (2, 4, b"acb")]  # index order 0, 1, 2
    got, st = messages([dgram(3, 1, 0, b"a", more=True), dgram(3, 1, 0, b"c", fidx=2)])  # index 1 missing
    assert got == [] and st == [P, P]


def test_oracle_rpc_reuse_after_completion():
    got, _ = messages([dgram(4, 1, 0, b"one"), dgram(4, 1, 0, b"two"), dgram(4, 2, 0, b"th"), dgram(4, 2, 1, b"ree")])
    assert got == [(4, 0, b"one"), (4, 1, b"two"), (4, 3, b"three")]


def test_oracle_parse_errors():
    got, st = messages([b"", dgram(1, 1, 0, b"e", ptype=3), dgram(1, 1, 0, b"u", ptype=9), b"\x01" * 30,
                        dgram(1, 1, 0, b"short", plen=100), dgram(1, 1, 0, b"ok", extra=b"trailing"),
                        dgram(2, 1, 0, b"resp", ptype=2)])
    assert st == [oracle.RX_TOO_SHORT, oracle.RX_NOT_DATA, oracle.RX_NOT_DATA, oracle.RX_TOO_SHORT,
                  oracle.RX_BAD_LENGTH, C, C]
    assert got == [(1, 5, b"ok"), (2, 6, b"resp")]


def packetized(cfg, n, max_udp_payload=1400):
    kw = dict(cfg, n=n)
    b = datagen.make_batch(**kw)
    stream, off = oracle.encode_batch(b.fixed, b.var, 1, 2)
    rpc = (np.arange(n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ np.uint64(0x1234)
    wire, dg_off, *_ = oracle.fragment_batch(stream, off, rpc, max_udp_payload=max_udp_payload)
    return stream, off, rpc, wire, dg_off


def shuffled(wire, dg_off, perm):
    dgs = [wire[int(dg_off[j]):int(dg_off[j + 1])].tobytes() for j in perm]
    return batch(dgs)


@pytest.mark.parametrize("mtu", [1400, 200])
def test_oracle_round_trip_through_packetizer(mtu):
    stream, off, rpc, wire, dg_off = packetized(datagen.CONFIG3, 300, mtu)
    nd = len(dg_off) - 1
    for perm in (np.arange(nd), np.random.default_rng(1).permutation(nd)):
        msg, moff, mrpc, mdg, st = oracle.reassemble(*shuffled(wire, dg_off, perm))
        assert (st == C).all() and len(mrpc) == 300
        want = {int(rpc[i]): stream[int(off[i]):int(off[i + 1])].tobytes() for i in range(300)}
        got = {int(mrpc[i]): msg[int(moff[i]):int(moff[i + 1])].tobytes() for i in range(300)}
        assert got == want


def adversarial(n_msgs, seed):
    """Messages of 1-40 fragments (some with fragment indices), shuffled and interleaved; duplicates,
    drops, RPCID collisions, wrong totals, corrupt headers."""
    rng = np.random.default_rng(seed)
    dgs = []
    for m in range(n_msgs):
        rpc = int(rng.integers(0, n_msgs // 3 + 2)) if rng.random() < 0.3 else int(rng.integers(0, 1 << 63))
        if rng.random() < 0.02:
            rpc = (1 << 64) - 1  # the hash table's empty key
        T = int(rng.choice([1, 1, 2, 3, rng.integers(1, 41)]))
        for s in range(T):
            nf = 1 if rng.random() < 0.8 else int(rng.integers(1, 4))
            for f in range(nf):
                dgs.append(dgram(rpc, T, s, rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes(),
                                 more=f < nf - 1, fidx=f))
        if rng.random() < 0.1:
            dgs.append(dgram(rpc, T, int(rng.integers(0, T + 3)), b"dup"))
        if rng.random() < 0.05:
            dgs.append(dgram(rpc, int(rng.integers(0, T + 2)), 0, b"tot"))
    for _ in range(len(dgs) // 50):
        dgs.insert(int(rng.integers(0, len(dgs) + 1)),
                   rng.choice([b"", b"\x03" * 40, b"\x01" * 12, dgram(1, 1, 0, b"x", plen=77)]))
    order = rng.permutation(len(dgs)) if seed % 2 else np.argsort(rng.random(len(dgs)) + np.arange(len(dgs)) / 20)
    drop = rng.random(len(dgs)) < 0.03
    return [dgs[i] for i in order if not drop[i]]


def test_oracle_adversarial_is_mixed():
    got, st = messages(adversarial(400, 3))
    assert len(got) > 100 and {C, P, oracle.RX_NOT_DATA, oracle.RX_TOO_SHORT, oracle.RX_BAD_LENGTH} <= set(st)


# ------------------------------------------------------------------ HIP reassembler (GPU)
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


def _gpu_vs_oracle(codec, dev, wire, dg_off, misalign=0, cap=None):
    import torch
    want = oracle.reassemble(wire, dg_off)
    buf = torch.full((wire.size + misalign + 32,), 0xA5, dtype=torch.uint8, device=dev)
    if wire.size:
        buf[misalign:misalign + wire.size].copy_(torch.from_numpy(wire))
    w = buf[misalign:misalign + wire.size]
    o = torch.from_numpy(dg_off.view(np.int64).copy()).to(dev)
    r = codec.reassemble(w, o, cap=cap)
    codec.check()
    k = int(r.nmsg.item())
    assert k == len(want[2]), (k, len(want[2]))
    np.testing.assert_array_equal(r.status.cpu().numpy(), want[4], err_msg="status")
    np.testing.assert_array_equal(r.offsets[:k + 1].cpu().numpy().view(np.uint64), want[1], err_msg="msg_off")
    np.testing.assert_array_equal(r.rpc_id[:k].cpu().numpy().view(np.uint64), want[2], err_msg="rpc")
    np.testing.assert_array_equal(r.dgram[:k].cpu().numpy().view(np.uint64), want[3], err_msg="completing dgram")
    np.testing.assert_array_equal(r.data[:int(want[1][-1])].cpu().numpy(), want[0], err_msg="message bytes")
    return want


@pytest.mark.gpu
def test_reassembly_kats_gpu(gcodec, gdev):
    dgs = [dgram(7, 1, 0, b"hello"), dgram(9, 3, 2, b"C"), dgram(9, 3, 0, b"A"), dgram(9, 3, 1, b"B"),
           dgram(5, 2, 0, b"old"), dgram(5, 2, 0, b"new"), dgram(5, 2, 1, b"!"), dgram(8, 3, 0, b"A"),
           dgram(8, 2, 1, b"B"), dgram(1, 1, 0, b"-second", fidx=1), dgram(1, 1, 0, b"first", more=True),
           dgram(4, 1, 0, b"one"), dgram(4, 1, 0, b"two"), b"", dgram(1, 1, 0, b"e", ptype=3), b"\x01" * 30,
           dgram(1, 1, 0, b"short", plen=100), dgram(1, 1, 0, b"ok", extra=b"trailing"),
           dgram(3, 3, 0, b"x"), dgram(6, 0, 0, b"z"), dgram((1 << 64) - 1, 1, 0, b"max")]
    _gpu_vs_oracle(gcodec, gdev, *batch(dgs), misalign=3)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_reassembly_adversarial_gpu(gcodec, gdev, seed):
    _gpu_vs_oracle(gcodec, gdev, *batch(adversarial(1500, seed)), misalign=seed)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 255, 256, 257])
def test_reassembly_edge_counts_gpu(gcodec, gdev, n):
    rng = np.random.default_rng(n)
    _gpu_vs_oracle(gcodec, gdev, *batch([dgram(int(rng.integers(0, 40)), int(rng.integers(1, 3)), int(rng.integers(0, 2)),
                                               b"p" * int(rng.integers(0, 50))) for _ in range(n)]))


@pytest.mark.gpu
def test_reassembly_large_message_gpu(gcodec, gdev):
    rng = np.random.default_rng(5)
    dgs = [dgram(77, 3000, s, bytes([s & 255]) * 13) for s in rng.permutation(3000)]
    want = _gpu_vs_oracle(gcodec, gdev, *batch(dgs))
    assert len(want[2]) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,mtu", [("config2", 1400), ("config3", 1400), ("config3", 300)])
def test_reassembly_round_trip_gpu(gcodec, gdev, cfg, mtu):
    stream, off, rpc, wire, dg_off = packetized(datagen.CONFIG2 if cfg == "config2" else datagen.CONFIG3, 20000, mtu)
    perm = np.random.default_rng(7).permutation(len(dg_off) - 1)
    want = _gpu_vs_oracle(gcodec, gdev, *shuffled(wire, dg_off, perm))
    assert len(want[2]) == 20000 and (want[4] == C).all()


@pytest.mark.gpu
def test_reassembly_large_shuffled_gpu(gcodec, gdev):
    """Single-datagram messages in a random order: still a simple batch (every DataPacket completes its
    own message on arrival), whatever the order."""
    stream, off, rpc, wire, dg_off = packetized(datagen.CONFIG2, 600000, 1400)
    perm = np.random.default_rng(11).permutation(len(dg_off) - 1)
    want = _gpu_vs_oracle(gcodec, gdev, *shuffled(wire, dg_off, perm))
    assert len(want[2]) == 600000 and (want[4] == C).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n,mtu,window", [(300000, 1400, 0), (60000, 300, 64)])
def test_reassembly_reordered_gpu(gcodec, gdev, n, mtu, window):
    """Config-3 records packetized and reordered, the general path against the oracle: a full
    permutation (~400k datagrams: ~200 sort tiles of 2048, three radix passes), or windows of 64 as
    UDP's local reordering does (bench.py's reassembly_config3_reordered at a 300-byte MTU: messages of
    up to ~16 packets in any order -- the group passes' permutation case -- and RPCIDs that another
    workgroup's datagram claimed in the table -- key_kernel's lookup)."""
    stream, off, rpc, wire, dg_off = packetized(datagen.CONFIG3, n, mtu)
    nd = len(dg_off) - 1
    rng = np.random.default_rng(n + window)
    perm = np.argsort(np.arange(nd) // window + rng.random(nd), kind="stable") if window else rng.permutation(nd)
    want = _gpu_vs_oracle(gcodec, gdev, *shuffled(wire, dg_off, perm))
    assert len(want[2]) == n and (want[4] == C).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 64, 257, 5000])
def test_reassembly_simple_batch_gpu(gcodec, gdev, n):
    """Batches of complete single-datagram messages take the device fast path (no grouping): parse
    errors and reused RPC IDs in between, with every misalignment of the wire buffer."""
    rng = np.random.default_rng(100 + n)
    bad = [b"", b"\x03" * 40, b"\x01" * 12, dgram(1, 1, 0, b"x", plen=77), dgram(2, 1, 0, b"e", ptype=3)]
    dgs = []
    for k in range(n):
        if rng.random() < 0.1:
            dgs.append(bad[int(rng.integers(0, len(bad)))])
        else:
            dgs.append(dgram(int(rng.integers(0, 50)), 1, 0, bytes(rng.integers(0, 256, int(rng.integers(0, 90)),
                                                                               dtype=np.uint8))))
    want = _gpu_vs_oracle(gcodec, gdev, *batch(dgs), misalign=n % 7)
    assert len(want[2]) == sum(1 for s in want[4] if s == C)


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_reassembly_one_fragment_makes_batch_general_gpu(gcodec, gdev, where):
    """One two-fragment message among single-datagram ones sends the batch down the general path."""
    singles = [dgram(k, 1, 0, bytes([k & 255]) * (k % 40)) for k in range(300)]
    pos = {"first": 0, "middle": 150, "last": 300}[where]
    dgs = singles[:pos] + [dgram(999, 2, 1, b"tail"), dgram(999, 2, 0, b"head")] + singles[pos:]
    want = _gpu_vs_oracle(gcodec, gdev, *batch(dgs))
    assert len(want[2]) == 301


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,mtu", [("config2", 1400), ("config3", 1400), ("config3", 300)])
def test_reassembly_send_order_gpu(gcodec, gdev, cfg, mtu):
    """The packetizer's send order with hashed RPCIDs (not increasing, so not packetizer runs): the
    general path's hash table, whose claiming arrivals come out in order (no sort), and groups that are
    one message of packets 0..T-1 each (no per-sequence state)."""
    stream, off, rpc, wire, dg_off = packetized(datagen.CONFIG2 if cfg == "config2" else datagen.CONFIG3, 20000, mtu)
    want = _gpu_vs_oracle(gcodec, gdev, wire, dg_off)
    assert len(want[2]) == 20000 and (want[4] == C).all()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_reassembly_nondecreasing_rpcids_gpu(gcodec, gdev, seed):
    """RPCIDs that never decrease but whose runs are not one clean message each: an RPCID reused
    back to back, packets out of order or duplicated inside a run, incomplete runs, extra
    sequences, fragment indices -- the run-head grouping with the full ProcessFragment machine."""
    rng = np.random.default_rng(seed)
    dgs = []
    r = 10
    for _ in range(400):
        r += int(rng.integers(0, 3))  # 0: the previous RPCID again
        T = int(rng.integers(1, 5))
        seqs = list(range(T))
        kind = int(rng.integers(0, 5))
        if kind == 1:
            rng.shuffle(seqs)
        elif kind == 2:
            seqs = seqs + [int(rng.integers(0, T))]  # a duplicate
        elif kind == 3 and T > 1:
            seqs = seqs[:-1]  # incomplete
        elif kind == 4:
            seqs = seqs + [T + 1]  # a sequence number past TotalPackets
        for s in seqs:
            if kind == 4 and T == 1 and rng.random() < 0.3:
                dgs.append(dgram(r, T, s, b"-second", fidx=1))
                dgs.append(dgram(r, T, s, b"first", more=True))
            else:
                dgs.append(dgram(r, T, s, bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))))
    _gpu_vs_oracle(gcodec, gdev, *batch(dgs), misalign=seed)


@pytest.mark.gpu
def test_reassembly_one_rpcid_over_a_large_batch_gpu(gcodec, gdev):
    """One RPCID repeated over 2^17 datagrams (non-decreasing, so the run-head path): pairs of
    packets 0, 1 of TotalPackets 2, each pair completing a message (RPCID reuse after completion,
    fragmentation.go:62-181), a duplicate and an incomplete tail.  The run head is found by a gallop
    and a binary search (the one-step walk back was O(run^2))."""
    n = 1 << 17
    dgs = []
    for k in range(n // 2):
        dgs.append(dgram(42, 2, 0, bytes([k & 255]) * (k % 23)))
        if k == 777:
            dgs.append(dgram(42, 2, 0, b"dup"))
        dgs.append(dgram(42, 2, 1, b"#"))
    dgs.append(dgram(42, 2, 0, b"left open"))
    want = _gpu_vs_oracle(gcodec, gdev, *batch(dgs))
    assert len(want[2]) == n // 2


@pytest.mark.gpu
def test_reassembly_packetizer_runs_gpu(gcodec, gdev):
    """Batches of packetizer runs (every datagram a DataPacket, RPCIDs non-decreasing, each run of
    equal RPCIDs sequence numbers 0..k-1 of TotalPackets k, one fragment each) complete without the
    general path (reassemble.hip parse_kernel / emit_kernel, "runs"); every near miss -- a run
    reusing the previous RPCID, a missing or duplicated packet, interleaved RPCIDs, an error packet
    between runs, a second fragment, a TotalPackets that changes inside a run, an incomplete last run --
    takes the general path.  All against the oracle, then capacities: one the messages exceed (an
    error), and one the wire exceeds but the messages fit."""
    import torch
    from arpc_amd import _native
    runs = [dgram(1, 2, 0, b"ab"), dgram(1, 2, 1, b"cd"), dgram(2, 1, 0, b"e"), dgram(3, 3, 0, b"f"),
            dgram(3, 3, 1, b""), dgram(3, 3, 2, b"h"), dgram(7, 1, 0, b"")]
    near = [
        runs[:2] + [dgram(1, 2, 0, b"AB"), dgram(1, 2, 1, b"CD")],        # the same RPCID again
        runs[:1] + runs[2:],                                              # a missing packet
        runs[:2] + [dgram(1, 2, 1, b"cd")] + runs[2:],                    # a duplicate
        [dgram(1, 2, 0, b"ab"), dgram(2, 2, 0, b"xy"), dgram(1, 2, 1, b"cd"), dgram(2, 2, 1, b"zw")],
        runs[:2] + [dgram(2, 1, 0, b"e", ptype=3)] + runs[3:],           # an error packet
        runs[:2] + [dgram(2, 1, 0, b"e", fidx=1)] + runs[3:],            # a second fragment
        runs[:3] + [dgram(3, 3, 0, b"f"), dgram(3, 2, 1, b""), dgram(3, 3, 2, b"h")],
        runs + [dgram(9, 2, 0, b"open")],                                 # an incomplete last run
        runs[:2] + [dgram(2, 1, 0, b"e", more=True)] + runs[3:],         # more fragments announced
    ]
    for dgs in [runs] + near:
        _gpu_vs_oracle(gcodec, gdev, *batch(dgs))
    for lo in range(1, 5):  # runs across workgroup edges
        dgs = []
        for r in range(600):
            k = 1 + (r * 7 + lo) % 5
            dgs += [dgram(100 + r, k, q, bytes([r & 255]) * ((r + q) % 9)) for q in range(k)]
        _gpu_vs_oracle(gcodec, gdev, *batch(dgs), misalign=lo)
    wire, off = batch(runs)
    w, o = torch.from_numpy(wire).to(gdev), torch.from_numpy(off.view(np.int64).copy()).to(gdev)
    gcodec.reassemble(w, o, cap=5)  # the messages hold 7 bytes
    with pytest.raises(_native.SymphonyHipError):
        gcodec.check()
    gcodec.check()
    big_open = [dgram(1, 2, 0, b"a" * 100), dgram(1, 2, 1, b"b" * 100), dgram(9, 2, 0, b"z" * 5000)]
    want = _gpu_vs_oracle(gcodec, gdev, *batch(big_open), cap=300)  # the wire holds 5293 bytes, the messages 200
    assert int(want[1][-1]) == 200

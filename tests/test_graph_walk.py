"""Tree walks captured as HIP graphs (arpc_amd.flat.EncodeGraph / DecodeGraph).

A replay must give exactly what the eager walk gives: the encode's bytes equal to the restatement's
MarshalSymphony (oracle/nested_ref.py) per record, and the decode's fields and statuses equal to
the restatement's UnmarshalSymphony -- also after the bound buffers are refilled with another batch
(including corrupted records, whose statuses and failure positions come from the device).
"""
import numpy as np
import pytest

from oracle import nested_ref as ref

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


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


def _records(data, off, n):
    b = data.cpu().numpy().tobytes()
    o = off.cpu().numpy()
    return [b[o[i]:o[i + 1]] for i in range(n)]


def test_encode_graph_boutique_and_refill(codec, dev):
    """PlaceOrderResponses: replay == restatement per record; the bound columns refilled in place
    (same shapes, new values) -> the replay encodes the new values."""
    from arpc_amd import datagen, flat
    from tests.test_nested import tree_records
    sch = flat.OB_PLACE_ORDER_RESPONSE
    n = 300
    tree = datagen.ob_place_order(n, seed=11)
    cols = flat.columns_from_tree(sch, tree[1], dev)
    g = flat.EncodeGraph(dev, sch, cols)
    for rep in range(2):
        data, off = g.replay()
        torch.cuda.synchronize()
        g.codec.check()
        assert _records(data, off, n) == [ref.marshal(sch, r) for r in tree_records(sch, tree[1], n)]
        # refill: the Money units of every order item's cost and the zip codes, in place
        money = tree[1][0][1][4][1][1][1][1]  # OrderResult.Items -> OrderItem.Cost -> Money.Units
        money[:] = money * 3 + rep + 1
        zipc = tree[1][0][1][3][1][4]
        zipc[:] = zipc + 7
        cols[0].cols[4].cols[1].cols[1].copy_(torch.from_numpy(money).to(dev))
        cols[0].cols[3].cols[4].copy_(torch.from_numpy(zipc).to(dev))


def test_decode_graph_batches_and_corruption(codec, dev):
    """Three batches of n orders through one DecodeGraph's bound buffers: two clean, one with
    corrupted records; fields, statuses and failure positions equal the eager decode's, and the
    clean ones re-encode to their input."""
    from arpc_amd import datagen, flat
    sch = flat.OB_PLACE_ORDER_RESPONSE
    n = 400
    batches = []
    for seed in (21, 22):
        data, off = flat.encode(codec, sch, flat.columns_from_tree(sch, datagen.ob_place_order(n, seed=seed)[1], dev))
        batches.append((data.clone(), off.clone()))
    bad = batches[1][0].clone()
    o = batches[1][1].cpu().numpy()
    rng = np.random.default_rng(5)
    for i in rng.choice(n, 40, replace=False):  # a byte of the header / table / first prefix of 40 records
        bad[int(o[i]) + int(rng.integers(0, 40))] ^= 0xFF
    batches.append((bad, batches[1][1].clone()))
    cap = int(1.5 * max(d.numel() for d, _ in batches))
    dbuf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    obuf = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    dbuf[:batches[0][0].numel()] = batches[0][0]
    obuf.copy_(batches[0][1])
    g = flat.DecodeGraph(dev, sch, dbuf, obuf)
    for k, (d, o) in enumerate(batches):
        dbuf[:d.numel()] = d
        obuf.copy_(o)
        cols, st, fail = g.replay(with_fail=True)
        ecols, est, efail = flat.decode(codec, sch, d, o, span=d.numel(), with_fail=True)
        torch.cuda.synchronize()
        g.codec.check()
        codec.check()
        assert torch.equal(st, est) and torch.equal(fail, efail)
        if k < 2:
            assert bool((st == 0).all().item())
            rd, ro = flat.encode(codec, sch, cols)
            assert torch.equal(rd, d) and torch.equal(ro, o)
        else:
            assert int((st != 0).sum().item()) > 0
            # the records that decode cleanly decode to the same fields as eager
            ok = (st == 0).cpu().numpy()
            a = flat.encode(codec, sch, cols)
            b = flat.encode(codec, sch, ecols)
            assert [r for r, good in zip(_records(*a, n), ok) if good] == \
                [r for r, good in zip(_records(*b, n), ok) if good]


def test_graphs_flat_schema(codec, dev):
    """A flat schema (one level, no lists): both graphs equal the eager calls."""
    from arpc_amd import flat
    sch = flat.TEST_FIXED
    n = 1000
    gen = torch.Generator().manual_seed(3)
    cols = []
    for f in sch.fields:
        dt = flat.DTYPE[f.kind]
        cols.append(torch.randint(-2 ** 31, 2 ** 31 - 1, (n,), generator=gen, dtype=torch.int64).to(dt).to(dev)
                    if dt != torch.uint8 else torch.randint(0, 2, (n,), generator=gen, dtype=torch.uint8).to(dev))
    data, off = flat.encode(codec, sch, cols)
    eg = flat.EncodeGraph(dev, sch, cols)
    gd, go = eg.replay()
    torch.cuda.synchronize()
    assert torch.equal(gd, data) and torch.equal(go, off)
    dg = flat.DecodeGraph(dev, sch, data.clone(), off.clone())
    dcols, st = dg.replay()
    torch.cuda.synchronize()
    assert bool((st == 0).all().item())
    for a, b in zip(dcols, cols):
        assert torch.equal(a, b)


def test_user_capture_of_branching_encode(codec, dev):
    """A caller's own torch.cuda.graph around the eager flat.encode of a tree whose levels are large
    enough to fork branch streams (2^17 orders: OrderResult has three message fields, OrderItem two,
    so the eager walk forks from a fork -- the topology this ROCm's hipStreamEndCapture segfaults on,
    DESIGN.md section 4).  Under capture the walk takes no branches (flat._fork_min), the capture ends,
    and the replay equals the eager (branching) encode byte for byte and the restatement per record."""
    from arpc_amd import datagen, flat
    from tests.test_nested import tree_records
    sch = flat.OB_PLACE_ORDER_RESPONSE
    n = 1 << 17
    tree = datagen.ob_place_order(n, seed=17)
    cols = flat.columns_from_tree(sch, tree[1], dev)
    want, woff = flat.encode(codec, sch, cols)
    torch.cuda.synchronize()
    codec.check()
    assert len(codec.__dict__.get("_branches", [])) >= 2  # the eager walk did fork, twice deep
    buf = torch.empty(want.numel() + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):  # warm-up on a side stream, as torch's graph docs prescribe
        flat.encode(codec, sch, cols, out=(buf, off))
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        flat.encode(codec, sch, cols, out=(buf, off))
    buf.zero_()
    off.zero_()
    g.replay()
    torch.cuda.synchronize()
    codec.check()
    assert torch.equal(off, woff) and torch.equal(buf[:want.numel()], want)
    recs = tree_records(sch, tree[1], n)
    idx = np.random.default_rng(3).choice(n, 500, replace=False)
    got = _records(buf, off, n)
    assert [got[i] for i in idx] == [ref.marshal(sch, recs[i]) for i in idx]
    with pytest.raises(ValueError):  # the walks that need a host read say so instead of breaking a capture
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            flat.decode(codec, sch, want, woff)

"""Sharded (multi-GPU) record batches: ranges, offset rebasing and the cross-rank offset scan.

The N>1 path is exercised with world_size 2 on the gloo backend (CPU).  The oracle stands
in for each rank's encoder here: what is under test is the host-side sharding logic, whose
contract is that concatenating the shards' streams in rank order, with record offsets
rebased by the exclusive scan of shard totals, equals a single encode of the whole batch.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from arpc_amd import datagen, shard
from oracle import oracle


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [z - a for a, z in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_shards_concatenate_to_single_stream():
    b = datagen.make_batch(**datagen.CORPORA["set_mixed"])
    whole, whole_off = oracle.encode_batch(b.fixed, b.var)
    parts, totals = [], []
    for r in range(3):
        lo, hi = shard.shard_range(b.n, 3, r)
        data, off = oracle.encode_batch([], shard.shard_columns(b.var, lo, hi))
        parts.append((data, off))
        totals.append(int(off[-1]))
    bases = shard.exclusive_scan(totals)
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), whole)
    glob = np.concatenate([p[1][:-1] + np.uint64(base) for p, base in zip(parts, bases)] + [[sum(totals)]])
    np.testing.assert_array_equal(glob.astype(np.uint64), whole_off)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = datagen.make_batch(**datagen.CORPORA["set_tiny"])
        lo, hi = shard.shard_range(b.n, world, rank)
        data, off = oracle.encode_batch([], shard.shard_columns(b.var, lo, hi))
        base, total = shard.global_base(int(off[-1]))
        q.put((rank, base, total, data.tobytes(), (off + np.uint64(base)).tobytes()))
    finally:
        dist.destroy_process_group()


def test_global_base_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = datagen.make_batch(**datagen.CORPORA["set_tiny"])
    whole, whole_off = oracle.encode_batch(b.fixed, b.var)
    assert got[0][1] == 0 and got[1][1] == len(got[0][3])
    assert all(g[2] == len(whole) for g in got)
    assert b"".join(g[3] for g in got) == whole.tobytes()
    offs = [np.frombuffer(g[4], dtype=np.uint64) for g in got]
    np.testing.assert_array_equal(np.concatenate([offs[0][:-1], offs[1]]), whole_off)

"""One rank of the world-2 HIP sharding test (tests/test_full_size.py::test_world2_hip_shards).

Started as a child process (subprocess, a fresh interpreter) with RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set; every rank uses device 0 of the one-GPU box and gloo for the control traffic, as
`bench.py` does under SYMHIP_BENCH_ONE_GPU=1.  Rank g encodes ITS shard (config-4 seeds,
0x5EED0003 + g) with the HIP encoder through the C ABI, decodes it back with the HIP decoder and
checks every column, rebases its record offsets with shard.global_base (the one all_gather of shard
totals), and writes its stream and global offsets to OUT_DIR for the parent to
compare with the C oracle's single-batch encoding.

  python tests/shard_worker.py OUT_DIR RECORDS
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir, records = sys.argv[1], int(sys.argv[2])
    import torch
    import torch.distributed as dist

    from arpc_amd import datagen, shard
    from arpc_amd.codec import Codec, to_device

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        codec = Codec(dev)
        b = datagen.make_batch(**datagen.config4_shard(rank, records))
        fixed, var = to_device(b, dev)
        enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
        dec = codec.decode(b.schema, enc.data, enc.offsets, caps=[int(o[-1]) for _, o in b.var])
        codec.check()
        assert int(dec.status.sum().item()) == 0, "decode status"
        for f, (bcol, ocol) in enumerate(var):
            assert torch.equal(dec.var[f][1], ocol - ocol[0]), f"decoded offsets, field {f}"
            assert torch.equal(dec.var[f][0][:bcol.numel()], bcol), f"decoded bytes, field {f}"
        total = b.encoded_size()
        base, gtotal = shard.global_base(total)
        stream = enc.data[:total].cpu().numpy()
        goff = enc.offsets.cpu().numpy().view(np.uint64) + np.uint64(base)
        np.save(os.path.join(out_dir, f"stream{rank}.npy"), stream)
        np.save(os.path.join(out_dir, f"off{rank}.npy"), goff)
        with open(os.path.join(out_dir, f"meta{rank}.txt"), "w") as f:
            f.write(f"{base} {gtotal} {total}\n")
        codec.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Writes tests/golden/full_size_digests.json: SHA-256 pins of the C oracle's encoding of the
BASELINE.json workloads at their full sizes.

  config2        2^20 SetRequest, K=64, V=256, seed 0x5EED0001
  config3        2^20 SetRequest, K=64, V log-uniform 16-4096, seed 0x5EED0002
  config2_mixed  2^20 Get/Set requests at the trace's 36.9 % Set, client IDs 1 / 1 / 2
  config4_shard0 2^23 SetRequest, K=64, V=256, seed 0x5EED0003 (shard 0 of the 2^26-record batch)
  config4_w2     shards 0 and 1 of 2^20 records each (seeds 0x5EED0003 + g) encoded as ONE batch:
                 what the world-2 test's concatenated per-rank HIP streams must equal

These are self-consistency pins of the oracle (oracle/symphony_oracle.c, a restatement of the
generated Go in benchmark/kv-store-symphony/symphony/kv.syn.go:74-132, :611-678), so the GPU tests
can check a whole stream against a value fixed in the repo as well as against the oracle run beside
them.  Run: python tests/golden/make_full_digests.py  (about a minute, ~12 GB of host memory).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from arpc_amd import datagen  # noqa: E402
from oracle import oracle  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def concat_shards(batches):
    """String columns of several batches as one batch's columns (offsets rebased)."""
    cols = []
    for f in range(len(batches[0].var)):
        by = np.concatenate([b.var[f][0] for b in batches])
        offs, base = [np.zeros(1, np.uint64)], np.uint64(0)
        for b in batches:
            o = b.var[f][1]
            offs.append(o[1:] - o[0] + base)
            base += np.uint64(o[-1] - o[0])
        cols.append((by, np.concatenate(offs)))
    return cols


def pin(stream: np.ndarray, off: np.ndarray) -> dict:
    return {"sha256_stream": sha(stream), "sha256_offsets": sha(off.astype(np.uint64)),
            "stream_bytes": int(stream.size), "records": int(off.size - 1)}


def main():
    out = {}
    for name, kw in (("config2", datagen.CONFIG2), ("config3", datagen.CONFIG3),
                     ("config4_shard0", datagen.config4_shard(0))):
        b = datagen.make_batch(**kw)
        s, o = oracle.encode_batch(b.fixed, b.var)
        out[name] = pin(s, o)
        del b, s, o
    m = datagen.make_mixed_batch(**datagen.CONFIG2_MIXED)
    s, o = oracle.encode_kv_mixed(m.type, m.key, m.val, 1, 1, 2)
    out["config2_mixed"] = pin(s, o)
    del m, s, o
    shards = [datagen.make_batch(**datagen.config4_shard(g, 1 << 20)) for g in range(2)]
    s, o = oracle.encode_batch([], concat_shards(shards))
    out["config4_w2"] = pin(s, o)
    with open(os.path.join(HERE, "full_size_digests.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

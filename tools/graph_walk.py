"""The boutique tree walk (bench `boutique` leg: 2^18 PlaceOrderResponses) eager against captured as a
HIP graph (arpc_amd.flat.EncodeGraph / DecodeGraph): results equal, then the host clock of each.

    python tools/graph_walk.py [--n 262144] [--reps 10]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from arpc_amd import datagen, flat
    from arpc_amd.codec import Codec
    dev = torch.device("cuda:0")
    codec = Codec(dev)
    sch = flat.OB_PLACE_ORDER_RESPONSE
    cols = flat.columns_from_tree(sch, datagen.ob_place_order(a.n)[1], dev)
    data, off = flat.encode(codec, sch, cols)
    torch.cuda.synchronize()
    print("eager encode done", flush=True)
    t0 = time.perf_counter()
    eg = flat.EncodeGraph(dev, sch, cols)
    t1 = time.perf_counter()
    gd, go = eg.replay()
    print(f"encode graph captured in {1e3 * (t1 - t0):.1f} ms; replay equal: "
          f"{torch.equal(gd, data) and torch.equal(go, off)}", flush=True)
    # a second batch of the same n, in the same bound buffers
    cols2 = flat.columns_from_tree(sch, datagen.ob_place_order(a.n, seed=7)[1], dev)
    data2, off2 = flat.encode(codec, sch, cols2)
    cap = int(1.25 * max(data.numel(), data2.numel()))
    dbuf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    obuf = off.clone()
    dbuf[:data.numel()] = data
    dg = flat.DecodeGraph(dev, sch, dbuf, obuf)
    for name, (d, o) in (("batch 1", (data, off)), ("batch 2", (data2, off2))):
        dbuf[:d.numel()] = d
        obuf.copy_(o)
        dcols, st = dg.replay()
        rd, ro = flat.encode(codec, sch, dcols)
        ecols, est = flat.decode(codec, sch, d, o, span=d.numel())
        print(f"decode graph {name}: status ok {bool((st == 0).all().item())}, re-encode equal "
              f"{torch.equal(rd, d) and torch.equal(ro, o)}, statuses as eager {torch.equal(st, est)}", flush=True)
    codec.check()
    eg.codec.check()
    dg.codec.check()
    dbuf[:data.numel()] = data
    obuf.copy_(off)

    def timed(fn):
        fn()
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return float(np.median(ts)) * 1e3
    for _ in range(2):
        e_enc = timed(lambda: flat.encode(codec, sch, cols))
        g_enc = timed(lambda: eg.replay())
        e_dec = timed(lambda: flat.decode(codec, sch, data, off, span=data.numel()))
        g_dec = timed(lambda: dg.replay())
        print(f"encode eager {e_enc:.3f} ms graph {g_enc:.3f} ms; decode eager {e_dec:.3f} ms graph {g_dec:.3f} ms; "
              f"eager {e_enc + e_dec:.3f} graph {g_enc + g_dec:.3f}", flush=True)


if __name__ == "__main__":
    main()

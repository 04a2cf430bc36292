"""Online-boutique PlaceOrderResponse tree (bench.py boutique leg) encoded and decoded `--reps` times,
for rocprofv3 kernel traces of the N5 nested path alone.

  python tools/boutique_run.py [--orders 262144] [--reps 5]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arpc_amd import datagen, flat  # noqa: E402
from arpc_amd.codec import Codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--orders", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    sch = flat.OB_PLACE_ORDER_RESPONSE
    tree = datagen.ob_place_order(a.orders)
    cols = flat.columns_from_tree(sch, tree[1], dev)
    data, off = flat.encode(codec, sch, cols)
    dcols, st = flat.decode(codec, sch, data, off)
    torch.cuda.synchronize()
    codec.check()
    te, td = [], []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d2, o2 = flat.encode(codec, sch, cols)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        flat.decode(codec, sch, data, off, span=data.numel())
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        te.append(t1 - t0)
        td.append(t2 - t1)
    codec.check()
    ok = bool(torch.equal(d2, data)) and bool(torch.equal(o2, off)) and bool((st == 0).all().item())
    print(f"orders {a.orders}, stream {int(off[-1].item())} B, round trip ok {ok}: encode {np.median(te) * 1e3:.3f} ms, "
          f"decode {np.median(td) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()

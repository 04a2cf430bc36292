"""Where a boutique graph replay's host-clocked time goes (bench.py boutique_leg's graphs), one process.

  python tools/boutique_replay_parts.py [--reps 20] [--n 262144]

For EncodeGraph and DecodeGraph: the median host time of replay() (what bench.py times), of launch()
plus a wait for its sizes (the GPU work and the D2H of the sizes), and of result() alone after that
wait (the Python that cuts the columns to the replay's sizes).
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from arpc_amd import datagen, flat  # noqa: E402
from arpc_amd.codec import Codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=1 << 18)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    sch = flat.OB_PLACE_ORDER_RESPONSE
    tree = datagen.ob_place_order(a.n)
    cols = flat.columns_from_tree(sch, tree[1], dev)
    data, off = flat.encode(codec, sch, cols)
    torch.cuda.synchronize()
    for name, g in (("encode", flat.EncodeGraph(dev, sch, cols)), ("decode", flat.DecodeGraph(dev, sch, data, off))):
        g.replay()
        torch.cuda.synchronize()
        t_rep, t_launch, t_res = [], [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            t_rep.append(time.perf_counter() - t0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.launch()
            g._sizes_read()
            t1 = time.perf_counter()
            g.result()
            t2 = time.perf_counter()
            t_launch.append(t1 - t0)
            t_res.append(t2 - t1)
        med = lambda x: statistics.median(x) * 1e6  # noqa: E731
        print(f"{name}: replay {med(t_rep):7.1f} us; launch + sizes {med(t_launch):7.1f} us; result() {med(t_res):6.1f} us",
              flush=True)
        g.codec.check()


if __name__ == "__main__":
    main()

"""Which tree walks capture as a HIP graph: flat encode / decode, then the boutique encode without and
with branch streams, each stage printed before it starts (a crash names its stage).  Its round-4 run
(profiles/r04_graph_stages.txt) crashed in hipStreamEndCapture at stage 5, the only one whose walk
forked branch streams inside the capture (a fork of a fork crashes it with torch ops alone:
tools/graph_fork.py); captures now keep every subtree on the capturing stream (arpc_amd/flat.py
_capture), and stage 5 is gone."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    from arpc_amd import datagen, flat
    from arpc_amd.codec import Codec
    dev = torch.device("cuda:0")
    codec = Codec(dev)
    n = 4096
    sch = flat.ELEMENT_SET_REQUEST
    g = torch.Generator().manual_seed(1)

    def strings(lo, hi):
        ln = torch.randint(lo, hi + 1, (n,), generator=g)
        o = torch.zeros(n + 1, dtype=torch.int64)
        o[1:] = torch.cumsum(ln, 0)
        return torch.randint(0, 256, (int(o[-1]),), generator=g, dtype=torch.uint8).to(dev), o.to(dev)
    cols = [torch.randint(0, 100, (n,), generator=g, dtype=torch.int32).to(dev), strings(4, 12), strings(16, 64),
            strings(64, 256)]
    data, off = flat.encode(codec, sch, cols)
    torch.cuda.synchronize()
    print("stage 1: flat encode graph", flush=True)
    eg = flat.EncodeGraph(dev, sch, cols)
    d, o = eg.replay()
    print("  equal", torch.equal(d, data) and torch.equal(o, off), flush=True)
    print("stage 2: flat decode graph", flush=True)
    dg = flat.DecodeGraph(dev, sch, data, off)
    c, st = dg.replay()
    d2, o2 = flat.encode(codec, sch, c)
    print("  re-encode equal", torch.equal(d2, data) and torch.equal(o2, off), flush=True)
    sch = flat.OB_PLACE_ORDER_RESPONSE
    for stage, nb, branch_min in ((3, 4096, 1 << 62), (4, 1 << 17, 1 << 62)):
        flat._BRANCH_MIN = branch_min
        cols = flat.columns_from_tree(sch, datagen.ob_place_order(nb)[1], dev)
        data, off = flat.encode(codec, sch, cols)
        torch.cuda.synchronize()
        print(f"stage {stage}: boutique encode graph, {nb} orders, branches from {branch_min}", flush=True)
        eg = flat.EncodeGraph(dev, sch, cols)
        d, o = eg.replay()
        print("  equal", torch.equal(d, data) and torch.equal(o, off), flush=True)
        print(f"stage {stage}b: boutique decode graph", flush=True)
        dg = flat.DecodeGraph(dev, sch, data, off)
        c, st = dg.replay()
        d2, o2 = flat.encode(codec, sch, c)
        print("  re-encode equal", torch.equal(d2, data) and torch.equal(o2, off), flush=True)
    print("all stages ok", flush=True)


if __name__ == "__main__":
    main()

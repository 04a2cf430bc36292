"""Multi-stream HIP graph capture on this ROCm: (1) torch ops only, one fork / join; (2) a nested
fork (a branch forking a branch); (3) arpc_amd's boutique encode walk with its branch streams,
capture_error_mode "relaxed".  Each stage prints before it starts: a crash names it."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

dev = torch.device("cuda:0")
x = torch.ones(1 << 20, device=dev)
s, b1, b2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def walk(nested):
    y = x * 2
    b1.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(b1):
        z = y + 1
        if nested:
            b2.wait_stream(b1)
            with torch.cuda.stream(b2):
                w = z * 3
            b1.wait_stream(b2)
            z = z + w
    torch.cuda.current_stream().wait_stream(b1)
    return y + z


for stage, nested in ((1, False), (2, True)):
    print(f"stage {stage}: torch fork/join{' nested' if nested else ''}", flush=True)
    with torch.cuda.stream(s):
        walk(nested)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = walk(nested)
    g.replay()
    torch.cuda.synchronize()
    print("  ok", float(out[0]), flush=True)

from arpc_amd import datagen, flat  # noqa: E402
from arpc_amd.codec import Codec  # noqa: E402
print("stage 3: boutique encode walk with branches, relaxed capture", flush=True)
codec = Codec(dev)
sch = flat.OB_PLACE_ORDER_RESPONSE
cols = flat.columns_from_tree(sch, datagen.ob_place_order(1 << 17)[1], dev)
data, off = flat.encode(codec, sch, cols)
c2 = Codec(dev)


def run(st):
    keep = []
    return flat._encode(c2, c2._ctx, sch, cols, 0, 0, st, None, None, False, keep, [0, flat._BRANCH_MIN]), keep


with torch.cuda.stream(s):
    run(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
    (buf, o), keep = run(s)
g.replay()
torch.cuda.synchronize()
print("  equal", torch.equal(buf[:data.numel()], data) and torch.equal(o, off), flush=True)

"""N5 decode / encode of the boutique tree: how long the host takes to queue the tree (the calls
return) against the whole call (queued + synchronised), to tell host-bound from device-bound."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arpc_amd import datagen, flat  # noqa: E402
from arpc_amd.codec import Codec  # noqa: E402

dev = torch.device("cuda", 0)
codec = Codec(dev)
sch = flat.OB_PLACE_ORDER_RESPONSE
cols = flat.columns_from_tree(sch, datagen.ob_place_order(1 << 18)[1], dev)
data, off = flat.encode(codec, sch, cols)
span = data.numel()
for _ in range(3):
    flat.decode(codec, sch, data, off, span=span)
    flat.encode(codec, sch, cols, out=(torch.empty_like(data), torch.empty_like(off)))
torch.cuda.synchronize()
orig = flat._finish_level
for it in range(5):
    marks = {}

    def fin(lvl, n, sizes, _o=orig):
        marks.setdefault("finish", time.perf_counter())
        return _o(lvl, n, sizes)
    flat._finish_level = fin
    cat = torch.cat

    def tcat(xs, *a, **k):
        marks["queued"] = time.perf_counter()
        return cat(xs, *a, **k)
    torch.cat = tcat
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    flat.decode(codec, sch, data, off, span=span)
    t1 = time.perf_counter()
    torch.cat = cat
    flat._finish_level = orig
    outb = (torch.empty_like(data), torch.empty_like(off))
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    flat.encode(codec, sch, cols, out=outb)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"decode: queued {1e3 * (marks['queued'] - t0):.3f} ms, sizes read {1e3 * (marks['finish'] - marks['queued']):.3f} ms, "
          f"total {1e3 * (t1 - t0):.3f} ms | encode: queued {1e3 * (t3 - t2):.3f} ms, total {1e3 * (t4 - t2):.3f} ms", flush=True)

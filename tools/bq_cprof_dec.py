"""Host profile of the N5 boutique decode alone (what the 0.36 ms of queueing is made of)."""
import cProfile
import os
import pstats
import sys

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
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    flat.decode(codec, sch, data, off, span=span)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)

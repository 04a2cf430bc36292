"""The boutique encode's levels, eager, `--reps` times (2^18 PlaceOrderResponses), for a kernel trace:
    rocprofv3 --kernel-trace --stats -d gpurun_out/el -- python tools/enc_levels.py
With the tuning library and SYMHIP_FLAT_VARIANT=1 each level's kernel runs its phase 1 only (wrong
output; timing), so the two traces split every level into phase 1 and the copy."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arpc_amd import datagen, flat  # noqa: E402
from arpc_amd.codec import Codec  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
codec = Codec(dev)
sch = flat.OB_PLACE_ORDER_RESPONSE
cols = flat.columns_from_tree(sch, datagen.ob_place_order(1 << 18)[1], dev)
for _ in range(reps):
    flat.encode(codec, sch, cols)
torch.cuda.synchronize()
print("done")

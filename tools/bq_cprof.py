import cProfile, pstats, sys, os
sys.path.insert(0, os.getcwd())
import torch
from arpc_amd import datagen, flat
from arpc_amd.codec import Codec
dev = torch.device("cuda", 0)
codec = Codec(dev)
sch = flat.OB_PLACE_ORDER_RESPONSE
tree = datagen.ob_place_order(1 << 18)
cols = flat.columns_from_tree(sch, tree[1], dev)
data, off = flat.encode(codec, sch, cols)
for _ in range(3):
    flat.decode(codec, sch, data, off); flat.encode(codec, sch, cols)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    flat.decode(codec, sch, data, off)
    torch.cuda.synchronize()
    flat.encode(codec, sch, cols)
    torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)

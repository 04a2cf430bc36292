"""Each boutique level's encoded stream size: every sub-tree encoded as its own batch (unframed records;
the tree walk frames inner levels, + 4 B each).  python tools/level_sizes.py"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from arpc_amd import datagen, flat
from arpc_amd.codec import Codec
dev = torch.device("cuda:0"); codec = Codec(dev)
root = flat.OB_PLACE_ORDER_RESPONSE
tree = datagen.ob_place_order(1 << 18)
def walk(sch, fields, rec, name, depth=0):
    cols = flat.columns_from_tree(sch, fields, dev)
    data, off = flat.encode(codec, sch, cols)
    nrec = off.numel() - 1
    print(f"{'  '*depth}{name}: {nrec} records, {int(off[-1].item() - off[0].item())} bytes", flush=True)
    for f, t in zip(sch.fields, fields):
        if getattr(f, 'kind', None) == 'message':
            walk(f.message, t[1], t[2], f.name, depth + 1)
walk(root, tree[1], None, "PlaceOrderResponse")

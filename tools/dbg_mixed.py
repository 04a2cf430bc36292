import sys, numpy as np, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, ".")
from arpc_amd.codec import Codec
from arpc_amd import datagen
from oracle import oracle
dev = torch.device("cuda", 0)
c = Codec(dev)
for n in (1024, 1100, 2048, 6000, 20000):
    b = datagen.make_mixed_batch(n=n, key=("uniform", 0, 20), value=("uniform", 0, 40), set_fraction=0.5, seed=3)
    want, woff = oracle.encode_kv_mixed(b.type, b.key, b.val)
    t = torch.from_numpy(b.type).to(dev)
    key = (torch.from_numpy(np.concatenate([b.key[0], np.zeros(16, np.uint8)])).to(dev), torch.from_numpy(b.key[1].view(np.int64)).to(dev))
    val = (torch.from_numpy(np.concatenate([b.val[0], np.zeros(16, np.uint8)])).to(dev), torch.from_numpy(b.val[1].view(np.int64)).to(dev))
    enc = c.encode_kv_mixed(t, key, val, out_bytes=len(want) + 64)
    torch.cuda.synchronize()
    try:
        c.check()
    except Exception as e:
        print("check:", e)
    off = enc.offsets.cpu().numpy().view(np.uint64)
    bad = np.nonzero(off != woff)[0]
    print(n, "bad offsets:", len(bad), "first", bad[:3], "got", off[bad[:3]] if len(bad) else None, "want", woff[bad[:3]] if len(bad) else None)
    if len(bad):
        d = off.astype(np.int64) - woff.astype(np.int64)
        tiles = np.unique(bad // 64)
        print("   bad tiles", tiles[:20], "delta per tile", [int(d[t*64]) for t in tiles[:20]])

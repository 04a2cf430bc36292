"""Cost of the speculative decode's re-decode: config-2 SetRequests where every k-th record carries
bytes after its last field (Go accepts them; the speculative lengths are then wrong and the gate
decodes the batch again exactly).  Times the default decode against the exact-parser pipeline
(tuning variant 710) in one process and checks both against each other.

  python tools/spec_misfit.py [--records 1048576] [--every 0,1000000,1000,1] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SYMHIP_LIBRARY", os.path.join(ROOT, "tools", "lib", "libsymphony_hip_tuning.so"))

from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--every", default="0,1000000,1000,1")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_batch(**dict(datagen.CONFIG2, n=a.records))
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    torch.cuda.synchronize()
    n, L = b.n, 350
    recs = enc.data[:n * L].view(n, L)
    for k in (int(x) for x in a.every.split(",")):
        if k == 0:
            data, off = enc.data, enc.offsets
        else:  # one trailing byte after records 0, k, 2k, ...
            extra = torch.zeros(n, dtype=torch.int64, device=dev)
            extra[::k] = 1
            off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(L + extra, 0)
            data = torch.zeros(int(off[-1].item()) + 16, dtype=torch.uint8, device=dev)
            idx = off[:-1].unsqueeze(1) + torch.arange(L, device=dev).unsqueeze(0)
            data[idx.reshape(-1)] = recs.reshape(-1)
        caps = [64 * n, 256 * n]
        times, digests = {}, {}
        for v in (0, 710):
            os.environ["SYMHIP_DECODE_VARIANT"] = str(v)
            ts = []
            for r in range(a.rounds + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                out = codec.decode(b.schema, data, off, caps=caps)
                e1.record()
                e1.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            codec.check()
            times[v] = statistics.median(ts)
            digests[v] = tuple(int(x.to(torch.int64).sum().item()) for x in (out.var[0][0], out.var[0][1], out.var[1][0],
                                                                             out.var[1][1], out.status))
        assert digests[0] == digests[710], f"every {k}: the speculative decode differs from the exact one"
        print(f"misfit every {k or 'none'}: default {times[0] * 1e3:8.1f} us   exact parsers (710) {times[710] * 1e3:8.1f} us")


if __name__ == "__main__":
    main()

"""N3 reassembly eager vs captured once as a HIP graph and replayed (torch.cuda.graph), one process.

  python tools/rx_graph.py [--reps 10]

config 3 packetized (the general path: ~25 launches, most of them gated no-ops for an in-order
stream) and config 2 packetized (the simple path).  HIP events around each call; the replayed
outputs are compared with the eager ones.
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    for name, cfg in (("config3", datagen.CONFIG3), ("config2", datagen.CONFIG2)):
        b = datagen.make_batch(**cfg)
        f, v = to_device(b, dev)
        e = codec.encode(b.schema, f, v, var_total=b.encoded_size() - b.n * b.schema.overhead)
        rpc = torch.arange(b.n, dtype=torch.int64, device=dev)
        dg = codec.fragment(e.data, e.offsets, rpc)
        del f, v
        torch.cuda.synchronize()
        ref = codec.reassemble(dg.wire, dg.dg_off)
        torch.cuda.synchronize()
        codec.check()
        k = int(ref.nmsg.item())
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):  # warm the side stream, then capture
            codec.reassemble(dg.wire, dg.dg_off)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = codec.reassemble(dg.wire, dg.dg_off)
        g.replay()
        torch.cuda.synchronize()
        codec.check()
        kb = int(ref.offsets[k].item())
        ok = int(out.nmsg.item()) == k and torch.equal(out.data[:kb], ref.data[:kb]) and \
            torch.equal(out.offsets[:k + 1], ref.offsets[:k + 1]) and torch.equal(out.status, ref.status)

        def timed(fn):
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            return statistics.median(ts), min(ts)
        te = timed(lambda: codec.reassemble(dg.wire, dg.dg_off))
        tg = timed(g.replay)
        print(f"{name}: eager median {te[0]:8.1f} us (min {te[1]:8.1f}); graph replay median {tg[0]:8.1f} us "
              f"(min {tg[1]:8.1f}); replay matches eager: {ok}", flush=True)
        del g, out, ref, dg, e


if __name__ == "__main__":
    main()

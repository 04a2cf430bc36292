"""Is the N3 reassembly call bound by the host's launch submission?  One process.

  python tools/rx_hostbound.py [--reps 10]

For config 3 (packetizer runs), config 2 (single-datagram messages) and config 3 with the datagrams
shuffled within windows of 64 (the general path, as bench.py's reassembly_config3_reordered) packetized: the call's host time (perf_counter
around codec.reassemble, no sync) and its GPU time (HIP events around it), once as is and once queued
behind a ~3 ms spin kernel (torch.cuda._sleep), so that every launch of the call is submitted before
the GPU reaches the first one.  If the second GPU time is much shorter, the host's submission rate,
not the kernels, sets the chain's pace.
"""
import argparse
import os
import statistics
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402
from bench import byte_gather  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="", help="run only this workload: config3, config2 or reordered")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    for key, name, cfg, window in (("config3", "config3", datagen.CONFIG3, 0), ("config2", "config2", datagen.CONFIG2, 0),
                                   ("reordered", "config3 reordered (windows of 64)", datagen.CONFIG3, 64)):
        if a.only and a.only != key:
            continue
        b = datagen.make_batch(**cfg)
        f, v = to_device(b, dev)
        e = codec.encode(b.schema, f, v, var_total=b.encoded_size() - b.n * b.schema.overhead)
        rpc = torch.arange(b.n, dtype=torch.int64, device=dev)
        dg = codec.fragment(e.data, e.offsets, rpc)
        del f, v
        if window:  # bench.py reassembly_leg's reordering
            nd = dg.dg_off.numel() - 1
            g = torch.Generator(device=dev)
            g.manual_seed(7)
            key = torch.div(torch.arange(nd, device=dev), window, rounding_mode="floor").double() + \
                torch.rand(nd, device=dev, dtype=torch.float64, generator=g)
            perm = torch.argsort(key)
            lens = (dg.dg_off[1:] - dg.dg_off[:-1])[perm]
            wire = byte_gather(dg.wire, dg.dg_off[:-1][perm], lens)
            off = torch.zeros(nd + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            dg = type(dg)(wire, off, *dg[2:]) if hasattr(dg, "_fields") else SimpleNamespace(wire=wire, dg_off=off)
        codec.reassemble(dg.wire, dg.dg_off)
        torch.cuda.synchronize()
        for behind in (False, True):
            host, gpu = [], []
            for _ in range(a.reps):
                if behind:
                    torch.cuda._sleep(3_000_000)  # ~1+ ms of spinning at 2.4 GHz
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                t0 = time.perf_counter()
                codec.reassemble(dg.wire, dg.dg_off)
                host.append((time.perf_counter() - t0) * 1e6)
                e1.record()
                torch.cuda.synchronize()
                gpu.append(e0.elapsed_time(e1) * 1e3)
            print(f"{name} {'behind a spin kernel' if behind else 'as is             '}: GPU median "
                  f"{statistics.median(gpu):8.1f} us, host submit median {statistics.median(host):8.1f} us", flush=True)
        codec.check()
        del dg, e


if __name__ == "__main__":
    main()

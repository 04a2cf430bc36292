"""Is the N3 reassembly call bound by the host's launch submission?  One process.

  python tools/rx_hostbound.py [--reps 10]

For config 3 (general path) and config 2 (simple path) packetized: the call's host time (perf_counter
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

"""A/B of segment-gather variants (tuning library, SYMHIP_GATHER_VARIANT) in ONE process, like kbench.py.

  python tools/rx_ab.py [--variants 0,3] [--rounds 10]

Workloads: N3 reassembly of config 3 packetized (multi-datagram messages, segments of ~640 bytes: the
packetizer-runs path), of config 2 packetized (single-datagram messages) and of config 3 packetized with
the datagrams shuffled within windows of 64 (the general path), and the N1 firewall (kept records
gathered).
Each round runs every variant once per workload, HIP events around each call; prints median / min per
variant and reports any defined output (message bytes, the first nmsg+1 offsets, ...) of a variant that
differs from the first variant's.
"""
import argparse
import os
import statistics
import sys
from types import SimpleNamespace

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SYMHIP_LIBRARY", os.path.join(ROOT, "tools", "lib", "libsymphony_hip_tuning.so"))

from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402
from bench import byte_gather  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,3")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--env", default="SYMHIP_GATHER_VARIANT", help="the tuning variable the variants set")
    a = ap.parse_args()
    variants = [int(v) for v in a.variants.split(",")]
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    work = {}
    for name, cfg, window in (("rx_config3", datagen.CONFIG3, 0), ("rx_config2", datagen.CONFIG2, 0),
                              ("rx_config3_w64", datagen.CONFIG3, 64)):
        b = datagen.make_batch(**cfg)
        f, v = to_device(b, dev)
        e = codec.encode(b.schema, f, v, var_total=b.encoded_size() - b.n * b.schema.overhead)
        rpc = torch.arange(b.n, dtype=torch.int64, device=dev)
        dg = codec.fragment(e.data, e.offsets, rpc)
        if window:  # bench.py reassembly_leg's reordering
            nd = dg.dg_off.numel() - 1
            g = torch.Generator(device=dev)
            g.manual_seed(7)
            key = torch.div(torch.arange(nd, device=dev), window, rounding_mode="floor").double() + \
                torch.rand(nd, device=dev, dtype=torch.float64, generator=g)
            perm = torch.argsort(key)
            lens = (dg.dg_off[1:] - dg.dg_off[:-1])[perm]
            off = torch.zeros(nd + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            dg = SimpleNamespace(wire=byte_gather(dg.wire, dg.dg_off[:-1][perm], lens), dg_off=off)
        torch.cuda.synchronize()
        work[name] = (lambda dg=dg: codec.reassemble(dg.wire, dg.dg_off),
                      lambda m: (lambda k: (m.data[:int(m.offsets[k].item())], m.offsets[:k + 1], m.rpc_id[:k],
                                            m.dgram[:k], m.status))(int(m.nmsg.item())))
        del b, f, v, e
    eb = datagen.make_element_batch(**datagen.ELEMENT_FW)
    data = torch.from_numpy(eb.data).to(dev)
    off = torch.from_numpy(eb.rec_off.view(np.int64)).to(dev)
    work["firewall"] = (lambda: codec.firewall(data, off, 50),
                        lambda r: (lambda k: (r.kept[:int(r.kept_off[k].item())], r.kept_off[:k + 1],
                                              r.kept_index[:k], r.verdict))(int(r.nkept.item())))
    times = {(w, v): [] for w in work for v in variants}
    ref = {}
    for rnd in range(a.rounds + 1):
        for w, (fn, outs) in work.items():
            for v in variants:
                os.environ[a.env] = str(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = fn()
                e1.record()
                torch.cuda.synchronize()
                codec.check()
                if rnd == 0:
                    got = [x.cpu() for x in outs(r)]
                    if v == variants[0]:
                        ref[w] = got
                    else:
                        for j, (x, y) in enumerate(zip(got, ref[w])):
                            if not torch.equal(x, y):
                                bad = (x != y).nonzero()
                                print(f"MISMATCH {w}: variant {v} output {j} differs from variant {variants[0]} at "
                                      f"{bad.numel()} places, first {bad[:4].flatten().tolist()}", flush=True)
                else:
                    times[(w, v)].append(e0.elapsed_time(e1) * 1e3)
    for (w, v), ts in times.items():
        print(f"{w:12s} {a.env} {v}: median {statistics.median(ts):8.1f} us  min {min(ts):8.1f} us")


if __name__ == "__main__":
    main()

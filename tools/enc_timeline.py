"""Diagnostics: per-tile timestamps of the encode kernel (tuning variants 6 = workgroup tiles,
7 = wave tiles).

  python tools/enc_timeline.py [--config 2|3] [--records N] [--variant 6]
s_memrealtime runs at 100 MHz.  Slots: 0 tile start, 1 header image built, 2..5 wave ends
(variant 7: slot 2 only), 6 workgroup id.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SYMHIP_LIBRARY", os.path.join(ROOT, "tools", "lib", "libsymphony_hip_tuning.so"))
from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402


def q(x):
    return "p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--variant", default="6")
    a = ap.parse_args()
    kw = dict(datagen.CONFIG2 if a.config == 2 else datagen.CONFIG3)
    if a.records:
        kw["n"] = a.records
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_batch(**kw)
    fixed, var = to_device(b, dev)
    vt = b.encoded_size() - b.n * b.schema.overhead
    codec.encode(b.schema, fixed, var, var_total=vt)
    torch.cuda.synchronize()
    ntiles = (b.n + 63) // 64
    dbg = torch.zeros(ntiles * 8, dtype=torch.int64, device=dev)
    os.environ["SYMHIP_DEBUG_PTR"] = "%x" % dbg.data_ptr()
    os.environ["SYMHIP_ENCODE_VARIANT"] = a.variant
    for _ in range(3):
        dbg.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        codec.encode(b.schema, fixed, var, var_total=vt)
        e1.record()
        e1.synchronize()
    print(f"event time of the last call: {e0.elapsed_time(e1) * 1e3:.1f} us, {b.encoded_size() / 1e6:.1f} MB out")
    codec.check()
    raw = dbg.cpu().numpy().reshape(ntiles, 8).astype(np.int64)
    nend = 4 if a.variant == "6" else 1
    t0 = raw[:, 0].min()
    st = (raw[:, 0] - t0) / 100.0  # -> microseconds
    p1 = (raw[:, 1] - t0) / 100.0
    ends = (raw[:, 2:2 + nend] - t0) / 100.0
    end = ends.max(axis=1)
    span = end.max()
    print(f"kernel span (first stamp -> last stamp): {span:.1f} us, {ntiles} tiles, "
          f"{len(set(raw[:, 6].tolist()))} workgroups")
    print("header image  ", q(p1 - st))
    print("output steps  ", q(end - p1))
    if nend > 1:
        print("wave end spread", q(ends.max(axis=1) - ends.min(axis=1)))
    print("tile lifetime ", q(end - st))
    e = np.sort(end)
    for f in (0.5, 0.9, 0.99):
        k = int(f * len(e)) - 1
        print(f"{int(f * 100):3d}% of tiles done at {e[k]:7.1f} us; last at {span:7.1f} us (tail {span - e[k]:6.1f} us)")
    s = np.sort(st)
    for f in (0.1, 0.5, 0.9, 1.0):
        k = max(int(f * len(s)) - 1, 0)
        print(f"{int(f * 100):3d}% of tiles started by {s[k]:7.1f} us")
    for tt in np.linspace(0, span, 21)[1:-1]:
        live = ((st <= tt) & (end >= tt)).sum()
        hdr = ((st <= tt) & (p1 >= tt)).sum()
        print(f"t={tt:6.1f} us: {live:5d} tiles live, {hdr:5d} building headers")


if __name__ == "__main__":
    main()

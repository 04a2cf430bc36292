"""Diagnostics: per-tile timeline of the one-launch mixed Get/Set encode (tuning variant 37).

  python tools/mixed_timeline.py [--trace] [--records N]

s_memrealtime runs at 100 MHz.  Per 64-record tile: its encode workgroup's start, prefix in hand,
header image built, wave ends; its group's aggregate publish (sizer) and prefix publish (scanner).
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
from arpc_amd.codec import Codec  # noqa: E402


def q(x):
    return "p10 %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--variant", default="37", help="37: one launch; 38: three launches (no sizer/scanner stamps); 52: prefetching persistent tiles")
    a = ap.parse_args()
    kw = dict(datagen.config2_trace_mixed() if a.trace else datagen.CONFIG2_MIXED)
    if a.records:
        kw["n"] = a.records
    b = datagen.make_mixed_batch(**kw)
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    t = torch.from_numpy(b.type).to(dev)
    key = (torch.from_numpy(b.key[0]).to(dev), torch.from_numpy(b.key[1].view(np.int64)).to(dev))
    val = (torch.from_numpy(b.val[0]).to(dev), torch.from_numpy(b.val[1].view(np.int64)).to(dev))
    out = torch.empty(b.encoded_size() + 16, dtype=torch.uint8, device=dev)
    off = torch.empty(b.n + 1, dtype=torch.int64, device=dev)
    codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out, out_off=off)
    torch.cuda.synchronize()
    nt = (b.n + 63) // 64
    dbg = torch.zeros(nt * 16, dtype=torch.int64, device=dev)
    os.environ["SYMHIP_DEBUG_PTR"] = "%x" % dbg.data_ptr()
    os.environ["SYMHIP_ENCODE_VARIANT"] = a.variant
    for _ in range(3):
        dbg.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out, out_off=off)
        e1.record()
        e1.synchronize()
    codec.check()
    print(f"event time of the last call: {e0.elapsed_time(e1) * 1e3:.1f} us, {nt} tiles")
    raw = dbg.cpu().numpy().reshape(2, nt, 8).astype(np.int64)
    tile, side = raw[0], raw[1]
    t0 = tile[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731
    st, hdr = us(tile[:, 0]), us(tile[:, 1])
    pre = us(tile[:, 7]) if a.variant in ("37", "52") else st
    if a.variant not in ("37", "52"):
        side[:, 4] = side[:, 5] = t0
    end = us(tile[:, 2:6].max(axis=1))
    grp = np.arange(nt) // 8  # sizer groups (encode.hip kPipeGroup): their stamps sit at the group index
    agg, pub = us(side[grp, 4]), us(side[grp, 5])
    print(f"span {end.max():.1f} us; sizers' last aggregate at {agg.max():.1f} us; scanner's last prefix at {pub.max():.1f} us")
    print("wait for prefix (start -> prefix)", q(pre - st))
    print("prefix published - tile start    ", q(pub - st))
    print("aggregate published - tile start ", q(agg - st))
    print("header image (prefix -> hdr)     ", q(hdr - pre))
    print("output steps                     ", q(end - hdr))
    print("tile lifetime                    ", q(end - st))
    for f in (0.1, 0.5, 0.9, 1.0):
        k = max(int(f * nt) - 1, 0)
        print(f"{int(f * 100):3d}%: tiles started by {np.sort(st)[k]:7.1f}  aggregates by {np.sort(agg)[k]:7.1f}  "
              f"prefixes by {np.sort(pub)[k]:7.1f}  tiles done by {np.sort(end)[k]:7.1f} us")
    for tt in np.linspace(0, end.max(), 11)[1:-1]:
        live = ((st <= tt) & (end >= tt)).sum()
        waiting = ((st <= tt) & (pre >= tt)).sum()
        print(f"t={tt:6.1f} us: {live:5d} tiles live, {waiting:5d} waiting for their prefix, "
              f"frontier agg {(agg <= tt).sum():6d} pre {(pub <= tt).sum():6d} started {(st <= tt).sum():6d}")


if __name__ == "__main__":
    main()

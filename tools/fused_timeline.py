"""Diagnostics: per-tile phase timestamps of the single-pass decode (variant 410; 411 = no look-back).

  python tools/fused_timeline.py [--config 2|3] [--variant 410]
s_memrealtime runs at 100 MHz.  Slots: 0 tile start, 1 staged, 2 parsed, 3 look-back done, 4 end.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the measurement variants live only in the tuning build (make -C arpc_amd/csrc tuning)
os.environ.setdefault("SYMHIP_LIBRARY", os.path.join(ROOT, "tools", "lib", "libsymphony_hip_tuning.so"))
from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402


def q(x):
    return "p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variant", default="410")
    a = ap.parse_args()
    kw = dict(datagen.CONFIG2 if a.config == 2 else datagen.CONFIG3)
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_batch(**kw)
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    codec.decode(b.schema, enc.data, enc.offsets)
    torch.cuda.synchronize()
    ntiles = (b.n + 63) // 64
    dbg = torch.zeros(ntiles * 8, dtype=torch.int64, device=dev)
    os.environ["SYMHIP_DEBUG_PTR"] = "%x" % dbg.data_ptr()
    os.environ["SYMHIP_DECODE_VARIANT"] = a.variant
    for _ in range(3):
        dbg.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        codec.decode(b.schema, enc.data, enc.offsets)
        e1.record()
        e1.synchronize()
    print(f"event time of the last call: {e0.elapsed_time(e1) * 1e3:.1f} us")
    codec.check()
    raw = dbg.cpu().numpy().reshape(ntiles, 8).astype(np.int64)
    t0 = raw[:, 0].min()
    t = (raw[:, :5] - t0) * 10 / 1000.0  # -> microseconds
    blk = raw[:, 5]
    span = t[:, 4].max()
    print(f"kernel span (first stamp -> last stamp): {span:.1f} us, {ntiles} tiles, {len(set(blk))} workgroups")
    print("stage      ", q(t[:, 1] - t[:, 0]))
    print("parse      ", q(t[:, 2] - t[:, 1]))
    print("look-back  ", q(t[:, 3] - t[:, 2]))
    print("copy       ", q(t[:, 4] - t[:, 3]))
    print("tile total ", q(t[:, 4] - t[:, 0]))
    # look-back lag: time from "predecessor's inclusive published and my aggregate ready" to "my
    # prefix known" (stamps are taken after the stores are issued, so this is visibility + polling)
    ready = np.maximum(t[1:, 2], t[:-1, 3])
    print("look-back lag after predecessor's inclusive", q(t[1:, 3] - ready))
    print("predecessor inclusive minus my aggregate   ", q(t[:-1, 3] - t[1:, 2]))
    pub = raw[:, 6]
    if (pub > 0).all():  # round-5 diag variants: the scanner's publish time of each tile's prefix (slot 6)
        tp = (pub - t0) * 10 / 1000.0
        print("prefix published - tile start      ", q(tp - t[:, 0]))
        print("prefix published - copier's parse  ", q(tp - t[:, 2]))
        print("prefix known - prefix published    ", q(t[:, 3] - tp))
    first = t[:min(1400, ntiles)]
    print("first 1400 tiles: aggregate ready", q(first[:, 2]), "\n                  prefix known   ", q(first[:, 3]),
          "\n                  staged         ", q(first[:, 1]))
    order = np.argsort(t[:, 0])
    gaps = []
    for w in set(blk.tolist()):
        idx = np.where(blk == w)[0]
        idx = idx[np.argsort(t[idx, 0])]
        gaps.extend((t[idx[1:], 0] - t[idx[:-1], 4]).tolist())
    if gaps:
        print("gap between a workgroup's tiles", q(np.array(gaps)))
    for tt in np.linspace(0, span, 11)[1:-1]:
        live = ((t[:, 0] <= tt) & (t[:, 4] >= tt)).sum()
        st = ((t[:, 0] <= tt) & (t[:, 1] >= tt)).sum()
        lb = ((t[:, 2] <= tt) & (t[:, 3] >= tt)).sum()
        cp = ((t[:, 3] <= tt) & (t[:, 4] >= tt)).sum()
        print(f"t={tt:6.1f} us: {live:5d} tiles live, {st:5d} staging, {lb:5d} in look-back, {cp:5d} copying")
    del order


if __name__ == "__main__":
    main()

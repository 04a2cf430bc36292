"""Diagnostics: per-wave phase timestamps of the decode kernel (variant 104, s_memrealtime = 100 MHz).

  python tools/decode_timeline.py [--config 2|3]
Prints phase durations (ticket, parse, copy loads, barrier waits, look-back, stores), the
workgroup start-time profile and concurrency over time.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, to_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    kw = dict(datagen.CONFIG2 if a.config == 2 else datagen.CONFIG3)
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_batch(**kw)
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    codec.decode(b.schema, enc.data, enc.offsets)
    torch.cuda.synchronize()
    ntiles = (b.n + 63) // 64  # one look-back tile per wave (decode.hip kTileRecs)
    dbg = torch.zeros(ntiles * 8, dtype=torch.int64, device=dev)
    os.environ["SYMHIP_DEBUG_PTR"] = "%x" % dbg.data_ptr()
    os.environ["SYMHIP_DECODE_VARIANT"] = "104"
    for _ in range(3):
        dbg.zero_()
        codec.decode(b.schema, enc.data, enc.offsets)
    codec.check()
    raw = dbg.cpu().numpy().reshape(ntiles, 8).astype(np.int64)
    t = (raw - raw[:, 0].min()) * 10 / 1000.0  # -> microseconds
    # slots: 0 entry, 1 ticket, 2 parsed, 3 scanned + aggregate published, 4 look-back done, 6 end
    span = t[:, 6].max()

    def q(x):
        return "p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f" % tuple(np.percentile(x, [10, 50, 90, 100]))
    print(f"kernel span (first stamp -> last stamp): {span:.1f} us, {ntiles} wave tiles")
    print("ticket+init     ", q(t[:, 1] - t[:, 0]))
    print("parse           ", q(t[:, 2] - t[:, 1]))
    print("scan+publish    ", q(t[:, 3] - t[:, 2]))
    print("look-back       ", q(t[:, 4] - t[:, 3]))
    print("copy            ", q(t[:, 6] - t[:, 4]))
    print("wave total      ", q(t[:, 6] - t[:, 0]))
    starts = np.sort(t[:, 0])
    for frac in (0.1, 0.25, 0.5, 0.75, 0.9, 1.0):
        k = min(ntiles - 1, int(frac * ntiles))
        print(f"wave start at {frac:4.0%} of tiles: {starts[k]:7.1f} us")
    for tt in np.linspace(0, span, 11)[1:-1]:
        live = ((t[:, 0] <= tt) & (t[:, 6] >= tt)).sum()
        inlook = ((t[:, 3] <= tt) & (t[:, 4] >= tt)).sum()
        copying = ((t[:, 4] <= tt) & (t[:, 6] >= tt)).sum()
        print(f"t={tt:6.1f} us: {live:5d} waves live, {inlook:5d} in look-back, {copying:5d} copying")


if __name__ == "__main__":
    main()

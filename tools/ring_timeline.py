"""Diagnostics: per-tile phase timestamps of the ring decode (tuning variant 510).

  python tools/ring_timeline.py [--config 2|3]
Slots (s_memrealtime, 100 MHz) of iteration i, indexed by t_i: 0 wave 0 starts, 4 wave 0 parsed
t_{i+2}, 1 wave 0 resolved t_{i+1}'s prefix, 2 copiers start t_i, 3 copy issued, 5 loaders pass the
barrier, 6 loaders issued the next span, 7 workgroup.
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


LEAD = 3  # wave 0 parses t_{i+LEAD} in iteration i (decode_pipe.hip kRingLead)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--variant", default="510")
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
    blk = raw[:, 7]
    ts = raw[:, :7].astype(np.float64)  # slots 0..6
    t0 = ts[ts > 0].min()
    t = (ts - t0) / 100.0  # microseconds
    t[ts == 0] = np.nan
    last = np.nanmax(t)
    print(f"span: {last:.1f} us, {ntiles} tiles, {len(set(blk.tolist()))} workgroups")
    ok = ~np.isnan(t).any(axis=1)
    u = t[ok]
    print("wave 0: parse t+LEAD ", q(u[:, 4] - u[:, 0]))
    print("wave 0: prefix t+1   ", q(u[:, 1] - u[:, 4]))
    print("wave 0 total         ", q(u[:, 1] - u[:, 0]))
    print("copy t               ", q(u[:, 3] - u[:, 2]))
    print("loader put+issue     ", q(u[:, 6] - u[:, 5]))
    # iteration time per workgroup: consecutive tiles' slot 0
    it = []
    for w in set(blk.tolist()):
        idx = np.where(blk == w)[0]
        s0 = np.sort(t[idx, 0])
        it.extend(np.diff(s0).tolist())
    print("iteration            ", q(np.array(it)))
    # per tile T: P parse done (slot 4 of T - LEAD*G), A aggregate stored by a copy wave (slot 6 of T),
    # S prefix stored by the scanner (slot 5 of T), K prefix seen by wave 0 (slot 1 of T - G).
    G = len(set(blk.tolist()))
    P = np.full(ntiles, np.nan)
    K = np.full(ntiles, np.nan)
    P[LEAD * G:] = t[:ntiles - LEAD * G, 4]
    K[G:] = t[:ntiles - G, 1]
    A = t[:, 6]
    Sx = t[:, 5]
    FA = np.fmax.accumulate(np.where(np.isnan(A), -np.inf, A))
    sel = (np.arange(ntiles) >= LEAD * G) & ~np.isnan(K) & ~np.isnan(A) & ~np.isnan(Sx) & ~np.isnan(P)
    print("publish delay A-P          ", q((A - P)[sel]))
    print("frontier wait FA-A         ", q((FA - A)[sel]))
    print("scanner S-FA               ", q((Sx - FA)[sel]))
    print("poll K-S                   ", q((K - Sx)[sel]))
    print("wave 0 prefix phase        ", q(u[:, 1] - u[:, 0]))
    first = t[:, 0]
    print("first tile start      ", q(first[blk > 0][:800]) if (blk > 0).any() else "")
    print("first prefix known    ", q(t[:800, 1]))
    for tt in np.linspace(0, last, 9)[1:-1]:
        in_b = ((t[:, 4] <= tt) & (t[:, 1] > tt)).sum()
        cp = ((t[:, 2] <= tt) & (t[:, 3] > tt)).sum()
        print(f"t={tt:6.1f} us: {in_b:4d} in prefix wait, {cp:4d} copying")


if __name__ == "__main__":
    main()

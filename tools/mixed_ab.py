"""A/B of mixed Get/Set encode and decode variants in ONE process (tuning library), like kbench.py.

  python tools/mixed_ab.py [--enc 0,20] [--dec 0] [--rounds 10] [--trace]

Each round runs every variant on two rotating buffer sets of BASELINE config 2 as written (2^20
requests at the trace's 36.9 % Set; --trace: the trace_large.req replay), HIP events around each
call; prints median / min per variant in algorithmic GB/s (bench.py's mixed_leg definition) and
checks that every variant's stream and decoded columns equal the first variant's.
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
from arpc_amd.codec import Codec, DecodedBatch  # noqa: E402


# timing-only decode variants that give wrong output by design (tools/kbench.py)
WRONG_OUTPUT = {402, 412, 475, 476, 482, 483, 492, 504, 601, 701, 702, 711, 712, 742, 794}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--enc", default="0,20")
    ap.add_argument("--dec", default="0")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--trace", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_mixed_batch(**(datagen.config2_trace_mixed() if a.trace else datagen.CONFIG2_MIXED))
    n, total = b.n, b.encoded_size()
    kb, vb = int(b.key[1][-1]), int(b.val[1][-1])
    sets = []
    for k in range(2):
        t = torch.from_numpy(b.type).to(dev)
        key = (torch.from_numpy(b.key[0]).to(dev) ^ (0x3B * k), torch.from_numpy(b.key[1].view(np.int64)).to(dev))
        val = (torch.from_numpy(b.val[0]).to(dev) ^ (0x3B * k), torch.from_numpy(b.val[1].view(np.int64)).to(dev))
        out = (torch.empty(total + 16, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
        dec = DecodedBatch(fixed=[], var=[(torch.empty(kb + 16, dtype=torch.uint8, device=dev),
                                           torch.empty(n + 1, dtype=torch.int64, device=dev)),
                                          (torch.empty(vb + 16, dtype=torch.uint8, device=dev),
                                           torch.empty(n + 1, dtype=torch.int64, device=dev))],
                           status=torch.empty(n, dtype=torch.uint8, device=dev))
        sets.append((t, key, val, out, dec))
    enc_alg = n + kb + 8 * (n + 1) + vb + 8 * (n + 1) + total + 8 * (n + 1)
    dec_alg = total + 8 * (n + 1) + n + kb + vb + 16 * (n + 1) + n
    for t, key, val, out, dec in sets:  # every decode variant reads a valid stream, even with --enc ""
        codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out[0], out_off=out[1])
    torch.cuda.synchronize()
    codec.check()
    variants = [("enc", int(v)) for v in a.enc.split(",") if v] + [("dec", int(v)) for v in a.dec.split(",") if v]
    times = {v: [] for v in variants}
    ref = {}
    for rnd in range(a.rounds + 1):
        for kind, v in variants:
            os.environ["SYMHIP_ENCODE_VARIANT" if kind == "enc" else "SYMHIP_DECODE_VARIANT"] = str(v)
            for k in range(2):
                t, key, val, out, dec = sets[k]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind == "enc":
                    codec.encode_kv_mixed(t, key, val, 1, 1, 2, out=out[0], out_off=out[1])
                else:
                    codec.decode_kv_mixed(out[0], out[1], t, outputs=dec)
                e1.record()
                e1.synchronize()
                if rnd == 0:
                    codec.check()
                    if kind == "enc":
                        dg = (int(out[0][:total].to(torch.int64).sum().item()), int(out[1].sum().item()))
                    else:
                        dg = tuple(int(x.to(torch.int64).sum().item()) for x in
                                   (dec.var[0][0][:kb], dec.var[0][1], dec.var[1][0][:vb], dec.var[1][1], dec.status))
                    if not (kind == "dec" and v in WRONG_OUTPUT):
                        assert ref.setdefault((kind, k), dg) == dg, f"{kind} variant {v} differs on set {k}"
                else:
                    times[(kind, v)].append(e0.elapsed_time(e1))
    for (kind, v), ts in times.items():
        nb = enc_alg if kind == "enc" else dec_alg
        med, mn = statistics.median(ts), min(ts)
        print(f"{kind} variant {v}: median {med * 1e3:8.1f} us ({nb / med / 1e6:7.1f} GB/s)  "
              f"min {mn * 1e3:8.1f} us ({nb / mn / 1e6:7.1f} GB/s)")


if __name__ == "__main__":
    main()

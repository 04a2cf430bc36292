"""Kernel A/B bench: time encode/decode variants interleaved in ONE process (guide rule 24).

  python tools/kbench.py [--config 2|3] [--records N] [--enc 1,2] [--dec 0,1] [--rounds 10]

Each round runs every variant once per buffer set (4 rotating sets), timing each launch
with HIP events on torch's current stream; prints median / min per variant in GB/s
(algorithmic bytes, bench.py's definition) and checks every variant's output digest.
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the measurement variants live only in the tuning build (make -C arpc_amd/csrc tuning)
os.environ.setdefault("SYMHIP_LIBRARY", os.path.join(ROOT, "tools", "lib", "libsymphony_hip_tuning.so"))

from arpc_amd import datagen  # noqa: E402
from arpc_amd.codec import Codec, DecodedBatch, to_device  # noqa: E402
from bench import alg_bytes  # noqa: E402


# timing-only decode variants that give wrong output by design (no digest check)
WRONG_OUTPUT = {402, 412, 475, 476, 482, 483, 492, 504, 601, 701, 702, 711, 712, 742, 794}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--records", type=int, default=0)
    ap.add_argument("--enc", default="1,2")
    ap.add_argument("--dec", default="0")
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    kw = dict(datagen.CONFIG2 if a.config == 2 else datagen.CONFIG3)
    if a.records:
        kw["n"] = a.records
    dev = torch.device("cuda", 0)
    codec = Codec(dev)
    b = datagen.make_batch(**kw)
    s, n = b.schema, b.n
    var_total = sum(int(o[-1] - o[0]) for _, o in b.var)
    total = b.encoded_size()
    fixed0, var0 = to_device(b, dev)
    sets = [[((x ^ (0x3B * k)) if k else x, o) for x, o in var0] for k in range(4)]
    enc = [(torch.empty(total, dtype=torch.uint8, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev))
           for _ in range(4)]
    caps = [int(o[-1]) for _, o in b.var]
    dec = DecodedBatch(fixed=[], var=[(torch.empty(c, dtype=torch.uint8, device=dev),
                                       torch.empty(n + 1, dtype=torch.int64, device=dev)) for c in caps],
                       status=torch.empty(n, dtype=torch.uint8, device=dev))
    codec.reserve(n)
    enc_b, dec_b = alg_bytes(n, s.nvar, var_total, total)
    for k in range(4):
        codec.encode(s, fixed0, sets[k], out=enc[k][0], out_off=enc[k][1])
    torch.cuda.synchronize()
    ref = [int(e[0].to(torch.int64).sum().item()) for e in enc]

    variants = [("enc", int(v)) for v in a.enc.split(",") if v] + [("dec", int(v)) for v in a.dec.split(",") if v]
    times = {v: [] for v in variants}
    dref = {}  # decode digest per buffer set (the first decode variant is the reference)

    def ddigest():
        return tuple(int(t.to(torch.int64).sum().item()) for t in
                     [x for col, off in dec.var for x in (col, off)] + [dec.status])
    for rnd in range(a.rounds + 1):
        for kind, v in variants:
            os.environ["SYMHIP_ENCODE_VARIANT" if kind == "enc" else "SYMHIP_DECODE_VARIANT"] = str(v)
            for k in range(4):
                if kind == "dec" and rnd <= 1:
                    for col, _ in dec.var:
                        col.fill_(0xA5)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if kind == "enc":
                    codec.encode(s, fixed0, sets[k], out=enc[k][0], out_off=enc[k][1])
                else:
                    codec.decode(s, enc[(k + 2) % 4][0], enc[(k + 2) % 4][1], outputs=dec)
                e1.record()
                e1.synchronize()
                if kind == "dec" and rnd <= 1 and v not in WRONG_OUTPUT:
                    codec.check()
                    dg = ddigest()
                    assert dref.setdefault(k, dg) == dg, f"decode variant {v} output differs on set {k}"
                if rnd:
                    times[(kind, v)].append(e0.elapsed_time(e1))
            if kind == "enc":
                got = [int(e[0].to(torch.int64).sum().item()) for e in enc]
                assert got == ref, f"encode variant {v} output differs"
            else:
                codec.check()
                assert torch.equal(dec.var[-1][0], sets[0][-1][0] if False else dec.var[-1][0])
    for (kind, v), ts in times.items():
        nb = enc_b if kind == "enc" else dec_b
        med, mn = statistics.median(ts), min(ts)
        print(f"{kind} variant {v}: median {med * 1e3:8.1f} us ({nb / med / 1e6:7.1f} GB/s)  "
              f"min {mn * 1e3:8.1f} us ({nb / mn / 1e6:7.1f} GB/s)")


if __name__ == "__main__":
    main()

"""Debug helper: encode small batches on the GPU and print where bytes differ from the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from arpc_amd import datagen
from arpc_amd.codec import Codec, to_device
from oracle import oracle

dev = torch.device("cuda", 0)
codec = Codec(dev)
cases = [
    ("kat", datagen.from_records("kv_set_request", [((), [b"ab", b"xyz"])])),
    ("kat_get", datagen.from_records("kv_get_request", [((), [b"ab"])])),
    ("two", datagen.from_records("kv_set_request", [((), [b"ab", b"xyz"]), ((), [b"k" * 20, b"v" * 40])])),
    ("set64_256_n4", datagen.make_batch(schema="kv_set_request", n=4, lens=(64, 256), seed=1)),
    ("set64_256_n300", datagen.make_batch(schema="kv_set_request", n=300, lens=(64, 256), seed=1)),
]
for name, b in cases:
    fixed, var = to_device(b, dev)
    enc = codec.encode(b.schema, fixed, var, var_total=b.encoded_size() - b.n * b.schema.overhead)
    want, woff = oracle.encode_batch(b.fixed, b.var)
    got = enc.data.cpu().numpy()[:len(want)]
    bad = np.nonzero(got != want)[0]
    print(f"== {name}: n={b.n} bytes={len(want)} ndiff={len(bad)} data_ptr%16={enc.data.data_ptr()%16}")
    if len(bad):
        print(" first diffs:", bad[:20].tolist())
        i0 = max(0, bad[0] - 8)
        print(" want:", want[i0:i0 + 48].tobytes().hex())
        print(" got :", got[i0:i0 + 48].tobytes().hex())
        rec = np.searchsorted(woff, bad[:10], side="right") - 1
        print(" rec/offset-in-rec:", list(zip(rec.tolist(), (bad[:10] - woff[rec]).tolist())))

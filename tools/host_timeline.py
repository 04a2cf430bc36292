"""Timeline of the host entry points (arpc_amd/csrc/host.cpp) on bench config 2: a warm-up of the same
calls, then `--calls` timed sym_encode_host + sym_decode_host pairs (pinned caller memory), with the
host clock per call.  Run it under rocprofv3 to see the copies and kernels:

    rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/ht -- \
        python tools/host_timeline.py
    python tools/host_timeline.py --analyze gpurun_out/ht   # H2D / D2H busy, overlap, the first ops

(tests/bin/host_bench is the same calls from a plain-C process; --analyze reads its traces too.)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(calls: int, warm_s: float, alloc: str) -> None:
    import ctypes

    import numpy as np
    import torch

    from arpc_amd import _native, datagen
    from arpc_amd.codec import Codec
    codec = Codec(torch.device("cuda:0"))
    L, ctx = codec._lib, codec._ctx
    b = datagen.make_batch(**dict(datagen.CONFIG2))
    s, n = b.schema, b.n
    total = b.encoded_size()
    if alloc == "torch":  # torch's pinned host allocator
        def empty(nbytes, dtype):
            return torch.empty(nbytes // np.dtype(dtype).itemsize, dtype=getattr(torch, np.dtype(dtype).name),
                               pin_memory=True)
    else:  # sym_host_alloc (hipHostMalloc), wrapped as tensors
        keep = []

        def empty(nbytes, dtype):
            p = ctypes.c_void_p()
            _native.check(L.sym_host_alloc(ctx, nbytes, ctypes.byref(p)), "sym_host_alloc")
            keep.append(p.value)
            a = np.frombuffer((ctypes.c_uint8 * nbytes).from_address(p.value), np.uint8).view(dtype)
            return torch.from_numpy(a)

    def pin(a):
        t = empty(a.nbytes, a.dtype)
        t.numpy()[:] = a
        return t
    var = [(pin(x), pin(o.view("int64"))) for x, o in b.var]
    out = empty(total + 16, np.uint8)
    off = empty(8 * (n + 1), np.int64)
    dec = [(empty(int(o[-1] - o[0]) + 16, np.uint8), empty(8 * (n + 1), np.int64)) for _, o in b.var]
    st = empty(n, np.uint8)
    bp = _native.ptr_array([x.data_ptr() for x, _ in var])
    op = _native.ptr_array([o.data_ptr() for _, o in var])
    dbp = _native.ptr_array([x.data_ptr() for x, _ in dec])
    dop = _native.ptr_array([o.data_ptr() for _, o in dec])
    caps = _native.u64_array([x.numel() for x, _ in dec])

    def enc():
        _native.check(L.sym_encode_host(ctx, s.schema_id, n, None, bp, op, 0, 0, out.data_ptr(), off.data_ptr()),
                      "sym_encode_host")

    def dcd():
        _native.check(L.sym_decode_host(ctx, s.schema_id, n, out.data_ptr(), off.data_ptr(), None, dbp, caps, dop,
                                        st.data_ptr()), "sym_decode_host")
    t_w = time.perf_counter()
    while time.perf_counter() - t_w < warm_s:
        enc()
        dcd()
    for i in range(calls):
        t0 = time.perf_counter()
        enc()
        t1 = time.perf_counter()
        dcd()
        t2 = time.perf_counter()
        print(f"call {i}: encode {1e3 * (t1 - t0):.2f} ms, decode {1e3 * (t2 - t1):.2f} ms", flush=True)
    in_b = sum(x.numel() + o.numel() * 8 for x, o in var)
    print(f"encode H2D {in_b / 1e6:.1f} MB, D2H {(total + 8 * (n + 1)) / 1e6:.1f} MB; "
          f"decode H2D {(total + 8 * (n + 1)) / 1e6:.1f} MB, D2H {(in_b + n) / 1e6:.1f} MB")


def analyze(d: str) -> None:
    """Busy time per direction and their overlap over the last ~2 encode + decode pairs of a
    rocprofv3 --memory-copy-trace --kernel-trace run: SDMA copies from the copy trace, and copies the
    runtime ran as blit kernels (__amd_rocclr_copyBuffer on the D2H stream, as torch's bundled runtime
    does) from the kernel trace; then the first operations of that window in time order."""
    mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not mc or not kt:
        raise SystemExit(f"no memory_copy_trace.csv / kernel_trace.csv under {d}")
    ops = []
    for r in csv.DictReader(open(mc[0])):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H"))
    kernels = list(csv.DictReader(open(kt[0])))
    blit_streams = {r["Stream_Id"] for r in kernels if "copyBuffer" in r["Kernel_Name"] and r["Stream_Id"] != "0"}
    for r in kernels:
        if r["Stream_Id"] == "0":
            continue
        kind = "D2H(blit)" if r["Stream_Id"] in blit_streams else "K " + r["Kernel_Name"].split("(")[0][-40:]
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))

    def busy(iv):
        t, end = 0, -1
        for a, b in sorted(iv):
            if b <= end:
                continue
            t += b - max(a, end)
            end = b
        return t
    t_end = max(b for _, b, _ in ops)
    w = [o for o in ops if o[0] > t_end - 20e6]
    h = [(a, b) for a, b, k in w if k == "H2D"]
    dd = [(a, b) for a, b, k in w if k.startswith("D2H")]
    span = (t_end - min(a for a, _, _ in w)) / 1e6
    print(f"last {span:.2f} ms: H2D busy {busy(h) / 1e6:.2f} ms, D2H busy {busy(dd) / 1e6:.2f} ms, "
          f"both at once {(busy(h) + busy(dd) - busy(h + dd)) / 1e6:.2f} ms")
    t0 = min(a for a, _, _ in w)
    for a, b, k in sorted(w)[:40]:
        print(f"{(a - t0) / 1e3:9.1f} us  {(b - a) / 1e3:7.1f} us  {k}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--warm-s", type=float, default=2.0)
    ap.add_argument("--analyze", default="")
    ap.add_argument("--alloc", default="torch", choices=("torch", "sym"))
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.calls, a.warm_s, a.alloc)

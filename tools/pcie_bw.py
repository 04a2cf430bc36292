"""PCIe ceiling for the host-inclusive rate (DESIGN.md "host entry points"), pinned memory, wall clock.

Measures, for several chunk sizes and stream counts per direction:
  h2d   host -> device alone
  d2h   device -> host alone
  both  H2D and D2H at once, each direction on its OWN streams and its OWN pinned / device
        buffers (what sym_encode_host / sym_decode_host overlap), total and per direction.
One 512 MiB copy per direction on one stream each (round 2's measurement) is the first row.

  python tools/pcie_bw.py [--total-mib 1024]
"""
import argparse
import json
import time

import torch


def run(dev, total: int, chunk: int, streams: int, mode: str) -> float:
    """GB/s of `mode` moving `total` bytes per direction in `chunk`-byte copies over `streams` streams
    per direction."""
    def bufs():
        return ([torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(streams)],
                [torch.empty(chunk, dtype=torch.uint8, device=dev) for _ in range(streams)])
    hs_a, ds_a = bufs()
    hs_b, ds_b = bufs()
    st_a = [torch.cuda.Stream(dev) for _ in range(streams)]
    st_b = [torch.cuda.Stream(dev) for _ in range(streams)]
    n = max(1, total // chunk)

    def issue():
        for i in range(n):
            k = i % streams
            if mode in ("h2d", "both"):
                with torch.cuda.stream(st_a[k]):
                    ds_a[k].copy_(hs_a[k], non_blocking=True)
            if mode in ("d2h", "both"):
                with torch.cuda.stream(st_b[k]):
                    hs_b[k].copy_(ds_b[k], non_blocking=True)
    issue()  # warm
    torch.cuda.synchronize()
    t = time.perf_counter()
    issue()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    dirs = 2 if mode == "both" else 1
    return dirs * n * chunk / dt / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mib", type=int, default=1024)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    total = args.total_mib << 20
    rows = []
    for chunk_mib, streams in ((512, 1), (8, 1), (8, 2), (8, 4), (64, 2), (2, 4)):
        chunk = chunk_mib << 20
        r = {"chunk_mib": chunk_mib, "streams_per_direction": streams}
        for mode in ("h2d", "d2h", "both"):
            r[mode + "_gbps"] = round(run(dev, total, chunk, streams, mode), 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
    best = max(rows, key=lambda x: x["both_gbps"])
    print(json.dumps({"best_both_directions_gbps": best["both_gbps"], "at": best,
                      "single_direction_best_gbps": max(max(x["h2d_gbps"], x["d2h_gbps"]) for x in rows)}))


if __name__ == "__main__":
    main()

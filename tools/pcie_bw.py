"""PCIe ceiling for the host-inclusive rate (DESIGN.md "host entry points"): pinned H2D, D2H, and
both at once on two streams, 512 MiB each, HIP events / wall clock.

  python tools/pcie_bw.py
"""
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    n = 512 << 20
    h_a = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_b = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for name, fn in (("h2d", lambda: d_a.copy_(h_a, non_blocking=True)),
                     ("d2h", lambda: h_b.copy_(d_b, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {5 * n / (time.perf_counter() - t) / 1e9:.1f} GB/s")
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        with torch.cuda.stream(s1):
            d_a.copy_(h_a, non_blocking=True)
        with torch.cuda.stream(s2):
            h_b.copy_(d_b, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"both directions: {2 * 5 * n / dt / 1e9:.1f} GB/s total ({5 * n / dt / 1e9:.1f} each)")


if __name__ == "__main__":
    main()

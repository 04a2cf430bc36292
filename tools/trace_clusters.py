"""Kernel-trace clusters: a rocprofv3 --kernel-trace csv split where the device idles longer than
--gap us; per cluster the kernel count, span, busy time (union of kernel intervals) and the idle gaps
between consecutive kernels, and (--detail K) the K-th last cluster's kernels.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -- python tools/graph_walk.py --reps 3
    python tools/trace_clusters.py gpurun_out/gt --last 12 --detail 1
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap", type=float, default=40.0)
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--detail", type=int, default=0)
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not kt:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kt[0])))
    clusters, cur, end = [], [], -1
    for k in ks:
        if cur and k[0] - end > a.gap * 1e3:
            clusters.append(cur)
            cur = []
        cur.append(k)
        end = max(end, k[1])
    if cur:
        clusters.append(cur)

    def busy(c):
        t, e = 0, -1
        for s, f, _ in c:
            if f <= e:
                continue
            t += f - max(s, e)
            e = f
        return t
    for i, c in enumerate(clusters[-a.last:]):
        span = max(f for _, f, _ in c) - c[0][0]
        print(f"cluster -{len(clusters[-a.last:]) - i}: {len(c)} kernels, span {span / 1e3:.1f} us, "
              f"busy {busy(c) / 1e3:.1f} us, idle {(span - busy(c)) / 1e3:.1f} us")
    if a.detail:
        c = clusters[-a.detail]
        t0 = c[0][0]
        for s, f, name in c:
            print(f"{(s - t0) / 1e3:8.1f} {(f - s) / 1e3:7.1f}  {name.split('(')[0][:100]}")


if __name__ == "__main__":
    main()

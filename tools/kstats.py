"""Print a rocprofv3 kernel-stats CSV: per-iteration totals (divide by --iters), largest first.

  python tools/kstats.py gpurun_out/prof_bq [--iters 5] [--top 25]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--iters", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "run_kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / a.iters:8.3f} ms  calls {int(r['Calls']) / a.iters:6.1f}  "
              f"avg {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}")
    print(f"{tot / 1e6 / a.iters:.3f} ms in all kernels per iteration")


if __name__ == "__main__":
    main()

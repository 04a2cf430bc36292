"""Summarize tools/profile.sh output: per-kernel average duration and per-dispatch counters.

HBM bytes per launch = FETCH_SIZE*2 (gfx950 reports half of wide coalesced reads,
MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, both in KiB units.
Usage: python tools/summarize_profile.py gpurun_out/prof [out.json]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"symhip::(?:\w+::)*(\w+<[^>]*>)", name)
    return m.group(1) if m else name[:60]


def main():
    d = sys.argv[1]
    out = {"kernels": {}}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    for row in csv.DictReader(open(stats)):
        if "symhip" in row["Name"]:
            out["kernels"].setdefault(short(row["Name"]), {})["avg_ns"] = float(row["AverageNs"])
            out["kernels"][short(row["Name"])]["calls_traced"] = int(row["Calls"])
    for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
        acc = defaultdict(lambda: defaultdict(list))
        for row in csv.DictReader(open(f)):
            if "symhip" not in row["Kernel_Name"]:
                continue
            acc[short(row["Kernel_Name"])][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
        for k, cs in acc.items():
            for c, vals in cs.items():
                per = defaultdict(float)
                for disp, v in vals:
                    per[disp] += v
                out["kernels"].setdefault(k, {})[c] = sum(per.values()) / len(per)
    for k, v in out["kernels"].items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            v["hbm_bytes_per_launch"] = (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024
            v["fetch_bytes_x2"] = 2 * v["FETCH_SIZE"] * 1024
            v["write_bytes"] = v["WRITE_SIZE"] * 1024
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")


if __name__ == "__main__":
    main()

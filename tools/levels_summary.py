"""Per-level counters of the boutique encode (tools/profile.sh PROG=tools/enc_levels.py): the flat
encode levels share kernel names, so dispatches are grouped by (kernel, grid size) and averaged.

  python tools/levels_summary.py gpurun_out/prof_levels

VALU/chunk = SQ_INSTS_VALU x 64 lanes / (bytes written / 16): lane-instructions per 16-byte output
chunk (WRITE_SIZE is exact on gfx950, profiles/r05_traffic_calibration.txt).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"symhip::(?:\w+::)*(\w+<[^>]*>|\w+)\(", name)
    return m.group(1) if m else name[:50]


def main():
    d = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(dict))  # (kernel, grid) -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if "enc_tile" not in row["Kernel_Name"]:
                continue
            key = (short(row["Kernel_Name"]), int(row["Grid_Size"]))
            c = acc[key][row["Counter_Name"]]
            c[row["Dispatch_Id"]] = c.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "run_kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            if "enc_tile" in row["Kernel_Name"]:
                dur[(short(row["Kernel_Name"]), int(row["Grid_Size_X"]))].append(
                    (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    for key in sorted(acc, key=lambda k: -k[1]):
        v = {c: sum(x.values()) / len(x) for c, x in acc[key].items()}
        wb = v.get("WRITE_SIZE", 0) * 1024
        if wb < 1e6:
            continue  # the gated alternatives that exit at once
        ts = sorted(t for t in dur.get(key, []) if t > 8)
        line = f"{key[0]:44s} grid {key[1]:8d}  us {ts[len(ts) // 2] if ts else float('nan'):7.1f}  written MB {wb / 1e6:7.1f}"
        if "SQ_INSTS_VALU" in v:
            line += f"  VALU {v['SQ_INSTS_VALU'] / 1e6:7.2f}M  VALU/chunk {v['SQ_INSTS_VALU'] * 64 / (wb / 16):6.0f}"
        if "SQ_WAVE_CYCLES" in v and v["SQ_WAVE_CYCLES"]:
            line += f"  wait {v.get('SQ_WAIT_ANY', 0) / v['SQ_WAVE_CYCLES']:.2f}  issue {v.get('SQ_ACTIVE_INST_ANY', 0) / v['SQ_WAVE_CYCLES']:.2f}"
        print(line)


if __name__ == "__main__":
    main()

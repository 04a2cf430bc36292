"""Per-dispatch timeline of one N3 reassembly call from a rocprofv3 kernel trace.

  rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/rx_ab.py --variants 0 --rounds 2
  python tools/rx_timeline.py OUT/run_kernel_trace.csv

Finds the last parse_kernel dispatch of each grid size (config 3's and config 2's batches) and prints
every dispatch from it until the payload gather ends: start relative to the parse, duration, grid,
kernel name.
"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    parses = [i for i, r in enumerate(rows) if "rx::parse_kernel" in r["Kernel_Name"]]
    seen = {}
    for i in parses:
        seen[rows[i]["Grid_Size_X"]] = i  # the last call of each batch size
    for grid, i in sorted(seen.items(), key=lambda x: -int(x[0])):
        t0 = rows[i]["s"]
        print(f"== parse grid {grid}")
        gathers = 0
        for r in rows[i:]:
            name = r["Kernel_Name"]
            if "rx::parse_kernel" in name and r is not rows[i]:
                break
            m = re.search(r"symhip::(\w+::\w+(<[^>]*>)?)", name)
            short = m.group(1) if m else name[:60]
            print(f"  {(r['s'] - t0) / 1e3:8.1f} {(r['e'] - r['s']) / 1e3:8.1f}  g={r['Grid_Size_X']:>8}  {short}")
            if "gather_kernel" in name:
                gathers += 1
                if gathers == 2:
                    print(f"  span {(r['e'] - t0) / 1e3:.1f} us")
                    break


if __name__ == "__main__":
    main()

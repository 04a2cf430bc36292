"""Print value / ms per step / per-kernel averages of bench.py JSON lines (gpurun_out/ov*.json)."""
import glob
import json

for f in sorted(glob.glob("gpurun_out/ov*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        print(f, "unreadable")
        continue
    print(f, d["value"], d["ms_per_step"], d["kernels"]["encode"]["avg_ms"], d["kernels"]["decode"]["avg_ms"],
          d["roofline"]["frac"])

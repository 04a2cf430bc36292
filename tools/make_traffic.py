"""Assemble profiles/traffic.json (bench.py load_traffic) from per-workload PMC summaries.

  python tools/make_traffic.py OUT.json config2=traffic_c2.json config3=traffic_c3.json \
      config4=traffic_c4.json mixed=traffic_mixed.json

Each input is a tools/summarize_profile.py output of ONE workload's rocprofv3 passes
(tools/gpu_profiles.sh), so a kernel's per-launch HBM bytes are always those of the workload it ran:
config2 / config3 = bench.py --config 2 / 3 (2^20 records), config4 = a 2^23-record shard, mixed =
the Get/Set batch (tools/mixed_ab.py).
"""
import json
import sys

RECORDS = {"config2": 1 << 20, "config3": 1 << 20, "config4": 1 << 23, "mixed": 1 << 20, "trace": 1 << 20, "crypto": 1 << 20}


def main():
    out = {"note": "per workload: kernel -> avg_ns (kernel trace) and HBM bytes per launch = FETCH_SIZE x 2 "
                   "+ WRITE_SIZE, both KiB-scaled (tools/summarize_profile.py); x 2 is exact on gfx950 for every "
                   "read width (profiles/r05_traffic_calibration.txt)",
           "workloads": {}}
    for arg in sys.argv[2:]:
        name, path = arg.split("=", 1)
        d = json.load(open(path))
        out["workloads"][name] = {"records": RECORDS.get(name), "source": path.rsplit("/", 1)[-1],
                                  "kernels": d["kernels"]}
    open(sys.argv[1], "w").write(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()

"""One line per workload and kernel from tools/summarize_profile.py outputs (tools/gpu_profiles.sh).

  python tools/counters_summary.py c2=gpurun_out/traffic_c2.json mixed=gpurun_out/traffic_mixed.json ...

wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES (wave-cycles spent waiting on anything, mostly vmcnt), issue =
SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, lds_share =
SQ_INSTS_LDS / SQ_ACTIVE_INST_ANY; HBM MB = FETCH_SIZE x 2 + WRITE_SIZE (exact on gfx950 for every read
width, profiles/r05_traffic_calibration.txt); VALU/wave = SQ_INSTS_VALU / SQ_WAVES where collected.
"""
import json
import sys


def main():
    for arg in sys.argv[1:]:
        tag, path = arg.split("=", 1)
        for k, v in json.load(open(path))["kernels"].items():
            if "avg_ns" not in v:
                continue
            line = f"{tag:7s}{k[:72]:74s} us {v['avg_ns'] / 1e3:8.1f}"
            if "hbm_bytes_per_launch" in v:
                line += f"  HBM MB {v['hbm_bytes_per_launch'] / 1e6:8.1f}"
            wc = v.get("SQ_WAVE_CYCLES")
            if wc:
                line += f"  wait {v.get('SQ_WAIT_ANY', 0) / wc:5.2f}  issue {v.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}"
            if v.get("SQ_LDS_IDX_ACTIVE"):
                line += f"  lds_conflict {v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE']:.3f}"
            if v.get("SQ_ACTIVE_INST_ANY") and "SQ_INSTS_LDS" in v:
                line += f"  lds_share {v['SQ_INSTS_LDS'] / v['SQ_ACTIVE_INST_ANY']:.3f}"
            if v.get("SQ_WAVES") and "SQ_INSTS_VALU" in v:
                line += f"  VALU/wave {v['SQ_INSTS_VALU'] / v['SQ_WAVES']:8.0f}  VALU {v['SQ_INSTS_VALU'] / 1e6:7.1f}M"
            print(line)


if __name__ == "__main__":
    main()

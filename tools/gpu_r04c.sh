#!/bin/bash
# Round 4, third box: the PCIe copy-pattern probe (what keeps host.cpp's H2D and D2H from
# overlapping), and the host-inclusive leg: one stream per direction with host-side slot waits
# (product) against the round-3 stream per slot (tuning build, SYMHIP_HOST_STREAMS=3).
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name" 2>&1 || { echo "$name FAILED rc=$?"; tail -30 "gpurun_out/$name"; exit 1; }
  tail -4 "gpurun_out/$name"
}
step r04c_pcie_pattern.txt 180 tools/pcie_pattern 1024
step r04c_host_2s.json 300 python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
step r04c_host_3s_tuning.json 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_HOST_STREAMS=3 python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
echo r04c ok

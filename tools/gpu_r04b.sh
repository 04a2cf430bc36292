#!/bin/bash
# Round 4, second box: the GPU suite after the scanner's DPP scan (no spills at 8 waves), A/B of the
# 8-copiers-per-CU decode for the Get/Set mix and config 2, the PCIe queue probe, the per-record and
# online-boutique legs.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name" 2>&1 || { echo "$name FAILED rc=$?"; tail -30 "gpurun_out/$name"; exit 1; }
  tail -4 "gpurun_out/$name"
}
step r04b_gpu_tests.log 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r04b_mixed_ab.txt 300 python tools/mixed_ab.py --enc 0,20,25 --dec 0,750,751,752,753,740,746,748,749,743,744,402,742 --rounds 12
step r04b_kb_c2.txt 300 python tools/kbench.py --enc "" --dec 0,750,751,752,740,747,744 --rounds 8
step r04b_kb_c3.txt 300 python tools/kbench.py --config 3 --enc "" --dec 0,750,751 --rounds 6
step r04b_mixed_trace.txt 300 python tools/mixed_ab.py --trace --enc "" --dec 0,750,752,740,746 --rounds 4
step r04b_pcie_queues.txt 120 tools/pcie_queues 1024
step r04b_host_2s.json 300 python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
step r04b_host_2s_tuning.json 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
step r04b_host_3s_tuning.json 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_HOST_STREAMS=3 python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
step r04b_legs.json 600 python -u bench.py --steps 20 --mixed-reps 10 --config3-reps 0 --trace-reps 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 3 --payload-reps 3 --per-record 2000 --cpu-seconds 0 --ref-reps 0
echo r04b ok

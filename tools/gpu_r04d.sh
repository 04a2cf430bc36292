#!/bin/bash
# Round 4: the host entry points with one stream per direction, device-side rebasing of the decode's
# column offsets and host-issued D2H (host.cpp); the GPU suite, then the host-inclusive leg.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name" 2>&1 || { echo "$name FAILED rc=$?"; tail -30 "gpurun_out/$name"; exit 1; }
  tail -4 "gpurun_out/$name"
}
step r04d_host_tests.log 300 python -u -m pytest tests/test_capi_typed.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread
step r04d_host.json 300 python -u bench.py --steps 5 --host-steps 8 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
step r04d_gpu_tests.log 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
echo r04d ok

#!/bin/bash
# Round 4: host entry points with 32 MiB chunks, 3 slots, decode D2H one chunk behind: host tests,
# the plain-C caller's rate and copy timeline, the bench leg.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name" 2>&1 || { echo "$name FAILED rc=$?"; tail -30 "gpurun_out/$name"; exit 1; }
  tail -3 "gpurun_out/$name"
}
step r04f_host_tests.log 300 python -u -m pytest tests/test_capi_typed.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread
step r04f_host_bench.txt 120 tests/bin/host_bench 6 2
step r04f_hb_prof.txt 120 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d gpurun_out/r04f_hb -- tests/bin/host_bench 2 1
step r04f_host.json 300 python -u bench.py --steps 5 --host-steps 6 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --per-record 0 --cpu-seconds 0 --ref-reps 0
echo r04f ok

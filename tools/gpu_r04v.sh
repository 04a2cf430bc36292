#!/bin/bash
# Round 4: kernel trace of the N3 legs (reassembly config 2 and the general path on config 3).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 6"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rx -o rx -- python -u bench.py --steps 2 --warmup 1 $Z > gpurun_out/r04v_bench.json 2> gpurun_out/r04v_bench.err || { echo BENCH FAILED; tail gpurun_out/r04v_bench.err; exit 1; }
tail -c 400 gpurun_out/r04v_bench.json
echo r04v ok

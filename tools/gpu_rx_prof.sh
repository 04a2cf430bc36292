#!/bin/bash
# Reassembly legs alone (config 2 and config 3 packetized) under a rocprofv3 kernel trace (repo root, GPU box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0"
rm -rf gpurun_out/prof_rx
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rx -o run -- python3 $R/bench.py --steps 2 --warmup 1 $Z --reassembly-reps ${RX_REPS:-3}) > gpurun_out/prof_rx.log 2>&1 || { tail -20 gpurun_out/prof_rx.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/prof_rx.log').read().split('\n')[-1] or '{}')" 2>/dev/null
grep -h '^{' gpurun_out/prof_rx.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('reassembly','reassembly_config3')})"

#!/bin/bash
# Round 4: fast copies of in-window chunks (tiles with windows of 64 B or more on average): boutique
# levels and the flat leg, off (variant 9) against on.
set -u
mkdir -p gpurun_out
VARIANTS="9 0" bash tools/gpu_r04z.sh > gpurun_out/r04ae_levels.txt 2>&1 || { echo LEVELS FAILED; tail gpurun_out/r04ae_levels.txt; exit 1; }
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0"
for v in 9 0 9 0; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 $Z > gpurun_out/r04ae_flat_$v.json 2>/dev/null || { echo BENCH FAILED; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04ae_flat_$v.json').read().strip().splitlines()[-1]); f=d['flat']
print('variant $v flat', f['encode_ms'], f['decode_ms'], f['matches_oracle_marshal'])"
done
echo r04ae ok

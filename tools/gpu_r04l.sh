#!/bin/bash
# Round 4: flat encode chunks per lane per step (tuning build, SYMHIP_FLAT_VARIANT): 0 default, 4 = 2
# without lists (85 VGPRs), 5 = that and 1 with lists (97 VGPRs); boutique tree and the flat leg.
set -u
mkdir -p gpurun_out
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 5 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0"
for v in 0 4 5 0 4 5; do
timeout -k 10 200 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python tools/boutique_run.py --reps 8 > gpurun_out/r04l_bq_$v.txt 2>&1 || { echo BQ FAILED; tail gpurun_out/r04l_bq_$v.txt; exit 1; }
echo "variant $v: $(tail -1 gpurun_out/r04l_bq_$v.txt)"
done
for v in 0 4; do
timeout -k 10 200 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python -u bench.py --steps 2 --warmup 1 $Z > gpurun_out/r04l_flat_$v.json 2>&1 || { echo FLAT FAILED; tail gpurun_out/r04l_flat_$v.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04l_flat_$v.json').read().strip().splitlines()[-1]); print('flat variant $v', d['flat']['encode_ms'], d['flat']['decode_ms'])"
done
echo r04l ok

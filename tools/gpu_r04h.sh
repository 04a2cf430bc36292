#!/bin/bash
# Round 4: segment gather, chunks per lane per step 4 (default) / 2 / 8 (tuning build): reassembly
# config 2 / 3 and the flat leg.
set -u
mkdir -p gpurun_out
for v in 0 1 2 0; do
timeout -k 10 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_GATHER_VARIANT=$v python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 5 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 6 > gpurun_out/r04h_legs_$v.json 2>&1 || { echo BENCH FAILED; tail gpurun_out/r04h_legs_$v.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04h_legs_$v.json').read().strip().splitlines()[-1])
print('variant $v', [(k, d[k]['reassemble_ms'], d[k]['gbps_algorithmic']) for k in ('reassembly','reassembly_config3')], 'flat dec', d['flat']['decode_ms'])"
done
echo r04h ok

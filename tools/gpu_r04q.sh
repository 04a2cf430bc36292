#!/bin/bash
# Round 4: segment-stationary gather for long segments (tuning build, SYMHIP_GATHER_VARIANT=3):
# reassembly / raw tests under it, then reassembly config 2 / 3 against the default.
set -u
mkdir -p gpurun_out
timeout -k 10 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_GATHER_VARIANT=3 python -u -m pytest tests/test_reassembly.py tests/test_raw_fields.py tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04q_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04q_tests.log)"
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 6"
for v in 0 3 0 3; do
timeout -k 10 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_GATHER_VARIANT=$v python -u bench.py --steps 2 --warmup 1 $Z > gpurun_out/r04q_legs_$v.json 2>&1 || { echo BENCH FAILED; tail gpurun_out/r04q_legs_$v.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04q_legs_$v.json').read().strip().splitlines()[-1])
print('variant $v', [(k, d[k]['reassemble_ms'], d[k]['gbps_algorithmic']) for k in ('reassembly','reassembly_config3')])"
done
echo r04q ok

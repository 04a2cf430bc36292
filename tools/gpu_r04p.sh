#!/bin/bash
# Round 4: flat encode windows per chunk (tuning build, SYMHIP_FLAT_VARIANT 6: 4 windows x 2 chunks,
# 7: 3 x 3): nested / flat tests under each, then boutique and flat legs.
set -u
mkdir -p gpurun_out
for v in 6 7; do
timeout -k 10 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python -u -m pytest tests/test_nested.py tests/test_boutique.py tests/test_flat.py tests/test_wide_schema_entry_points.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p_tests_$v.log 2>&1 || { echo TESTS $v FAILED; tail -30 gpurun_out/r04p_tests_$v.log; exit 1; }
echo "tests $v: $(tail -1 gpurun_out/r04p_tests_$v.log)"
done
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 5 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0 --payload-reps 3"
for v in 0 6 7 0 6 7; do
timeout -k 10 300 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python -u bench.py --steps 5 $Z --boutique-reps 6 > gpurun_out/r04p_legs_$v.json 2>&1 || { echo A FAILED; tail gpurun_out/r04p_legs_$v.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04p_legs_$v.json').read().strip().splitlines()[-1]); b=d['boutique']; p=d['boutique_payloads']
print('variant $v boutique enc', b['encode_ms'], 'payloads enc', p['encode_ms'], 'flat enc', d['flat']['encode_ms'])"
done
echo r04p ok

#!/bin/bash
# Round 4: flat encode: 4 payload windows per chunk for levels of short strings (string_bytes hint).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nested.py tests/test_boutique.py tests/test_flat.py tests/test_wide_schema_entry_points.py tests/test_raw_setters.py tests/test_raw_fields.py tests/test_reassembly.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04o_tests.log; exit 1; }
tail -1 gpurun_out/r04o_tests.log
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 5 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0"
timeout -k 10 300 python -u bench.py --steps 5 $Z --boutique-reps 6 --payload-reps 5 > gpurun_out/r04o_legs.json 2>&1 || { echo A FAILED; tail gpurun_out/r04o_legs.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04o_legs.json').read().strip().splitlines()[-1]); b=d['boutique']; p=d['boutique_payloads']
print('boutique', b['encode_ms'], b['decode_ms'], b['decode_ms_each']); print('payloads', p['encode_ms'], p['decode_ms']); print('flat', d['flat']['encode_ms'], d['flat']['decode_ms'])"
echo r04o ok

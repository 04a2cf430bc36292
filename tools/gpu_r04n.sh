#!/bin/bash
# Round 4: nested tests, then the boutique and payload legs (forks only for levels of 2^16+ records).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nested.py tests/test_boutique.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04n_tests.log; exit 1; }
tail -1 gpurun_out/r04n_tests.log
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0"
timeout -k 10 300 python -u bench.py --steps 5 $Z --boutique-reps 6 --payload-reps 5 > gpurun_out/r04n_legs.json 2>&1 || { echo A FAILED; tail gpurun_out/r04n_legs.json; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04n_legs.json').read().strip().splitlines()[-1]); b=d['boutique']; p=d['boutique_payloads']
print('boutique', b['encode_ms'], b['decode_ms'], b['encode_ms_each'], b['decode_ms_each']); print('payloads', p['encode_ms'], p['decode_ms'])"
echo r04n ok

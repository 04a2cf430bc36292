#!/bin/bash
# Round 4: graph launch/result split (tests), then the boutique and payload legs with graph replays.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_walk.py tests/test_boutique.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04x_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04x_tests.log)"
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --trace-reps 0 --per-record 0 --reassembly-reps 0"
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 $Z > gpurun_out/r04x_legs.json 2> gpurun_out/r04x_legs.err || { echo BENCH FAILED; tail gpurun_out/r04x_legs.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04x_legs.json').read().strip().splitlines()[-1])
b=d['boutique']; p=d['boutique_payloads']
print('boutique eager', b['encode_ms'], b['decode_ms'], 'graph', b['graph'])
print('payloads eager', p['encode_ms'], p['decode_ms'], p['encode_msg_per_s'], p['decode_msg_per_s'], 'graph', p['graph'])"
echo r04x ok

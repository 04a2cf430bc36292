#!/bin/bash
# N5 (flat / nested) parity tests, the boutique timing + kernel trace, and the bench flat leg (repo root, GPU box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_nested.py tests/test_flat.py tests/test_reference_cases.py tests/test_wide_schema_entry_points.py tests/test_raw_setters.py > gpurun_out/n5_tests.log 2>&1 || { tail -30 gpurun_out/n5_tests.log; exit 1; }
tail -1 gpurun_out/n5_tests.log
bash tools/gpu_bq_prof.sh || exit 1
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --mixed-reps 0 --config3-reps 0 --ref-reps 0 --boutique-reps 3 --trace-reps 0 --per-record 0"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 $Z --flat-reps 5 > gpurun_out/n5_bench.json 2> gpurun_out/n5_bench.err || { tail -20 gpurun_out/n5_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/n5_bench.json').read().strip().splitlines()[-1]); print('flat', {k: d['flat'][k] for k in ('encode_ms','decode_ms','encode_gbps','decode_gbps')}); print('boutique', {k: d['boutique'][k] for k in ('encode_ms','decode_ms','round_trip_ok')})"

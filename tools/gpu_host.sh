#!/bin/bash
# Host-entry-point tests and the host-inclusive bench leg (run on the GPU box from the repo root).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_capi_typed.py tests/test_batcher.py > gpurun_out/gh.log 2>&1; rc=$?; tail -2 gpurun_out/gh.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --mixed-reps 0 --config3-reps 0 --trace-reps 0 --host-steps 5 --packetize-reps 0 --crypto-reps 0 --proxy-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --cpu-seconds 0 --per-record 0 --reassembly-reps 0 --ref-reps 0 > gpurun_out/hb.json 2>gpurun_out/hb.err
python -c "import json; print(json.dumps(json.load(open('gpurun_out/hb.json'))['host_inclusive']))"

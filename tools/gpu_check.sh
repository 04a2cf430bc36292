#!/bin/bash
# Standard GPU round trip (run on the GPU box from the repo root): smoke, GPU parity tests,
# one bench line.  Every GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke FAILED rc=$?"; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests FAILED rc=$?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench FAILED rc=$?"; tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json

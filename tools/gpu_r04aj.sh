#!/bin/bash
# Round 4: full GPU suite, smoke, and the default bench line (all legs).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04aj_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04aj_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04aj_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04aj_smoke.log 2>&1 || { echo SMOKE FAILED; tail gpurun_out/r04aj_smoke.log; exit 1; }
tail -1 gpurun_out/r04aj_smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/r04aj_bench.json 2> gpurun_out/r04aj_bench.err || { echo BENCH FAILED; tail gpurun_out/r04aj_bench.err; exit 1; }
tail -c 600 gpurun_out/r04aj_bench.json
echo r04aj ok

#!/bin/bash
# Round 4: full GPU suite and smoke after the graph launch/result split.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04y_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04y_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04y_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04y_smoke.log 2>&1 || { echo SMOKE FAILED; tail gpurun_out/r04y_smoke.log; exit 1; }
tail -1 gpurun_out/r04y_smoke.log
echo r04y ok

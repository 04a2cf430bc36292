#!/bin/bash
# Round 4: full GPU suite + smoke with the in-window fast copies, then the boutique walk timing.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04af_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04af_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04af_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04af_smoke.log 2>&1 || { echo SMOKE FAILED; tail gpurun_out/r04af_smoke.log; exit 1; }
tail -1 gpurun_out/r04af_smoke.log
timeout -k 10 200 python -u tools/graph_walk.py --reps 10 > gpurun_out/r04af_graph.txt 2>&1 || { echo GRAPH FAILED; tail gpurun_out/r04af_graph.txt; exit 1; }
grep -E 'equal|eager' gpurun_out/r04af_graph.txt
echo r04af ok

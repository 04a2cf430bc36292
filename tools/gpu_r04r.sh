#!/bin/bash
# Round 4: graph-captured tree walks (tests) and the parse's one-store fixed fields; boutique eager vs graph.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_walk.py tests/test_nested.py tests/test_boutique.py tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04r_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04r_tests.log)"
timeout -k 10 200 python -u tools/graph_walk.py > gpurun_out/r04r_graph2.txt 2>&1 || { echo GRAPH FAILED; tail gpurun_out/r04r_graph2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04r_graph2.txt
echo r04r ok

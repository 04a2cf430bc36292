#!/bin/bash
# Round 4: in-window fast copies on workgroup tiles too (tuning variant 13): nested/boutique tests
# under it, then boutique levels and walk timing, default against 13.
set -u
mkdir -p gpurun_out
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=13 timeout -k 10 300 python -u -m pytest tests/test_flat.py tests/test_nested.py tests/test_boutique.py tests/test_graph_walk.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ai_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04ai_tests.log; exit 1; }
echo "tests (variant 13): $(tail -1 gpurun_out/r04ai_tests.log)"
VARIANTS="0 13" bash tools/gpu_r04z.sh > gpurun_out/r04ai_levels.txt 2>&1 || { echo LEVELS FAILED; tail gpurun_out/r04ai_levels.txt; exit 1; }
for v in 0 13 0 13; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 200 python -u tools/graph_walk.py --reps 10 > gpurun_out/r04ai_$v.txt 2>&1 || { echo RUN $v FAILED; tail gpurun_out/r04ai_$v.txt; exit 1; }
echo "variant $v: $(grep -E 'eager' gpurun_out/r04ai_$v.txt | tail -1)"
done
echo r04ai ok

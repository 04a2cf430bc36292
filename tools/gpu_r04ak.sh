#!/bin/bash
# Round 4: short flat records staged in LDS (product library: tests), then levels and walk timing,
# staging off (tuning variant 14) against on.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py tests/test_nested.py tests/test_boutique.py tests/test_graph_walk.py tests/test_reference_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ak_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04ak_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04ak_tests.log)"
VARIANTS="14 0" bash tools/gpu_r04z.sh > gpurun_out/r04ak_levels.txt 2>&1 || { echo LEVELS FAILED; tail gpurun_out/r04ak_levels.txt; exit 1; }
for v in 14 0 14 0; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 200 python -u tools/graph_walk.py --reps 10 > gpurun_out/r04ak_$v.txt 2>&1 || { echo RUN $v FAILED; tail gpurun_out/r04ak_$v.txt; exit 1; }
echo "variant $v: $(grep -E 'eager' gpurun_out/r04ak_$v.txt | tail -1)"
done
echo r04ak ok

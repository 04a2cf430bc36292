#!/bin/bash
# Round 4: interior chunks copied window by window in the flat encode: tests, then boutique timing
# (product library) and the tuning build with it off (variant 9) and on.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py tests/test_nested.py tests/test_boutique.py tests/test_graph_walk.py tests/test_reference_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04ac_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r04ac_tests.log)"
for v in 0 10 11 12 0 10; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 200 python -u tools/graph_walk.py --reps 10 > gpurun_out/r04ac_$v.txt 2>&1 || { echo RUN $v FAILED; tail gpurun_out/r04ac_$v.txt; exit 1; }
echo "variant $v: $(grep -E 'eager' gpurun_out/r04ac_$v.txt | tail -1)"
done
echo r04ac ok

#!/bin/bash
# Round 4: the N5 decode walk without a host read per level (sym_flat_decode_ex3 with device counts):
# nested / boutique / flat GPU tests, then the boutique tree timing and its kernel trace.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nested.py tests/test_boutique.py tests/test_flat.py tests/test_wide_schema_entry_points.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r04j_tests.log; exit 1; }
tail -2 gpurun_out/r04j_tests.log
timeout -k 10 200 python tools/boutique_run.py --reps 8 > gpurun_out/r04j_bq.txt 2>&1 || { echo BQ FAILED; tail gpurun_out/r04j_bq.txt; exit 1; }
tail -1 gpurun_out/r04j_bq.txt
echo r04j ok

#!/bin/bash
# Round 4: per-record ring path (16-wave worker, hot slot polling, results built word by word):
# the batcher tests, then records/s against the number of caller threads (plain-C driver).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_batcher.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_batcher_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04g_batcher_tests.log; exit 1; }
tail -2 gpurun_out/r04g_batcher_tests.log
: > gpurun_out/r04g_ring_scaling.txt
for t in 1 4 16 32 64; do
  per=$(( 32000 / t ))
  timeout -k 10 60 tests/bin/batcher_driver $t $per - bench >> gpurun_out/r04g_ring_scaling.txt 2>&1 || { echo FAILED $t; tail gpurun_out/r04g_ring_scaling.txt; exit 1; }
  echo "threads=$t per=$per $(tail -1 gpurun_out/r04g_ring_scaling.txt)"
done
echo r04g ok

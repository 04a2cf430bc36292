#!/bin/bash
# Speculative decode round (GPU box, repo root): its own tests, the whole GPU suite, then A/B of the
# speculative default (0) against exact parsers (710) on config 2 and the mixed batch.  Each GPU step
# has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_speculation.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/spec_tests.log 2>&1 || { echo "spec tests FAILED"; tail -40 gpurun_out/spec_tests.log; exit 1; }
tail -1 gpurun_out/spec_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests FAILED"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/kbench.py --enc "" --dec 0,710 --rounds 16 > gpurun_out/kb_spec2.txt 2>&1 || { echo "kbench FAILED"; cat gpurun_out/kb_spec2.txt; exit 1; }
timeout -k 10 200 python tools/mixed_ab.py --enc "" --dec 0,710 --rounds 16 >> gpurun_out/kb_spec2.txt 2>&1 || { echo "mixed_ab FAILED"; cat gpurun_out/kb_spec2.txt; exit 1; }
cat gpurun_out/kb_spec2.txt

#!/bin/bash
# Mixed encode size scan: parity of the three implementations (tests/test_mixed.py), then the A/B of
# the one-launch pipeline (0), its sizer counts (30: CUs/8, 31: CUs/2, 32: none) and the three-launch
# path (40).  Run on the GPU box from the repo root; stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mixed.py > gpurun_out/mp_tests.log 2>&1 || { tail -30 gpurun_out/mp_tests.log; exit 1; }
tail -2 gpurun_out/mp_tests.log
timeout -k 10 200 python tools/mixed_ab.py --enc 0,34,35,30,31,40 --dec 0 --rounds 12 > gpurun_out/mp_ab.txt 2>&1 || { tail -20 gpurun_out/mp_ab.txt; exit 1; }
tail -7 gpurun_out/mp_ab.txt
timeout -k 10 200 python tools/mixed_ab.py --enc 0,40 --dec 0 --rounds 6 --trace > gpurun_out/mp_ab_t.txt 2>&1 || { tail -20 gpurun_out/mp_ab_t.txt; exit 1; }
tail -3 gpurun_out/mp_ab_t.txt
timeout -k 10 200 python tools/mixed_timeline.py > gpurun_out/mp_tl.txt 2>&1 || { tail -20 gpurun_out/mp_tl.txt; exit 1; }
cat gpurun_out/mp_tl.txt

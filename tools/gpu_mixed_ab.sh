#!/bin/bash
# A/B of the mixed encode tile variants (tools/mixed_ab.py) and the config-2 128-record tile (kbench), then
# the mixed parity tests with the 128-record encode forced.  Run on the GPU box from the repo root.
mkdir -p gpurun_out
timeout -k 10 200 python tools/mixed_ab.py --enc 0,20 --dec 0 --rounds 12 > gpurun_out/mab.txt 2>&1; tail -4 gpurun_out/mab.txt
timeout -k 10 200 python tools/mixed_ab.py --enc 0,20 --dec 0 --rounds 6 --trace > gpurun_out/mab_t.txt 2>&1; tail -4 gpurun_out/mab_t.txt
timeout -k 10 300 python tools/kbench.py --enc 1,21 --dec 0 --rounds 10 > gpurun_out/kb21.txt 2>&1; tail -4 gpurun_out/kb21.txt
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_ENCODE_VARIANT=20 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mixed.py > gpurun_out/g20.log 2>&1; tail -2 gpurun_out/g20.log

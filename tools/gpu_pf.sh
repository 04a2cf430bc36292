#!/bin/bash
# The prefetching persistent encode (tuning variants 50/51): parity with the variant forced through
# the flat and mixed GPU tests, then A/B against the default and the timelines.  Repo root, GPU box.
set -o pipefail
mkdir -p gpurun_out
export SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so
SYMHIP_ENCODE_VARIANT=51 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_mixed.py > gpurun_out/pf_mixed.log 2>&1 || { tail -30 gpurun_out/pf_mixed.log; exit 1; }
tail -1 gpurun_out/pf_mixed.log
SYMHIP_ENCODE_VARIANT=50 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/pf_flat.log 2>&1 || { tail -30 gpurun_out/pf_flat.log; exit 1; }
tail -1 gpurun_out/pf_flat.log
unset SYMHIP_LIBRARY
timeout -k 10 200 python tools/mixed_ab.py --enc 0,51 --dec 0 --rounds 12 > gpurun_out/pf_mab.txt 2>&1 || { tail -20 gpurun_out/pf_mab.txt; exit 1; }
tail -3 gpurun_out/pf_mab.txt
timeout -k 10 300 python tools/kbench.py --config 2 --enc 1,50 --dec 0 --rounds 10 > gpurun_out/pf_kb2.txt 2>&1 || { tail -20 gpurun_out/pf_kb2.txt; exit 1; }
tail -3 gpurun_out/pf_kb2.txt
timeout -k 10 300 python tools/kbench.py --config 3 --enc 1,50 --dec 0 --rounds 10 > gpurun_out/pf_kb3.txt 2>&1 || { tail -20 gpurun_out/pf_kb3.txt; exit 1; }
tail -3 gpurun_out/pf_kb3.txt
timeout -k 10 200 python tools/mixed_timeline.py --variant 52 > gpurun_out/pf_tl.txt 2>&1 || { tail -20 gpurun_out/pf_tl.txt; exit 1; }
cat gpurun_out/pf_tl.txt

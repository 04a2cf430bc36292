#!/bin/bash
# Parity of an experimental decode variant (env SYMHIP_DECODE_VARIANT for the whole test run),
# then an A/B and optional timelines.   bash tools/gpu_pipe.sh VARIANT DEC_LIST [TIMELINE...]
set -u
V=$1; DEC=$2; shift 2
mkdir -p gpurun_out
SYMHIP_DECODE_VARIANT=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/t.log 2>&1 || { echo "gpu tests FAILED (variant $V)"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python tools/kbench.py --enc "" --dec "$DEC" --rounds 8 || { echo "kbench FAILED"; exit 1; }
for v in "$@"; do
    timeout -k 10 100 python tools/fused_timeline.py --variant "$v" || { echo "timeline FAILED"; exit 1; }
done

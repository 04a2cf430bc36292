#!/bin/bash
# GPU A/B round (run on the GPU box from the repo root): parity tests, then decode/encode kernel
# variants timed in one process, then optional fused-decode timelines.  Every GPU step has its own
# time limit; stop at the first failure.
#   bash tools/gpu_ab.sh [DEC] [ENC] [TIMELINE variants...]
#   e.g. bash tools/gpu_ab.sh 300,0,500 "" 410 510
set -u
DEC=${1:-300,0}
ENC=${2:-}
shift 2 2>/dev/null || shift $#
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/t.log 2>&1 || { echo "gpu tests FAILED"; tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python tools/kbench.py --enc "$ENC" --dec "$DEC" --rounds 8 || { echo "kbench FAILED"; exit 1; }
for v in "$@"; do
    timeout -k 10 100 python tools/fused_timeline.py --variant "$v" || { echo "timeline FAILED"; exit 1; }
done

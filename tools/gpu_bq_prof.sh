#!/bin/bash
# N5 boutique tree: timing, then a rocprofv3 kernel trace of tools/boutique_run.py (repo root, GPU box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 200 python tools/boutique_run.py ${BQ_ARGS:-} > gpurun_out/bq.txt 2>&1 || { cat gpurun_out/bq.txt; exit 1; }
cat gpurun_out/bq.txt
rm -rf gpurun_out/prof_bq
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bq -o run -- python3 $R/tools/boutique_run.py --reps 3 ${BQ_ARGS:-}) > gpurun_out/prof_bq.log 2>&1 || { tail -20 gpurun_out/prof_bq.log; exit 1; }
echo profiled

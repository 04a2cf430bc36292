#!/bin/bash
# Round 4: the boutique encode's kernels, full and phase 1 only (tuning variant 1).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/el0 -o run -- python -u tools/enc_levels.py > gpurun_out/r04s_0.txt 2>&1 || { echo RUN0 FAILED; tail gpurun_out/r04s_0.txt; exit 1; }
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/el1 -o run -- python -u tools/enc_levels.py > gpurun_out/r04s_1.txt 2>&1 || { echo RUN1 FAILED; tail gpurun_out/r04s_1.txt; exit 1; }
for d in el0 el1; do echo "== $d"; f=$(find gpurun_out/$d -name '*kernel_stats.csv' | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'enc_tile' in r['Name']: print(r['Calls'], r['AverageNs'], r['Name'][:110])
"; done
echo r04s ok

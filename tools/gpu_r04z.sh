#!/bin/bash
# Round 4: the boutique encode's kernels per level, default vs 4 chunks per lane on list levels (variant 5).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-0 5}; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ez$v -o run -- python -u tools/enc_levels.py > gpurun_out/r04z_$v.txt 2>&1 || { echo RUN $v FAILED; tail gpurun_out/r04z_$v.txt; exit 1; }
echo "== variant $v"
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/ez$v/run_kernel_stats.csv')):
    if 'enc_tile' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:100])
"
done
echo r04z ok

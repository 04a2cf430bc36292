#!/bin/bash
# Round 4: workgroup tiles for every nested level (tuning variant 4) against the default, boutique encode.
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-0 4 0 4}; do
SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v timeout -k 10 200 python -u tools/graph_walk.py --reps 10 > gpurun_out/r04t_$v.txt 2>&1 || { echo RUN $v FAILED; tail gpurun_out/r04t_$v.txt; exit 1; }
echo "variant $v: $(grep -v amdgpu.ids gpurun_out/r04t_$v.txt | grep -E 'equal|eager' | tr '\n' ' ')"
done
echo r04t ok

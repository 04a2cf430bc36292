#!/bin/bash
# Round 4: framed N5 encode: workgroup vs wave tiles for the framed OrderResult level (tuning build),
# then the kernel trace of the boutique tree.
set -u
mkdir -p gpurun_out
for v in 0 3 0 3; do
timeout -k 10 200 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python tools/boutique_run.py --reps 8 > gpurun_out/r04k_bq_$v.txt 2>&1 || { echo BQ FAILED; tail gpurun_out/r04k_bq_$v.txt; exit 1; }
echo "variant $v: $(tail -1 gpurun_out/r04k_bq_$v.txt)"
done
bash tools/gpu_bq_prof.sh
echo r04k ok

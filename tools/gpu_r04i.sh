#!/bin/bash
# Round 4: the GPU suite (gather chunks per lane by segment length, ring worker), then the boutique
# tree with 4 / 8 waves per OrderResult tile (tuning build, SYMHIP_FLAT_VARIANT=2).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r04i_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04i_gpu_tests.log
for v in 0 2 0 2; do
timeout -k 10 200 env SYMHIP_LIBRARY=tools/lib/libsymphony_hip_tuning.so SYMHIP_FLAT_VARIANT=$v python tools/boutique_run.py --reps 8 > gpurun_out/r04i_bq_$v.txt 2>&1 || { echo BQ FAILED; tail gpurun_out/r04i_bq_$v.txt; exit 1; }
echo "variant $v: $(tail -1 gpurun_out/r04i_bq_$v.txt)"
done
echo r04i ok

#!/bin/bash
# Round 4 profiles: kernel trace + FETCH_SIZE + WRITE_SIZE + one SQ/LDS counter pass per workload
# (config 2, config 3, a config-4 shard, the mixed Get/Set batch), then their summaries.
set -u
mkdir -p gpurun_out
WHICH="c2 c3 c4 mixed" PMC_EXTRA="SQ_LDS_IDX_ACTIVE,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY" \
  timeout -k 10 1100 bash tools/gpu_profiles.sh > gpurun_out/r04_prof.log 2>&1 || { echo "profiles FAILED"; tail -20 gpurun_out/r04_prof.log; exit 1; }
tail -3 gpurun_out/r04_prof.log
echo r04prof ok

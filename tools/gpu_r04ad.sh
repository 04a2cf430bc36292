#!/bin/bash
# Round 4: SQ counters of the boutique encode's levels (one --pmc pass, 8 SQ counters).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d gpurun_out/epmc -o pmc -- python -u tools/enc_levels.py 3 > gpurun_out/r04ad.txt 2>&1 || { echo PMC FAILED; tail gpurun_out/r04ad.txt; exit 1; }
ls gpurun_out/epmc
echo r04ad ok

#!/bin/bash
# Round 4, first box: the GPU suite, A/B of the mixed Get/Set decode at 8 copiers per CU (740) against the
# default, the exact parsers and the copiers-only bound, the same variants on config 2 / 3 and the trace
# replay, then rocprof passes (trace, FETCH, WRITE, SQ/LDS counters) of the default mixed kernels.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name" 2>&1 || { echo "$name FAILED rc=$?"; tail -30 "gpurun_out/$name"; exit 1; }
  tail -3 "gpurun_out/$name"
}
step r04a_gpu_tests.log 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step r04a_mixed_ab.txt 300 python tools/mixed_ab.py --enc 0,20,21 --dec 0,740,743,744,745,746,402,742,710,713 --rounds 12
step r04a_kb_c2.txt 300 python tools/kbench.py --enc "" --dec 0,740,744,745 --rounds 8
step r04a_kb_c3.txt 300 python tools/kbench.py --config 3 --enc "" --dec 0,740,744,745 --rounds 6
step r04a_mixed_trace.txt 300 python tools/mixed_ab.py --trace --enc "" --dec 0,740,744,746 --rounds 4
WHICH="mixed" PMC_EXTRA="SQ_LDS_IDX_ACTIVE,SQ_LDS_BANK_CONFLICT,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY" \
  timeout -k 10 600 bash tools/gpu_profiles.sh > gpurun_out/r04a_prof.log 2>&1 || { echo "profiles FAILED"; tail -20 gpurun_out/r04a_prof.log; exit 1; }
tail -3 gpurun_out/r04a_prof.log
echo r04a ok

#!/bin/bash
# On the GPU box: smoke, the default bench line, then rocprofv3 kernel stats + FETCH/WRITE passes of
# the headline (tools/profile.sh).  Every GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
    || { echo "smoke FAILED"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 600 python -u bench.py ${BENCH:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench FAILED"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json
[ "${PROFILE:-1}" = "1" ] || exit 0
OUT=gpurun_out/prof_$TAG bash tools/profile.sh || exit 1
python tools/summarize_profile.py gpurun_out/prof_$TAG gpurun_out/traffic_$TAG.json > /dev/null || exit 1
cp gpurun_out/prof_$TAG/trace/run_kernel_stats.csv gpurun_out/kernel_stats_$TAG.csv
echo "profile ok"

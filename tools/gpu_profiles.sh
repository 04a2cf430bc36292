#!/bin/bash
# One workload per rocprofv3 run (kernel trace, FETCH_SIZE, WRITE_SIZE passes each, plus the counter sets
# in $PMC_EXTRA, one pass each), repo root on the GPU box:
#   c2: the headline (config 2), c3: bench.py --config 3 as the step, c4: bench.py --config 4 (a 2^23-record
#   shard) as the step, mixed: tools/mixed_ab.py on the product library (one-launch encode + pipeline
#   decode), trace: the trace-replay mixed batch (tools/mixed_ab.py --trace), crypto: the bench's segment
#   cipher leg (its encrypt / decrypt kernels; $PMC_CRYPTO adds counter sets for it alone), rx_c3 / rx_c2 /
#   rx_w64: N3 reassembly (tools/rx_hostbound.py) of config 3 and config 2 packetized in send order and of
#   config 3 shuffled within windows of 64.
set -o pipefail
Z="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --config4-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0 --per-record 0"
W=${WHICH:-c2 c3 mixed}
X=${PMC_EXTRA:-}
LIB=$(pwd)/arpc_amd/lib/libsymphony_hip.so
[[ " $W " == *" c2 "* ]] && { OUT=gpurun_out/prof_c2 BENCH_ARGS="--steps 10 --warmup 2 $Z" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" c3 "* ]] && { OUT=gpurun_out/prof_c3 BENCH_ARGS="--config 3 --steps 10 --warmup 2 $Z" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" c4 "* ]] && { OUT=gpurun_out/prof_c4 BENCH_ARGS="--config 4 --steps 5 --warmup 2 $Z" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" mixed "* ]] && { OUT=gpurun_out/prof_mixed PROG=tools/mixed_ab.py SYMHIP_LIBRARY=$LIB BENCH_ARGS="--enc 0 --dec 0 --rounds 5" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" crypto "* ]] && { OUT=gpurun_out/prof_crypto BENCH_ARGS="--steps 2 --warmup 1 ${Z/--crypto-reps 0/--crypto-reps 3}" bash tools/profile.sh $X ${PMC_CRYPTO:-} || exit 1; }
[[ " $W " == *" rx_c3 "* ]] && { OUT=gpurun_out/prof_rx_c3 PROG=tools/rx_hostbound.py BENCH_ARGS="--reps 5 --only config3" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" rx_c2 "* ]] && { OUT=gpurun_out/prof_rx_c2 PROG=tools/rx_hostbound.py BENCH_ARGS="--reps 5 --only config2" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" rx_w64 "* ]] && { OUT=gpurun_out/prof_rx_w64 PROG=tools/rx_hostbound.py BENCH_ARGS="--reps 5 --only reordered" bash tools/profile.sh $X || exit 1; }
[[ " $W " == *" trace "* ]] && { OUT=gpurun_out/prof_trace PROG=tools/mixed_ab.py SYMHIP_LIBRARY=$LIB BENCH_ARGS="--enc 0 --dec 0 --rounds 3 --trace" bash tools/profile.sh $X || exit 1; }
for d in $W; do python3 tools/summarize_profile.py gpurun_out/prof_$d gpurun_out/traffic_$d.json > /dev/null || exit 1; done
echo done

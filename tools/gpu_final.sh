#!/bin/bash
# Round-end evidence on the GPU box (repo root): the whole GPU suite, the default bench line with its
# rocprof kernel stats and HBM traffic (tools/gpu_bench.sh), then config 4 on one GPU and its world-2
# rehearsal (two ranks sharing the card).  Each GPU step has its own time limit; stop at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-final}
LEGS0="--cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --boutique-reps 0 --payload-reps 0 --mixed-reps 0 --config3-reps 0 --config4-reps 0 --trace-reps 0 --per-record 0 --ref-reps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 \
    || { echo "gpu tests FAILED"; tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
TAG=$TAG bash tools/gpu_bench.sh || exit 1
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 3 $LEGS0 > gpurun_out/c4_n1_$TAG.json 2> gpurun_out/c4_n1_$TAG.err \
    || { echo "config 4 FAILED"; tail -5 gpurun_out/c4_n1_$TAG.err; exit 1; }
SYMHIP_BENCH_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --config 4 --steps 10 --warmup 3 $LEGS0 > gpurun_out/c4_w2_$TAG.json 2> gpurun_out/c4_w2_$TAG.err \
    || { echo "world-2 rehearsal FAILED"; tail -5 gpurun_out/c4_w2_$TAG.err; exit 1; }
echo final ok

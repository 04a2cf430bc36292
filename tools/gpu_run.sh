#!/bin/bash
# One GPU call (run on the GPU box from the repo root): the pytest selection in $TESTS (default: the
# whole -m gpu suite), then an optional command in $THEN.  Every GPU step has its own time limit and
# the script stops at the first failure.
set -u
mkdir -p gpurun_out
TAG=${TAG:-run}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 150 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { echo "gpu tests FAILED rc=$?"; tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
if [ -n "${THEN:-}" ]; then
    timeout -k 10 ${THEN_TIMEOUT:-600} bash -c "$THEN" > gpurun_out/then_$TAG.log 2>&1 || { echo "THEN FAILED rc=$?"; tail -40 gpurun_out/then_$TAG.log; exit 1; }
    tail -${THEN_TAIL:-20} gpurun_out/then_$TAG.log
fi
echo run ok

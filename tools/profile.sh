#!/bin/bash
# Profile bench.py kernels with rocprofv3 (run on the GPU box from the repo root).
#   pass 0: --kernel-trace --stats      (per-kernel durations)
#   pass 1: --pmc FETCH_SIZE            (HBM read side; x2 on gfx950, MI355X_MICROARCH.md HBM)
#   pass 2: --pmc WRITE_SIZE            (HBM write side)
#   pass 3+: extra counter sets given as arguments (counters of one set joined by commas), one pass each
# Each pass under its own timeout; stop at the first failure.
set -u
OUT=${OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 0 --host-steps 0 --packetize-reps 0 --proxy-reps 0 --reassembly-reps 0 --crypto-reps 0 --flat-reps 0 --mixed-reps 0 --config3-reps 0 --config4-reps 0 --ref-reps 0 --boutique-reps 0 --payload-reps 0 --trace-reps 0}
PROG=${PROG:-bench.py}   # e.g. PROG=tools/kbench.py BENCH_ARGS="--enc 0 --dec 0,102 --rounds 3"
REPO=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$REPO/$OUT/$name" -o run -- python3 "$REPO/$PROG" $ARGS) \
     > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
i=0
for set in "$@"; do
  i=$((i+1))
  run "pmc$i" --pmc ${set//,/ } || exit 1
done

#!/bin/bash
# Calibrate FETCH_SIZE / WRITE_SIZE per access width (tools/calib_traffic.hip) on the GPU box, from the
# repo root: the TCC counters rocprofv3 offers, then one pass per counter set, each under its own limit.
set -u
REPO=$(pwd)
OUT=${OUT:-gpurun_out/calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 60 rocprofv3 -L) > "$OUT/avail.txt" 2>&1 || (cd /tmp && timeout -k 10 60 rocprofv3 --list-avail) > "$OUT/avail.txt" 2>&1
grep -o "TCC_EA0_[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_REQ[A-Z0-9_]*" "$OUT/avail.txt" | sort -u > "$OUT/tcc_counters.txt" || true
timeout -k 10 60 "$REPO/tools/calib_traffic" 3 > "$OUT/plain.txt" 2>&1 || { echo "calib FAILED"; cat "$OUT/plain.txt"; exit 1; }
i=0
for set in ${SETS:-FETCH_SIZE WRITE_SIZE}; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --output-format csv -d "$REPO/$OUT/p$i" -o run -- "$REPO/tools/calib_traffic" 3) \
      > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($set) FAILED"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ($set) ok"
done
cat "$OUT/plain.txt"
echo calib ok

#!/bin/bash
# Per-kernel durations (rocprofv3 --kernel-trace --stats) of one command, summarized.
#   bash tools/ktrace.sh NAME python3 tools/kbench.py --enc 0 --dec 0 --rounds 5
# Run on the GPU box from the repo root; output under gpurun_out/ktrace/NAME.
set -u
NAME=$1; shift
REPO=$(pwd)
OUT="$REPO/gpurun_out/ktrace/$NAME"
mkdir -p "$OUT"
export TMPDIR=/tmp
PROG=$1; shift
case "$PROG" in python|python3) PROG=python3; SCRIPT="$REPO/$1"; shift ;; *) SCRIPT="" ;; esac
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- $PROG $SCRIPT "$@") > "$OUT/log.txt" 2>&1
rc=$?
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"symhip::(\w+(<[^>]*>)?)", r["Name"])
    if m:
        print("%-40s calls %4s  avg %8.1f us  min %8.1f us" % (m.group(1), r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
exit $rc

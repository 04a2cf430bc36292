#!/bin/bash
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/segtrace -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --enc "" --dec 4 --rounds 2 > $GRAFT_REPO_ROOT/gpurun_out/segtrace.log 2>&1

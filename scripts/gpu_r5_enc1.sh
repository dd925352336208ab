#!/bin/bash
# One-clip encode (C2's bf16x3 graph) under the kernel tracer: per-kernel device time per encode call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
d=gpurun_out/enc1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u scripts/prof_encode.py 1 4 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 30 > gpurun_out/enc1_summary.txt; rm -rf $d
tail -3 $d.log; cat gpurun_out/enc1_summary.txt

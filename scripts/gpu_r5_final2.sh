#!/bin/bash
# End-of-round evidence on the final kernels: GPU suite, bench line, kernel trace of the bench, kernel trace of the
# graph-replayed batch-32 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="tests bench trace" bash scripts/gpu_r5_round.sh || exit 1
d=gpurun_out/tr32
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 AB_M=32 AB_REPS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
  python3 -u scripts/prof_decode_ab.py 64 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 30 > gpurun_out/tr32_summary.txt; rm -rf $d
head -14 gpurun_out/tr32_summary.txt

#!/bin/bash
# Batch 2-6 decode on the two-launch layer (C4's six segments, c5_long): graph-replayed step times, then a kernel trace
# of the batch-6 step (per-launch durations of the attention launch, the FFN launch and the LM head).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 1 2 3 4 5 6; do AB_M=$m timeout -k 10 200 python -u scripts/prof_decode_ab.py 128 - 2>&1 | tee -a gpurun_out/m6_steps.log || exit 1; done
d=gpurun_out/tr6
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 AB_M=6 AB_REPS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
  python3 -u scripts/prof_decode_ab.py 64 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 20 > gpurun_out/tr6_summary.txt; rm -rf $d
cat gpurun_out/tr6_summary.txt

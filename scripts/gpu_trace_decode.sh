#!/bin/bash
# kernel durations of graph-replayed decode steps (batch 32 and batch 1), no eager launch overhead in the trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 32 1; do
  rm -rf gpurun_out/td
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/td -o run -- python3 scripts/prof_batch_decode.py $B 64 > gpurun_out/td_$B.log 2>&1 || { tail -5 gpurun_out/td_$B.log; exit 1; }
  db=$(find gpurun_out/td -name "*results.db" | head -1)
  python3 scripts/prof_summary.py "$db" 16 > gpurun_out/trace_decode_b$B.txt
  cat gpurun_out/trace_decode_b$B.txt | cut -c1-150
done
rm -rf gpurun_out/td

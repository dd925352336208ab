#!/bin/bash
# kernel-trace of encoder-only runs (B=1 and B=32, default GEMM mode) -> per-kernel summaries
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 1 32; do
  R=$([ $B = 1 ] && echo 10 || echo 3)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pe$B -o run -- python3 scripts/prof_encode.py $B $R ${MODE:-bf16x3} > gpurun_out/pe$B.log 2>&1 || { tail -5 gpurun_out/pe$B.log; exit 1; }
  f=gpurun_out/pe$B/run_results.db
  python3 scripts/prof_summary.py "$f" 25 > gpurun_out/pe${B}_summary.txt && cat gpurun_out/pe${B}_summary.txt | cut -c1-200
done

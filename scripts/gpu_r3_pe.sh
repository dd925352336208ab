#!/bin/bash
# kernel classes of the batch-32 and single-clip encodes (bf16x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 32 1; do
  rm -rf gpurun_out/pe
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pe -o run -- python3 scripts/prof_encode.py $B 3 > gpurun_out/pe_$B.log 2>&1 || { tail -5 gpurun_out/pe_$B.log; exit 1; }
  grep "encode batch" gpurun_out/pe_$B.log
  db=$(find gpurun_out/pe -name "*results.db" | head -1)
  python3 scripts/prof_summary.py "$db" 14 > gpurun_out/pe_summary_$B.txt && cut -c1-170 gpurun_out/pe_summary_$B.txt
done
rm -rf gpurun_out/pe

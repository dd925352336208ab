#!/bin/bash
# batch-32 decode step: wall time with graphs, then a kernel trace of eager steps -> per-kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=${B:-32}
timeout -k 10 200 python3 scripts/prof_batch_decode.py $B 64 || exit 1
FUNASR_GRAPHS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb -o run -- python3 scripts/prof_batch_decode.py $B 32 > gpurun_out/pb.log 2>&1 || { tail -5 gpurun_out/pb.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/pb/run_results.db 30 | cut -c1-200

#!/bin/bash
# batched prefill wall time, then a kernel trace -> per-kernel summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/prof_batch_prefill.py ${B:-32} ${T:-204} 3 || exit 1
rm -rf gpurun_out/pp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pp -o run -- python3 scripts/prof_batch_prefill.py ${B:-32} ${T:-204} 1 > gpurun_out/pp.log 2>&1 || { tail -5 gpurun_out/pp.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/pp/run_results.db 14 | cut -c1-150

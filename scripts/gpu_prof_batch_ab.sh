#!/bin/bash
# kernel traces of batch-32 eager decode steps with a knob off / on -> per-kernel summaries
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1; do
  rm -rf gpurun_out/pb$v
  env ${KNOB:-FUNASR_DECODE_NRM}=$v FUNASR_GRAPHS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pb$v -o run -- python3 scripts/prof_batch_decode.py ${B:-32} 32 > gpurun_out/pb$v.log 2>&1 || { tail -5 gpurun_out/pb$v.log; exit 1; }
  echo "== ${KNOB:-FUNASR_DECODE_NRM}=$v"; python3 scripts/prof_summary.py gpurun_out/pb$v/run_results.db 14 | cut -c1-150
done

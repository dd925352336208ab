#!/bin/bash
# Kernel classes of the batch-32 encode (bf16x3) and the one-clip encodes (bf16x3, exact f32, fp16) on this tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "32 bf16x3" "1 bf16x3" "1 f32" "1 fp16"; do
  set -- $cfg
  d=gpurun_out/pe2_$1_$2
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u scripts/prof_encode.py $1 3 $2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 14 > $d.summary.txt; rm -rf $d
  echo "== batch $1 $2"; grep "ms per call" $d.log; head -9 $d.summary.txt
done

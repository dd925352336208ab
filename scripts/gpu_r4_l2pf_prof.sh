#!/bin/bash
# kernel trace of the graph-replayed batch-1 step with and without the L2 prefetch slab
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for s in 0:0 16:50; do
  d=gpurun_out/prof_l2pf_${s/:/_}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 -u scripts/prof_l2pf.py 64 $s > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  tail -1 $d.log
  f=$(find $d -name "*results.db" | head -1)
  python3 scripts/prof_summary.py $f 12 | tee $d.txt
done

#!/bin/bash
# Round 5, second evidence call: the counter passes behind roofline.traffic (gpu_r5_round.sh STEPS=pmc), a kernel
# trace of the graph-replayed batch-32 decode step (per-launch durations of the five layer launches), then the
# graph-profiling bisection of VERDICT r4 item 7 last (it may end in a queue abort; nothing runs after it).
# Raw profiler databases are summarised on the box and deleted (gpurun copies back at most 64 MiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=pmc bash scripts/gpu_r5_round.sh || exit 1
d=gpurun_out/tr32
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 AB_M=32 AB_REPS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $d -o run -- \
  python3 -u scripts/prof_decode_ab.py 64 - > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
python3 scripts/prof_summary.py $(find $d -name "*results.db" | head -1) 30 > gpurun_out/tr32_summary.txt; rm -rf $d
echo "tr32 ok"
bash scripts/gpu_r5_graphprof.sh

#!/bin/bash
# decode step wall time (graph-replayed) over knob settings: batch 1 (C2 path) and batch 32 (C3 path)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in ${CFGS:-"FUNASR_GRAPH_STEPS=1" "FUNASR_GRAPH_STEPS=8" "FUNASR_GRAPH_STEPS=32"}; do
  for B in ${BS:-1 32}; do
    echo -n "$cfg B=$B: "
    env $cfg timeout -k 10 120 python3 scripts/prof_batch_decode.py $B 64 || exit 1
  done
done

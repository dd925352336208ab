#!/bin/bash
# prefetch slab of the batch-1 attention launch: XCD placement (mask 15 = every XCD pulls its neighbour's bytes) and
# the LM head rows in slices over the last FUNASR_L2PF_LM layers; graph-replayed step A/B (scripts/prof_l2pf.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/prof_l2pf.py 256 16:50:7 16:50:15 0:0 16:50:7 16:50:15 2>&1 | tee gpurun_out/l2pf6.log || exit 1
for lm in 0 4 8 2 0 4; do
  FUNASR_L2PF_LM=$lm timeout -k 10 200 python -u scripts/prof_l2pf.py 256 16:50:7 2>&1 | sed "s/^/lm=$lm /" | tee -a gpurun_out/l2pf6.log || exit 1
done

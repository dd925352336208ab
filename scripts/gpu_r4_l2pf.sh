#!/bin/bash
# L2 prefetch slab in the two-launch attention launch (FUNASR_L2PF / _DELAY / _MASK / _MAX_M): graph-replayed step
# A/B at decode batches $L2PF_MS (default 1 2 4 6)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
S="${L2PF_SETTINGS:-0:0 16:50 0:0 16:50}"
for m in ${L2PF_MS:-1 2 4 6}; do
  L2PF_M=$m timeout -k 10 300 python -u scripts/prof_l2pf.py 128 $S 2>&1 | tee -a gpurun_out/l2pf5.log || exit 1
done

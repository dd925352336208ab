#!/bin/bash
# L2 prefetch slab of the batch-1 attention launch (FUNASR_L2PF blocks per kv head : FUNASR_L2PF_DELAY ticks :
# FUNASR_L2PF_MASK byte sets), graph-replayed step A/B (scripts/prof_l2pf.py; profiles/r04_exp_l2pf*.txt). The
# placement (mask bit 8) and LM-head-slice diagnostics of profiles/r04_exp_l2pf_placement.txt were removed after.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/prof_l2pf.py 256 ${L2PF_SETTINGS:-0:0 16:50 0:0 16:50} 2>&1 | tee gpurun_out/l2pf.log

#!/bin/bash
# Batch-1 L2 prefetch slabs of the two-launch layer at small batches (M = 2-6): none / all families / q|k|v+o+FFN / FFN only
# (FUNASR_L2PF_MAX_M=6 with FUNASR_L2PF_MASK), graph-replayed decode steps, interleaved; then the per-batch table (default)
# against no slabs (FUNASR_L2PF=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$TABLE_ONLY" ]; then
for m in 2 3 4 5 6; do
  AB_M=$m AB_REPS=2 timeout -k 10 250 python -u scripts/prof_decode_ab.py 128 FUNASR_L2PF_MAX_M=1 FUNASR_L2PF_MAX_M=6 \
    FUNASR_L2PF_MAX_M=6,FUNASR_L2PF_MASK=3 FUNASR_L2PF_MAX_M=6,FUNASR_L2PF_MASK=1 FUNASR_L2PF_MAX_M=1 FUNASR_L2PF_MAX_M=6 \
    FUNASR_L2PF_MAX_M=6,FUNASR_L2PF_MASK=3 FUNASR_L2PF_MAX_M=6,FUNASR_L2PF_MASK=1 2>&1 | tee -a gpurun_out/pfm_ab2.log || exit 1
done
fi
for m in 1 2 3 4 5 6; do
  AB_M=$m AB_REPS=2 timeout -k 10 250 python -u scripts/prof_decode_ab.py 128 - FUNASR_L2PF_MAX_M=1 - FUNASR_L2PF_MAX_M=1 2>&1 \
    | tee -a gpurun_out/pfm_table.log || exit 1
done

#!/bin/bash
# Persistent LM-head grid (FUNASR_LM_GRID): 4748 32-row tiles over 768 resident blocks leave a 7th round for 140 of
# them; 679 blocks = 7 full rounds, 594 = 8. Graph-replayed decode steps at batch 6 (k_lm_head_s) and 32 (k_lm_head_b).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
AB_M=6 timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_GRID=768 FUNASR_LM_GRID=679 FUNASR_LM_GRID=594 \
  FUNASR_LM_GRID=768 FUNASR_LM_GRID=679 FUNASR_LM_GRID=594 2>&1 | tee gpurun_out/lmgrid.log || exit 1
AB_M=32 timeout -k 10 400 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_GRID=768 FUNASR_LM_GRID=679 FUNASR_LM_GRID=594 \
  FUNASR_LM_GRID=512 FUNASR_LM_GRID=768 FUNASR_LM_GRID=679 FUNASR_LM_GRID=594 FUNASR_LM_GRID=512 2>&1 | tee -a gpurun_out/lmgrid.log || exit 1

#!/bin/bash
# Batched LM head in the swapped-operand form (k_lm_head_b2, FUNASR_LM_HEAD_B2 = 1 / 2 = PF) vs k_lm_head_b (0): graph-
# replayed decode steps at batch 32 and 16 (interleaved; the tokens+logits hash must not change), then the GPU tests
# that run the batched LM head with it on.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 32 16; do
  AB_M=$m timeout -k 10 400 python -u scripts/prof_decode_ab.py 128 FUNASR_LM_HEAD_B2=0 FUNASR_LM_HEAD_B2=1 \
    FUNASR_LM_HEAD_B2=2 FUNASR_LM_HEAD_B2=0 FUNASR_LM_HEAD_B2=1 FUNASR_LM_HEAD_B2=2 2>&1 | tee -a gpurun_out/lmb2_ab.log || exit 1
done
FUNASR_LM_HEAD_B2=1 timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "batch32 or sampler or slot_reuse or c3 or small_batches or mixed_batch" > gpurun_out/lmb2_tests.log 2>&1 \
  || { tail -40 gpurun_out/lmb2_tests.log; exit 1; }
tail -2 gpurun_out/lmb2_tests.log

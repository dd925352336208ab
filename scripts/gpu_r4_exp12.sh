#!/bin/bash
# tokens per fused-FFN block at batches 4-6 (FUNASR_FFN_CT 2 vs 3): decode steps, then the batch-invariance tests with 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for ct in 2 3 2 3; do
  FUNASR_FFN_CT=$ct timeout -k 10 200 python -u scripts/prof_small_batch.py 32 2>&1 | grep -E "batch [3-6]" | sed "s/^/ct=$ct /" || exit 1
done
FUNASR_FFN_CT=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "invariant_width or c4_batch_of_6 or fused" -x -q -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/t_ffnct.log 2>&1 || { tail -30 gpurun_out/t_ffnct.log; exit 1; }
tail -2 gpurun_out/t_ffnct.log

#!/bin/bash
# Batched decode with gate|up + down in one launch (FUNASR_GU_DOWN): bit-identity tests first, then the graph-replayed
# batch-32 step interleaved with the two-launch form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "ffn_one_launch or l2_prefetch_bit_identical or batch32_wide" \
  --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/gudown_tests.log 2>&1 || { tail -30 gpurun_out/gudown_tests.log; exit 1; }
tail -3 gpurun_out/gudown_tests.log
AB_M=32 timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_GU_DOWN=0 FUNASR_GU_DOWN=1 FUNASR_GU_DOWN=0 \
  FUNASR_GU_DOWN=1 2>&1 | tee gpurun_out/gudown_ab.log

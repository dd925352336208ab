#!/bin/bash
# Batched-decode attention with the next pass's K/V pulled into LDS (FUNASR_ATTN_LDSPF): bit-identity tests, the
# attention microbenchmark (graph-replayed, 28 layers, 32 sequences of 201-461 keys), then the batch-32 step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "lds_prefetch or batch32_wide or ffn_one_launch" \
  --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/attnpf_tests.log 2>&1 || { tail -30 gpurun_out/attnpf_tests.log; exit 1; }
tail -3 gpurun_out/attnpf_tests.log
timeout -k 10 120 scripts/ubench/attn_batch 512 2>&1 | tee gpurun_out/attnpf_ubench.log
AB_M=32 timeout -k 10 300 python -u scripts/prof_decode_ab.py 128 FUNASR_ATTN_LDSPF=0 FUNASR_ATTN_LDSPF=1 FUNASR_ATTN_LDSPF=0 \
  FUNASR_ATTN_LDSPF=1 2>&1 | tee gpurun_out/attnpf_ab.log

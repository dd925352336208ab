#!/bin/bash
# fp16 graph (C5) on the bf16x3 kernel family + f16-MFMA attention: parity tests, then encode A/B (old / new kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "fp16" -x -v -m gpu --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/f16_tests.log 2>&1 || { tail -40 gpurun_out/f16_tests.log; exit 1; }
tail -6 gpurun_out/f16_tests.log
for b in 1 32; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    FUNASR_F16_GEMM=$1 FUNASR_F16_ATTN=$2 timeout -k 10 120 python -u scripts/prof_encode.py $b 5 fp16 2>&1 | tail -1 | sed "s/^/gemm=$1 attn=$2 /" || exit 1
  done
  timeout -k 10 120 python -u scripts/prof_encode.py $b 5 bf16x3 2>&1 | tail -1 || exit 1
done
